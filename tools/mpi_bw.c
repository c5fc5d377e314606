/*
 * mpi_bw.c -- host MPI bandwidth of one box in the per-rank backends'
 * message pattern: every rank posts MPI_Isend / MPI_Irecv of `msg` bytes of
 * pinned or pageable host memory to and from every other rank at once, then
 * MPI_Waitall; repeated. Prints per-rank send + receive GB/s (slowest rank),
 * the ceiling the host-MPI exchange of rank_mpi.c is set against
 * (tools/rank_bench.py).
 * usage: mpirun -np P tools/mpi_bw <msg_bytes> [reps]
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int p, r;
  MPI_Comm_size(MPI_COMM_WORLD, &p);
  MPI_Comm_rank(MPI_COMM_WORLD, &r);
  const size_t msg = argc > 1 ? (size_t) atoll(argv[1]) : (1u << 20);
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  char* sbuf = malloc(msg * (size_t) p);
  char* rbuf = malloc(msg * (size_t) p);
  memset(sbuf, r, msg * (size_t) p);
  memset(rbuf, 0, msg * (size_t) p);
  MPI_Request* req = malloc(sizeof(MPI_Request) * 2 * (size_t) p);
  double best = 1e30;
  for (int it = 0; it < reps + 1; ++it) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    int k = 0;
    for (int t = 0; t < p; ++t) {
      if (t == r) continue;
      MPI_Irecv(rbuf + (size_t) t * msg, (int) msg, MPI_BYTE, t, 0, MPI_COMM_WORLD, &req[k++]);
      MPI_Isend(sbuf + (size_t) t * msg, (int) msg, MPI_BYTE, t, 0, MPI_COMM_WORLD, &req[k++]);
    }
    MPI_Waitall(k, req, MPI_STATUSES_IGNORE);
    double dt = MPI_Wtime() - t0, dmax = 0;
    MPI_Allreduce(&dt, &dmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    if (it > 0 && dmax < best) best = dmax;
  }
  if (r == 0)
    printf("{\"ranks\": %d, \"msg_bytes\": %zu, \"per_rank_send_recv_GBps\": %.3f, \"seconds\": %.6f}\n", p, msg,
           2.0 * (double) (p - 1) * (double) msg / best / 1e9, best);
  free(sbuf);
  free(rbuf);
  free(req);
  MPI_Finalize();
  return 0;
}
