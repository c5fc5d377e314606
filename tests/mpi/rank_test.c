/*
 * rank_test.c -- one MPI rank of a redundancy set, driving the per-rank
 * backends of libredset_hip_mpi.so exactly as redset_apply_rs /
 * redset_recover_rs_rebuild drive a backend (src/redset_reedsolomon.c:
 * 498-545, :826-1006): open the redundancy file, write (or skip) a header,
 * leave fd_chunk positioned after it, call the backend, fsync + close.
 *
 * usage: rank_test <rs|xor> <encode|rebuild> <encoding> <dir> <buf_bytes> [lost ranks...]
 * Rank r reads <dir>/manifest_<r>.txt:
 *   nfiles \n path size \n ... chunk_size \n header_size \n redundancy_path
 * (written by tests/test_gpu_mpi.py). Exit 0 iff every rank succeeded.
 * RANK_TEST_EXCHANGE=host|sharded-mpi|sharded-host|rccl: the rebuild's exchange
 * (redset_hip_rank_set_exchange; default auto). Rank 0 prints the one used.
 * RANK_TEST_DEVICE_PER_RANK=1: rank r on GPU r mod (GPUs).
 * RANK_TEST_FAIL_READ=<rank>: that rank's logical-file reads fail from the
 * second call on (an I/O error in the middle of the collective loop).
 * The HIP runtime is initialised before the timed call (an application that
 * checkpoints already has its GPU context). RANK_TEST_REPEAT=<n>: call the
 * backend n times (fd repositioned after the header each time) and also
 * print the last call's time (warm: code object loaded, caches hot).
 */
#include <execinfo.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "redset_hip.h"
#include "redset_hip_mpi.h"

/* logical-file reads that start failing mid-loop (fault injection) */
static redset_hip_io inner_io;
static int reads_done = 0;
static int failing_read(void* ctx, int rank, int kind, int index, unsigned long long off, size_t len, void* dst) {
  if (reads_done++ >= 1) return -1;
  return inner_io.read(ctx, rank, kind, index, off, len, dst);
}

static int backend_call(int rs_scheme, int encode, int ranks, int encoding, int missing, const int* lost,
                        int need_rebuild, redset_hip_io* io, const char* red, int fd, unsigned long long chunk,
                        size_t buf) {
  if (!rs_scheme)
    return encode ? redset_hip_xor_encode_rank(MPI_COMM_WORLD, io, red, fd, chunk, buf)
                  : redset_hip_xor_decode_rank(MPI_COMM_WORLD, missing ? lost[0] : 0, io, red, fd, chunk, buf);
  redset_hip_rs* rs = NULL;
  int rc = redset_hip_rs_create(ranks, encoding, &rs);
  if (rc == REDSET_SUCCESS)
    rc = encode ? redset_hip_rs_encode_rank(rs, MPI_COMM_WORLD, io, red, fd, chunk, buf)
                : redset_hip_rs_decode_rank(rs, MPI_COMM_WORLD, missing, lost, need_rebuild, io, red, fd, chunk, buf);
  redset_hip_rs_destroy(rs);
  return rc;
}

static int exchange_mode(const char* s) {
  return strcmp(s, "host") == 0 ? REDSET_HIP_EXCHANGE_HOST_MPI
         : strcmp(s, "sharded-mpi") == 0 ? REDSET_HIP_EXCHANGE_SHARDED_MPI
         : strcmp(s, "rccl") == 0 ? REDSET_HIP_EXCHANGE_SHARDED_RCCL
         : strcmp(s, "sharded-host") == 0 ? REDSET_HIP_EXCHANGE_SHARDED_HOST
                                  : REDSET_HIP_EXCHANGE_AUTO;
}

static const char* exchange_name(int m) {
  return m == REDSET_HIP_EXCHANGE_HOST_MPI ? "host"
         : m == REDSET_HIP_EXCHANGE_SHARDED_MPI ? "sharded-mpi"
         : m == REDSET_HIP_EXCHANGE_SHARDED_RCCL ? "rccl"
         : m == REDSET_HIP_EXCHANGE_SHARDED_HOST ? "sharded-host"
                                                 : "none";
}

/* the last call's accounting (redset_hip_rank_last_stats), max and sum over
 * the ranks, as one JSON line from rank 0 (tools/rank_bench.py reads it) */
static void print_stats(int rank, const char* tag) {
  enum { NS = 16 };
  static const char* names[NS] = {"seconds", "read_seconds", "mpi_seconds", "gpu_seconds", "write_seconds",
                                  "read_bytes", "sent_bytes", "recv_bytes", "h2d_bytes", "d2h_bytes", "write_bytes",
                                  "stage_seconds", "copy_seconds", "plan_seconds", "exchange_seconds",
                                  "setup_seconds"};
  redset_hip_rank_stats st;
  memset(&st, 0, sizeof(st));
  (void) redset_hip_rank_last_stats(&st);
  double v[NS] = {st.seconds, st.read_seconds, st.mpi_seconds, st.gpu_seconds, st.write_seconds,
                  (double) st.read_bytes, (double) st.sent_bytes, (double) st.recv_bytes, (double) st.h2d_bytes,
                  (double) st.d2h_bytes, (double) st.write_bytes, st.stage_seconds, st.copy_seconds,
                  st.plan_seconds, st.exchange_seconds, st.setup_seconds};
  double mx[NS], sm[NS];
  MPI_Reduce(v, mx, NS, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  MPI_Reduce(v, sm, NS, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD);
  if (rank != 0) return;
  printf("rank_stats %s {", tag);
  for (int i = 0; i < NS; ++i) printf("%s\"%s\": [%.15g, %.15g]", i ? ", " : "", names[i], mx[i], sm[i]);
  printf("}\n");
}

/* a crash prints where it happened (test driver diagnostics) */
static void on_fatal(int sig) {
  void* bt[64];
  const int n = backtrace(bt, 64);
  fprintf(stderr, "rank_test: signal %d\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IOLBF, 0);
  /* on its own stack, so a stack overflow is reported too */
  static char alt[1 << 16];
  stack_t ss = {.ss_sp = alt, .ss_size = sizeof(alt), .ss_flags = 0};
  sigaltstack(&ss, NULL);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_fatal;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
  MPI_Init(&argc, &argv);
  int rank, ranks;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &ranks);
  /* RANK_TEST_DEVICE_PER_RANK=1: rank r uses GPU r mod (GPUs), the layout of
   * a node with a GPU per member (where AUTO's decode takes RCCL) */
  if (getenv("RANK_TEST_DEVICE_PER_RANK")) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1 || hipSetDevice(rank % ndev) != hipSuccess)
      MPI_Abort(MPI_COMM_WORLD, 7);
  }
  if (argc < 6) {
    if (rank == 0) fprintf(stderr, "usage: %s rs|xor encode|rebuild encoding dir buf [lost...]\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const int rs_scheme = strcmp(argv[1], "rs") == 0;
  const int encode = strcmp(argv[2], "encode") == 0;
  const int encoding = atoi(argv[3]);
  const char* dir = argv[4];
  const size_t buf = (size_t) atoll(argv[5]);
  int missing = argc - 6;
  int lost[256];
  int need_rebuild = 0;
  for (int i = 0; i < missing; ++i) {
    lost[i] = atoi(argv[6 + i]);
    if (lost[i] == rank) need_rebuild = 1;
  }

  char path[4096];
  snprintf(path, sizeof(path), "%s/manifest_%d.txt", dir, rank);
  FILE* mf = fopen(path, "r");
  if (!mf) MPI_Abort(MPI_COMM_WORLD, 3);
  int nfiles = 0;
  if (fscanf(mf, "%d", &nfiles) != 1) MPI_Abort(MPI_COMM_WORLD, 3);
  char** paths = calloc(nfiles + 1, sizeof(char*));
  unsigned long long* sizes = calloc(nfiles + 1, sizeof(unsigned long long));
  for (int i = 0; i < nfiles; ++i) {
    paths[i] = malloc(4096);
    if (fscanf(mf, "%4095s %llu", paths[i], &sizes[i]) != 2) MPI_Abort(MPI_COMM_WORLD, 3);
  }
  unsigned long long chunk = 0, header = 0;
  char red[4096];
  if (fscanf(mf, "%llu %llu %4095s", &chunk, &header, red) != 3) MPI_Abort(MPI_COMM_WORLD, 3);
  fclose(mf);

  /* this rank's logical file (redset_lofi_open, src/redset_lofi.c:306-405) */
  redset_hip_io io;
  redset_hip_fileio* files = NULL;
  int writable = encode ? 0 : need_rebuild;
  int rc = redset_hip_fileio_create(1, &nfiles, (const char* const*) paths, sizes, NULL, NULL, (size_t) chunk,
                                    &writable, &io, &files);
  if (rc != REDSET_SUCCESS) {
    fprintf(stderr, "rank %d: fileio: %s\n", rank, redset_hip_last_error());
    MPI_Abort(MPI_COMM_WORLD, 4);
  }

  const char* fr = getenv("RANK_TEST_FAIL_READ");
  if (fr && atoi(fr) == rank) {
    inner_io = io;
    io.read = failing_read;
  }

  /* redundancy file: header first, backend writes after it */
  int fd;
  if (encode || need_rebuild) {
    fd = open(red, O_RDWR | O_CREAT | O_TRUNC, 0600);
    char* h = malloc(header ? header : 1);
    memset(h, 'H', header);
    if (fd < 0 || write(fd, h, header) != (ssize_t) header) MPI_Abort(MPI_COMM_WORLD, 5);
    free(h);
  } else {
    fd = open(red, O_RDONLY);
    if (fd < 0 || lseek(fd, (off_t) header, SEEK_SET) < 0) MPI_Abort(MPI_COMM_WORLD, 5);
  }

  const char* ex = getenv("RANK_TEST_EXCHANGE");
  if (ex && redset_hip_rank_set_exchange(exchange_mode(ex)) != REDSET_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 6);
  (void) hipFree(NULL); /* runtime init outside the timed region */
  MPI_Barrier(MPI_COMM_WORLD);
  const double t0 = MPI_Wtime();
  rc = backend_call(rs_scheme, encode, ranks, encoding, missing, lost, need_rebuild, &io, red, fd, chunk, buf);
  if (rc != REDSET_SUCCESS) fprintf(stderr, "rank %d: backend failed: %s\n", rank, redset_hip_last_error());
  fsync(fd);
  /* backend call + fsync of what it wrote, slowest rank (the collective's time) */
  double dt = MPI_Wtime() - t0, dmax = 0;
  MPI_Reduce(&dt, &dmax, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
  if (rank == 0) printf("rank_test: %s %s %d ranks chunk %llu buf %zu: %.4f s\n", argv[1], argv[2], ranks, chunk, buf, dmax);
  if (rank == 0)
    printf("rank_test: %s exchange %s\n", encode ? "encode" : "rebuild", exchange_name(redset_hip_rank_last_exchange()));
  print_stats(rank, "first");

  const char* rep = getenv("RANK_TEST_REPEAT");
  const int repeat = rep && atoi(rep) > 1 ? atoi(rep) : 1;
  for (int it = 1; it < repeat; ++it) {
    int ok_i = rc == REDSET_SUCCESS, all_i = 0;
    MPI_Allreduce(&ok_i, &all_i, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD);
    if (!all_i) break;
    if (lseek(fd, (off_t) header, SEEK_SET) < 0) MPI_Abort(MPI_COMM_WORLD, 5);
    MPI_Barrier(MPI_COMM_WORLD);
    const double ti = MPI_Wtime();
    rc = backend_call(rs_scheme, encode, ranks, encoding, missing, lost, need_rebuild, &io, red, fd, chunk, buf);
    if (rc != REDSET_SUCCESS) fprintf(stderr, "rank %d: backend failed: %s\n", rank, redset_hip_last_error());
    fsync(fd);
    double d = MPI_Wtime() - ti, dm = 0;
    MPI_Reduce(&d, &dm, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (rank == 0) printf("rank_test: call %d of %d%s: %.4f s\n", it + 1, repeat, it == repeat - 1 ? " (warm)" : "", dm);
    if (it == repeat - 1) print_stats(rank, "warm");
  }
  close(fd);
  redset_hip_fileio_destroy(files);

  int ok = rc == REDSET_SUCCESS, all = 0;
  MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD); /* redset_alltrue */
  for (int i = 0; i < nfiles; ++i) free(paths[i]);
  free(paths);
  free(sizes);
  MPI_Finalize();
  return all ? 0 : 1;
}
