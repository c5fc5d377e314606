/*
 * adapter_test.c -- runs the reference-signature backend functions of
 * integration/redset_hip_backend.c (src/redset_internal.h:345-381) the way
 * redset's scheme drivers call them, one MPI process per set member:
 * redset_apply_rs / redset_apply_xor (src/redset_reedsolomon.c:498-545,
 * src/redset_xor.c:373-420) write the redundancy file's header, leave the fd
 * after it and call the encode slot with the member's redset_lofi by value;
 * redset_recover_rs_rebuild / redset_recover_xor_rebuild (src/redset_
 * reedsolomon.c:826-1006, src/redset_xor.c:560-671) open the lost members'
 * files for writing, rewrite their headers and call the decode slot.
 *
 * Test infrastructure, built only where the reference's headers exist (this
 * container; tests/adapter/Makefile): redset_base, redset_reedsolomon and
 * redset_lofi are the reference's own types. Three reference symbols the
 * adapter uses are defined here, test-only, as restatements:
 *   redset_lofi_pread / redset_lofi_pwrite -- src/redset_lofi.c:424-451 over
 *     redset_read_pad_n / redset_write_pad_n (:30-173): the files are one
 *     logical file; a read past the recorded sizes is zero-filled, a write
 *     past them is dropped; a short read of a file is a failure;
 *   redset_mpi_buf_size -- src/redset.c:45 (1 MiB default), from argv.
 *
 * usage: adapter_test <rs|xor> <encode|rebuild> <encoding> <dir> <buf_bytes> [lost ranks...]
 * Rank r reads <dir>/manifest_<r>.txt like tests/mpi/rank_test.c:
 *   nfiles \n path size \n ... chunk_size \n header_size \n redundancy_path
 * ADAPTER_TEST_REPEAT=<n>: call the slot n times (fd back after the header
 * each time; the RS codec the adapter caches is reused). Exit 0 iff every
 * rank's calls returned REDSET_SUCCESS.
 */
#include <fcntl.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "redset_hip_backend.h"
#include "redset_hip_mpi.h" /* the exchange selection, test-side only */

int redset_mpi_buf_size = 1024 * 1024;

/* byte range [off, off + n) of the logical file, file by file: fn(file,
 * position in file, count, buffer offset) for the covered pieces; returns
 * how many bytes the files cover */
typedef int (*piece_fn)(int fd, off_t pos, size_t n, char* buf);

static int walk(redset_lofi* rsf, char* buf, size_t count, off_t offset, piece_fn fn, size_t* covered) {
  off_t start = 0;
  size_t done = 0;
  for (int i = 0; i < rsf->numfiles && done < count; ++i) {
    const off_t size = (off_t) rsf->filesizes[i];
    const off_t at = offset + (off_t) done;
    if (at >= start + size) {
      start += size;
      continue;
    }
    const off_t pos = at - start;
    size_t n = (size_t) (size - pos);
    if (n > count - done) n = count - done;
    if (fn(rsf->fds[i], pos, n, buf + done)) return REDSET_FAILURE;
    done += n;
    start += size;
  }
  *covered = done;
  return REDSET_SUCCESS;
}

static int read_piece(int fd, off_t pos, size_t n, char* buf) {
  for (size_t got = 0; got < n;) {
    ssize_t r = pread(fd, buf + got, n - got, pos + (off_t) got);
    if (r <= 0) return 1; /* error, or the file is shorter than recorded */
    got += (size_t) r;
  }
  return 0;
}

static int write_piece(int fd, off_t pos, size_t n, char* buf) {
  for (size_t put = 0; put < n;) {
    ssize_t w = pwrite(fd, buf + put, n - put, pos + (off_t) put);
    if (w <= 0) return 1;
    put += (size_t) w;
  }
  return 0;
}

int redset_lofi_pread(redset_lofi* rsf, void* buf, size_t count, off_t offset) {
  size_t covered = 0;
  if (!rsf || walk(rsf, (char*) buf, count, offset, read_piece, &covered)) return REDSET_FAILURE;
  if (covered < count) memset((char*) buf + covered, 0, count - covered); /* zero padding */
  return REDSET_SUCCESS;
}

int redset_lofi_pwrite(redset_lofi* rsf, void* buf, size_t count, off_t offset) {
  size_t covered = 0; /* bytes past the recorded sizes are dropped */
  if (!rsf || walk(rsf, (char*) buf, count, offset, write_piece, &covered)) return REDSET_FAILURE;
  return REDSET_SUCCESS;
}

static int slot_call(int rs, int encode, const redset_base* d, int missing, int* lost, int need_rebuild,
                     redset_lofi rsf, const char* red, int fd, size_t chunk) {
  if (rs)
    return encode ? redset_reedsolomon_encode_hip(d, rsf, red, fd, chunk)
                  : redset_reedsolomon_decode_hip(d, missing, lost, need_rebuild, rsf, red, fd, chunk);
  return encode ? redset_xor_encode_hip(d, rsf, red, fd, chunk)
                : redset_xor_decode_hip(d, missing ? lost[0] : 0, rsf, red, fd, chunk);
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

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, ranks;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &ranks);
  if (argc < 6) {
    if (rank == 0) fprintf(stderr, "usage: %s rs|xor encode|rebuild encoding dir buf [lost...]\n", argv[0]);
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  const int rs = strcmp(argv[1], "rs") == 0;
  const int encode = strcmp(argv[2], "encode") == 0;
  redset_mpi_buf_size = atoi(argv[5]);
  int missing = argc - 6, lost[256], need_rebuild = 0;
  for (int i = 0; i < missing; ++i) {
    lost[i] = atoi(argv[6 + i]);
    need_rebuild |= lost[i] == rank;
  }

  char path[4096], red[4096];
  snprintf(path, sizeof(path), "%s/manifest_%d.txt", argv[4], rank);
  FILE* mf = fopen(path, "r");
  int nfiles = 0;
  if (!mf || fscanf(mf, "%d", &nfiles) != 1) MPI_Abort(MPI_COMM_WORLD, 3);
  const char** names = calloc(nfiles + 1, sizeof(char*));
  unsigned long* sizes = calloc(nfiles + 1, sizeof(unsigned long));
  int* fds = calloc(nfiles + 1, sizeof(int));
  off_t bytes = 0;
  /* redset_lofi_open (src/redset_lofi.c:306-405): survivors read, a lost
   * member's files are opened for writing */
  const int flags = (!encode && need_rebuild) ? O_WRONLY | O_CREAT | O_TRUNC : O_RDONLY;
  for (int i = 0; i < nfiles; ++i) {
    char* name = malloc(4096);
    if (fscanf(mf, "%4095s %lu", name, &sizes[i]) != 2) MPI_Abort(MPI_COMM_WORLD, 3);
    names[i] = name;
    fds[i] = open(name, flags, 0600);
    if (fds[i] < 0) MPI_Abort(MPI_COMM_WORLD, 4);
    bytes += (off_t) sizes[i];
  }
  unsigned long long chunk = 0, header = 0;
  if (fscanf(mf, "%llu %llu %4095s", &chunk, &header, red) != 3) MPI_Abort(MPI_COMM_WORLD, 3);
  fclose(mf);
  redset_lofi rsf = {nfiles, bytes, fds, names, sizes};

  /* the descriptor the scheme drivers hand the slot (src/redset_internal.h:
   * 39-51, :73-89); the adapter reads comm, ranks and encoding */
  redset_reedsolomon state;
  memset(&state, 0, sizeof(state));
  state.encoding = atoi(argv[3]);
  redset_base d;
  memset(&d, 0, sizeof(d));
  d.enabled = 1;
  d.type = rs ? REDSET_COPY_RS : REDSET_COPY_XOR;
  d.state = &state;
  d.parent_comm = MPI_COMM_WORLD;
  d.comm = MPI_COMM_WORLD;
  d.groups = 1;
  d.ranks = ranks;
  d.rank = rank;

  /* redundancy file: header first, the slot writes after it */
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

  /* ADAPTER_TEST_EXCHANGE=host|sharded-mpi|sharded-host|rccl: the rebuild's exchange
   * (include/redset_hip_mpi.h; default auto, which takes the host path when
   * the members share the box's one GPU) */
  const char* ex = getenv("ADAPTER_TEST_EXCHANGE");
  if (ex && redset_hip_rank_set_exchange(exchange_mode(ex)) != REDSET_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 6);
  const char* rep = getenv("ADAPTER_TEST_REPEAT");
  const int repeat = rep && atoi(rep) > 1 ? atoi(rep) : 1;
  int rc = REDSET_SUCCESS;
  for (int it = 0; it < repeat && rc == REDSET_SUCCESS; ++it) {
    if (it > 0 && lseek(fd, (off_t) header, SEEK_SET) < 0) MPI_Abort(MPI_COMM_WORLD, 5);
    rc = slot_call(rs, encode, &d, missing, lost, need_rebuild, rsf, red, fd, (size_t) chunk);
    if (rc != REDSET_SUCCESS) fprintf(stderr, "rank %d: slot failed\n", rank);
    int ok_i = rc == REDSET_SUCCESS, all_i = 0;
    MPI_Allreduce(&ok_i, &all_i, 1, MPI_INT, MPI_LAND, MPI_COMM_WORLD); /* redset_alltrue */
    if (!all_i) rc = REDSET_FAILURE;
  }
  fsync(fd);
  close(fd);
  for (int i = 0; i < nfiles; ++i) {
    fsync(fds[i]);
    close(fds[i]);
    free((char*) names[i]);
  }
  redset_hip_backend_finalize();
  if (rank == 0) printf("adapter_test: %s %s %d ranks chunk %llu x%d: %s\n", argv[1], argv[2], ranks, chunk, repeat,
                        rc == REDSET_SUCCESS ? "ok" : "FAILED");
  if (rank == 0 && !encode) printf("adapter_test: rebuild exchange %s\n", exchange_name(redset_hip_rank_last_exchange()));
  free(names);
  free(sizes);
  free(fds);
  MPI_Finalize();
  return rc == REDSET_SUCCESS ? 0 : 1;
}
