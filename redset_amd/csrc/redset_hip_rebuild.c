/*
 * redset_hip_rebuild -- single-process offline rebuild of a redundancy set on
 * one GPU: the job of redset_rebuild_rs / redset_rebuild_xor
 * (src/redset_reedsolomon_serial.c:345-693, src/redset_xor_serial.c:277-622),
 * which read every member's redundancy file in one process, find the members
 * whose files are gone, and regenerate their data files and redundancy
 * blocks.
 *
 * The reference learns the set (members, file lists, sizes, chunk size) from
 * the kvtree headers of the redundancy files; KVTree is not available here,
 * so the same facts come from one manifest per member instead
 * (<dir>/manifest_<r>.txt, the format tests/mpi/rank_test.c reads):
 *     nfiles
 *     <path> <size>        (nfiles lines, in logical-file order)
 *     chunk_size
 *     header_size
 *     <redundancy file path>
 * A member is missing when its redundancy file or any of its data files is
 * absent or shorter than recorded (redset_lofi_check_mapped's test,
 * src/redset_lofi.c). More missing members than the scheme tolerates is an
 * error, as in the reference (:507-519). The rebuilt redundancy file gets a
 * header copied from <dir>/header_<r>.bin if present (zeros otherwise).
 *
 * usage: redset_hip_rebuild rs|xor <ranks> <encoding> <dir>
 * Prints one JSON line with what was rebuilt and the stream statistics.
 */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "redset_hip.h"

typedef struct {
  int nfiles;
  char** paths;
  unsigned long long* sizes;
  unsigned long long chunk, header;
  char red[4096];
} member;

static int read_manifest(const char* dir, int r, member* m) {
  char path[4096];
  snprintf(path, sizeof(path), "%s/manifest_%d.txt", dir, r);
  FILE* f = fopen(path, "r");
  if (!f) {
    fprintf(stderr, "redset_hip_rebuild: open %s: %s\n", path, strerror(errno));
    return -1;
  }
  int ok = fscanf(f, "%d", &m->nfiles) == 1 && m->nfiles >= 0;
  m->paths = calloc((size_t) m->nfiles + 1, sizeof(char*));
  m->sizes = calloc((size_t) m->nfiles + 1, sizeof(unsigned long long));
  for (int k = 0; ok && k < m->nfiles; ++k) {
    m->paths[k] = malloc(4096);
    ok = fscanf(f, "%4095s %llu", m->paths[k], &m->sizes[k]) == 2;
  }
  ok = ok && fscanf(f, "%llu %llu %4095s", &m->chunk, &m->header, m->red) == 3;
  fclose(f);
  if (!ok) fprintf(stderr, "redset_hip_rebuild: malformed %s\n", path);
  return ok ? 0 : -1;
}

static int file_ok(const char* path, unsigned long long min_size) {
  struct stat st;
  return stat(path, &st) == 0 && (unsigned long long) st.st_size >= min_size;
}

int main(int argc, char** argv) {
  if (argc != 5 || (strcmp(argv[1], "rs") != 0 && strcmp(argv[1], "xor") != 0)) {
    fprintf(stderr, "usage: %s rs|xor <ranks> <encoding> <dir>\n", argv[0]);
    return 2;
  }
  const int rs_scheme = strcmp(argv[1], "rs") == 0;
  const int ranks = atoi(argv[2]);
  const int encoding = rs_scheme ? atoi(argv[3]) : 1;
  const char* dir = argv[4];
  if (ranks < 2 || encoding < 1 || encoding >= ranks) {
    fprintf(stderr, "redset_hip_rebuild: bad ranks/encoding\n");
    return 2;
  }

  member* m = calloc((size_t) ranks, sizeof(member));
  int* missing = calloc((size_t) ranks, sizeof(int));
  int nmissing = 0;
  for (int r = 0; r < ranks; ++r) {
    if (read_manifest(dir, r, &m[r]) != 0) return 1;
    if (m[r].chunk != m[0].chunk) {
      fprintf(stderr, "redset_hip_rebuild: members disagree on the chunk size\n");
      return 1;
    }
    /* expected redundancy file: header + encoding chunks */
    int gone = !file_ok(m[r].red, m[r].header + (unsigned long long) encoding * m[r].chunk);
    for (int k = 0; k < m[r].nfiles; ++k) gone |= !file_ok(m[r].paths[k], m[r].sizes[k]);
    if (gone) missing[nmissing++] = r;
  }
  if (nmissing == 0) {
    printf("{\"scheme\": \"%s\", \"missing\": [], \"rebuilt_bytes\": 0}\n", argv[1]);
    return 0;
  }
  if (nmissing > encoding) {
    fprintf(stderr, "redset_hip_rebuild: %d members missing, the set tolerates %d\n", nmissing, encoding);
    return 1;
  }

  /* regenerate the headers of the missing members' redundancy files */
  for (int i = 0; i < nmissing; ++i) {
    const member* x = &m[missing[i]];
    char hpath[4096];
    snprintf(hpath, sizeof(hpath), "%s/header_%d.bin", dir, missing[i]);
    unsigned char* h = calloc(x->header ? x->header : 1, 1);
    FILE* hf = fopen(hpath, "rb");
    if (hf) {
      size_t got = fread(h, 1, x->header, hf);
      (void) got;
      fclose(hf);
    }
    int fd = open(x->red, O_WRONLY | O_CREAT | O_TRUNC, 0600);
    if (fd < 0 || write(fd, h, x->header) != (ssize_t) x->header || close(fd) != 0) {
      fprintf(stderr, "redset_hip_rebuild: write header %s: %s\n", x->red, strerror(errno));
      return 1;
    }
    free(h);
  }

  /* one fileio over the whole set; the missing members' data files are
   * (re)created at their recorded sizes */
  int* nfiles = calloc((size_t) ranks, sizeof(int));
  int* writable = calloc((size_t) ranks, sizeof(int));
  const char** red = calloc((size_t) ranks, sizeof(char*));
  unsigned long long* hdr = calloc((size_t) ranks, sizeof(unsigned long long));
  int total = 0;
  for (int r = 0; r < ranks; ++r) total += m[r].nfiles;
  const char** paths = calloc((size_t) total + 1, sizeof(char*));
  unsigned long long* sizes = calloc((size_t) total + 1, sizeof(unsigned long long));
  for (int r = 0, k = 0; r < ranks; ++r) {
    nfiles[r] = m[r].nfiles;
    red[r] = m[r].red;
    hdr[r] = m[r].header;
    for (int j = 0; j < m[r].nfiles; ++j, ++k) {
      paths[k] = m[r].paths[j];
      sizes[k] = m[r].sizes[j];
    }
  }
  for (int i = 0; i < nmissing; ++i) writable[missing[i]] = 1;

  redset_hip_io io;
  redset_hip_fileio* fio = NULL;
  if (redset_hip_fileio_create(ranks, nfiles, paths, sizes, red, hdr, (size_t) m[0].chunk, writable, &io, &fio) != 0) {
    fprintf(stderr, "redset_hip_rebuild: %s\n", redset_hip_last_error());
    return 1;
  }
  redset_hip_stream_stats st;
  memset(&st, 0, sizeof(st));
  int rc;
  if (rs_scheme) {
    redset_hip_rs* rs = NULL;
    rc = redset_hip_rs_create(ranks, encoding, &rs);
    if (rc == 0)
      rc = redset_hip_rs_rebuild_stream(rs, nmissing, missing, (size_t) m[0].chunk, 0, 0, 0, 0, &io, &st);
    redset_hip_rs_destroy(rs);
  } else {
    rc = redset_hip_xor_rebuild_stream(ranks, missing[0], (size_t) m[0].chunk, 0, 0, 0, 0, &io, &st);
  }
  if (rc != 0) fprintf(stderr, "redset_hip_rebuild: %s\n", redset_hip_last_error());
  redset_hip_fileio_destroy(fio); /* fsyncs the written files */

  printf("{\"scheme\": \"%s\", \"missing\": [", argv[1]);
  for (int i = 0; i < nmissing; ++i) printf("%s%d", i ? ", " : "", missing[i]);
  printf("], \"ok\": %s, \"seconds\": %.6f, \"bytes_read\": %llu, \"bytes_written\": %llu, \"GBps\": %.3f}\n",
         rc == 0 ? "true" : "false", st.seconds, st.bytes_read, st.bytes_written,
         st.seconds > 0 ? (double) (st.bytes_read + st.bytes_written) / st.seconds / 1e9 : 0.0);
  return rc == 0 ? 0 : 1;
}
