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
 * Headers mode reads the set from the headers of the redundancy files named
 * on the command line instead, as the reference does
 * (src/redset_reedsolomon_serial.c:355-466): the headers redset_amd writes
 * (header_tree.h; redset's tree content, KVTree's bytes unpinned). Ranks,
 * CHUNK, scheme and CKSUM come from the first readable header, every
 * member's file list from whichever header carries it (its own or a right
 * neighbour's copy); a member is missing when its redundancy file is
 * unreadable or a data file is absent or not exactly its recorded size
 * (redset_lofi_check_mapped, src/redset_lofi.c:219-297). Lost members get
 * their header regenerated from the set and their files' mode and times
 * back (redset_meta_apply, src/redset_util.c:292-380).
 *
 * usage: redset_hip_rebuild rs|xor <ranks> <encoding> <dir>
 *        redset_hip_rebuild headers <redundancy file>...
 *        redset_hip_rebuild print-header <redundancy file>   (header text form)
 * Prints one JSON line with what was rebuilt and the stream statistics.
 */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "header_tree.h"
#include "redset_hip.h"

typedef struct {
  int nfiles;
  char** paths;
  unsigned long long* sizes;
  unsigned long long chunk, header;
  char red[4096];
  htree* hash; /* headers mode: the member's hash (FILES, FILE, DESC) */
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

static int exact_size(const char* path, unsigned long long size) {
  struct stat st;
  return stat(path, &st) == 0 && (unsigned long long) st.st_size == size;
}

static char* key_of(int r, char* buf) {
  snprintf(buf, 16, "%d", r);
  return buf;
}

/* headers mode: the set from the readable headers of `files` (see top) */
static int load_headers(int nfiles, char** files, int* ranks_out, int* rs_out, int* enc_out,
                        member** m_out, htree** group_out) {
  int ranks = 0, rs = 0, enc = 1, any = -1;
  unsigned long long chunk = 0;
  member* m = NULL;
  htree* group = NULL;
  char kb[16];
  /* the caller frees *m_out / *group_out (free_set) on success and failure alike */
  *m_out = NULL;
  *group_out = NULL;
  for (int i = 0; i < nfiles; ++i) {
    int fd = open(files[i], O_RDONLY);
    if (fd < 0) continue;
    unsigned long long hs = 0, me = 0;
    htree* h = ht_read_header(fd, &hs);
    close(fd);
    if (!h || ht_ull(h, "RANK", &me) != 0) {
      fprintf(stderr, "redset_hip_rebuild: %s: no readable header, member treated as lost\n", files[i]);
      ht_free(h);
      continue;
    }
    if (!m) {
      const htree* g = ht_get(h, "GROUP");
      const htree* d = ht_get(ht_get(ht_get(h, "DESC"), key_of((int) me, kb)), "DESC");
      const char* type = ht_val(d, "TYPE");
      unsigned long long n = 0, k = 1;
      int ok = g && ht_ull(g, "RANKS", &n) == 0 && n >= 2 && n <= 4096 && ht_ull(h, "CHUNK", &chunk) == 0 && type &&
               (strcmp(type, "RS") == 0 || strcmp(type, "XOR") == 0);
      if (ok && strcmp(type, "RS") == 0) ok = ht_ull(d, "CKSUM", &k) == 0 && k >= 1 && k < n;
      if (!ok) {
        fprintf(stderr, "redset_hip_rebuild: %s: header lacks the set facts\n", files[i]);
        ht_free(h);
        continue;
      }
      rs = strcmp(type, "RS") == 0;
      ranks = (int) n;
      enc = rs ? (int) k : 1;
      m = calloc((size_t) ranks, sizeof(member));
      group = ht_copy(g);
      *ranks_out = ranks;
      *m_out = m;
      *group_out = group;
    }
    if (me >= (unsigned long long) ranks) {
      ht_free(h);
      continue;
    }
    snprintf(m[me].red, sizeof(m[me].red), "%s", files[i]);
    m[me].header = hs;
    any = (int) me;
    const htree* desc = ht_get(h, "DESC");
    for (int c = 0; desc && c < desc->n; ++c) {
      int r = atoi(desc->kids[c]->key);
      if (r >= 0 && r < ranks && !m[r].hash) m[r].hash = ht_copy(desc->kids[c]);
    }
    ht_free(h);
  }
  if (!m) {
    fprintf(stderr, "redset_hip_rebuild: no readable redundancy-file header\n");
    return -1;
  }
  /* every member's file list, and the file name pattern's prefix */
  const htree* gm = ht_get(group, "RANK");
  unsigned long long gid = 0, groups = 1, wr = 0;
  const htree* d0 = ht_get(m[any].hash, "DESC");
  if (ht_ull(d0, "GROUP", &gid) || ht_ull(d0, "GROUPS", &groups) || ht_ull(gm, key_of(any, kb), &wr)) {
    fprintf(stderr, "redset_hip_rebuild: header lacks the group map\n");
    return -1;
  }
  const char* kind = rs ? "rs" : "xor";
  char tail[512];
  snprintf(tail, sizeof(tail), "%llu.%s.grp_%llu_of_%llu.mem_%d_of_%d.redset", wr, kind, gid + 1, groups, any + 1, ranks);
  size_t la = strlen(m[any].red), lt = strlen(tail);
  if (la < lt || strcmp(m[any].red + la - lt, tail) != 0) {
    fprintf(stderr, "redset_hip_rebuild: %s does not follow the redundancy file pattern\n", m[any].red);
    return -1;
  }
  for (int r = 0; r < ranks; ++r) {
    unsigned long long nf = 0;
    if (!m[r].hash || ht_ull(m[r].hash, "FILES", &nf) != 0 || nf > 1000000) {
      fprintf(stderr, "redset_hip_rebuild: no header carries the file list of member %d\n", r);
      return -1;
    }
    m[r].nfiles = (int) nf;
    m[r].chunk = chunk;
    m[r].paths = calloc(nf + 1, sizeof(char*));
    m[r].sizes = calloc(nf + 1, sizeof(unsigned long long));
    const htree* ft = ht_get(m[r].hash, "FILE");
    for (int k = 0; k < m[r].nfiles; ++k) {
      const htree* e = ht_get(ft, key_of(k, kb));
      if (!e || e->n != 1 || ht_ull(e->kids[0], "SIZE", &m[r].sizes[k]) != 0) {
        fprintf(stderr, "redset_hip_rebuild: member %d file %d: no SIZE\n", r, k);
        return -1;
      }
      m[r].paths[k] = strdup(e->kids[0]->key);
    }
    if (!m[r].red[0]) {
      if (ht_ull(gm, key_of(r, kb), &wr) != 0) {
        fprintf(stderr, "redset_hip_rebuild: group map lacks member %d\n", r);
        return -1;
      }
      snprintf(m[r].red, sizeof(m[r].red), "%.*s%llu.%s.grp_%llu_of_%llu.mem_%d_of_%d.redset", (int) (la - lt),
               m[any].red, wr, kind, gid + 1, groups, r + 1, ranks);
    }
  }
  *rs_out = rs;
  *enc_out = enc;
  return 0;
}

static void free_set(member* m, int ranks, htree* group) {
  for (int r = 0; m && r < ranks; ++r) {
    for (int k = 0; m[r].paths && k < m[r].nfiles; ++k) free(m[r].paths[k]);
    free(m[r].paths);
    free(m[r].sizes);
    ht_free(m[r].hash);
  }
  free(m);
  ht_free(group);
}

/* header of member r's redundancy file: its hash and its left neighbours'
 * under DESC, GROUP, CHUNK, RANK (src/redset_reedsolomon.c:450-496) */
static htree* member_header(const member* m, int ranks, int r, int left, const htree* group) {
  char kb[16];
  htree* h = ht_new("");
  ht_set_ull(h, "RANK", (unsigned long long) r);
  htree* desc = ht_child(h, "DESC");
  ht_put(desc, ht_copy(m[r].hash));
  for (int i = 1; i <= left; ++i) ht_put(desc, ht_copy(m[(r - i + ranks) % ranks].hash));
  ht_put(h, ht_copy(group));
  ht_set_ull(h, "CHUNK", m[r].chunk);
  (void) kb;
  return h;
}

/* redset_meta_apply for a rebuilt data file; returns 0 or -1 */
static int apply_meta(const char* path, const htree* meta) {
  unsigned long long mode, uid, gid, as, an, ms, mn;
  int rc = 0;
  if (ht_ull(meta, "MODE", &mode) == 0 && chmod(path, (mode_t) (mode & 07777)) != 0) rc = -1;
  struct stat st;
  if (ht_ull(meta, "UID", &uid) == 0 && ht_ull(meta, "GID", &gid) == 0 && stat(path, &st) == 0 &&
      (st.st_uid != (uid_t) uid || st.st_gid != (gid_t) gid) && chown(path, (uid_t) uid, (gid_t) gid) != 0)
    rc = -1;
  if (ht_ull(meta, "ATIME_SECS", &as) == 0 && ht_ull(meta, "ATIME_NSECS", &an) == 0 &&
      ht_ull(meta, "MTIME_SECS", &ms) == 0 && ht_ull(meta, "MTIME_NSECS", &mn) == 0) {
    struct timespec ts[2] = {{(time_t) as, (long) an}, {(time_t) ms, (long) mn}};
    if (utimensat(AT_FDCWD, path, ts, 0) != 0) rc = -1;
  }
  if (rc) fprintf(stderr, "redset_hip_rebuild: %s: restoring metadata: %s\n", path, strerror(errno));
  return rc;
}

int main(int argc, char** argv) {
  if (argc == 3 && strcmp(argv[1], "print-header") == 0) {
    int fd = open(argv[2], O_RDONLY);
    unsigned long long hs = 0;
    htree* h = fd < 0 ? NULL : ht_read_header(fd, &hs);
    if (fd >= 0) close(fd);
    if (!h) {
      fprintf(stderr, "redset_hip_rebuild: %s: no readable header\n", argv[2]);
      return 1;
    }
    char* text = ht_render(h);
    fputs(text, stdout);
    free(text);
    ht_free(h);
    return 0;
  }
  const int hdr_mode = argc >= 3 && strcmp(argv[1], "headers") == 0;
  if (!hdr_mode && (argc != 5 || (strcmp(argv[1], "rs") != 0 && strcmp(argv[1], "xor") != 0))) {
    fprintf(stderr, "usage: %s rs|xor <ranks> <encoding> <dir>\n       %s headers <redundancy file>...\n", argv[0],
            argv[0]);
    return 2;
  }
  int rs_scheme = 0, ranks = 0, encoding = 1;
  member* m = NULL;
  htree* group = NULL;
  int* missing = NULL;
  int nmissing = 0;
  int status = 1;
  int* nfiles = NULL;
  int* writable = NULL;
  const char** red = NULL;
  unsigned long long* hdr = NULL;
  const char** paths = NULL;
  unsigned long long* sizes = NULL;
  if (hdr_mode) {
    if (load_headers(argc - 2, argv + 2, &ranks, &rs_scheme, &encoding, &m, &group) != 0) goto out;
    missing = calloc((size_t) ranks, sizeof(int));
    for (int r = 0; r < ranks; ++r) {
      /* no readable header, parity cut short, or a data file absent / resized */
      int gone = m[r].header == 0 || !file_ok(m[r].red, m[r].header + (unsigned long long) encoding * m[r].chunk);
      for (int k = 0; k < m[r].nfiles; ++k) gone |= !exact_size(m[r].paths[k], m[r].sizes[k]);
      if (gone) missing[nmissing++] = r;
    }
  } else {
    rs_scheme = strcmp(argv[1], "rs") == 0;
    ranks = atoi(argv[2]);
    encoding = rs_scheme ? atoi(argv[3]) : 1;
    if (ranks < 2 || encoding < 1 || encoding >= ranks) {
      fprintf(stderr, "redset_hip_rebuild: bad ranks/encoding\n");
      ranks = 0;
      status = 2;
      goto out;
    }
    m = calloc((size_t) ranks, sizeof(member));
    missing = calloc((size_t) ranks, sizeof(int));
    for (int r = 0; r < ranks; ++r) {
      if (read_manifest(argv[4], r, &m[r]) != 0) goto out;
      if (m[r].chunk != m[0].chunk) {
        fprintf(stderr, "redset_hip_rebuild: members disagree on the chunk size\n");
        goto out;
      }
      /* expected redundancy file: header + encoding chunks */
      int gone = !file_ok(m[r].red, m[r].header + (unsigned long long) encoding * m[r].chunk);
      for (int k = 0; k < m[r].nfiles; ++k) gone |= !file_ok(m[r].paths[k], m[r].sizes[k]);
      if (gone) missing[nmissing++] = r;
    }
  }
  const char* scheme_name = rs_scheme ? "rs" : "xor";
  if (nmissing == 0) {
    printf("{\"scheme\": \"%s\", \"ranks\": %d, \"encoding\": %d, \"missing\": [], \"rebuilt_bytes\": 0}\n",
           scheme_name, ranks, encoding);
    status = 0;
    goto out;
  }
  if (nmissing > encoding) {
    fprintf(stderr, "redset_hip_rebuild: %d members missing, the set tolerates %d\n", nmissing, encoding);
    goto out;
  }

  /* regenerate the headers of the missing members' redundancy files */
  for (int i = 0; i < nmissing; ++i) {
    member* x = &m[missing[i]];
    if (hdr_mode) {
      for (int k = 0; k < x->nfiles; ++k) { /* data files come back at their recorded sizes */
        int fd = open(x->paths[k], O_WRONLY | O_CREAT | O_TRUNC, 0600);
        if (fd < 0 || close(fd) != 0) {
          fprintf(stderr, "redset_hip_rebuild: create %s: %s\n", x->paths[k], strerror(errno));
          goto out;
        }
      }
      htree* h = member_header(m, ranks, missing[i], rs_scheme ? encoding : 1, group);
      int fd = open(x->red, O_WRONLY | O_CREAT | O_TRUNC, 0600);
      long long hs = fd < 0 ? -1 : ht_write_header(fd, h);
      ht_free(h);
      if (hs < 0 || close(fd) != 0) {
        fprintf(stderr, "redset_hip_rebuild: write header %s: %s\n", x->red, strerror(errno));
        goto out;
      }
      x->header = (unsigned long long) hs;
      continue;
    }
    char hpath[4096];
    snprintf(hpath, sizeof(hpath), "%s/header_%d.bin", argv[4], missing[i]);
    unsigned char* h = calloc(x->header ? x->header : 1, 1);
    FILE* hf = fopen(hpath, "rb");
    if (hf) {
      size_t got = fread(h, 1, x->header, hf);
      (void) got;
      fclose(hf);
    }
    int fd = open(x->red, O_WRONLY | O_CREAT | O_TRUNC, 0600);
    int bad = fd < 0 || write(fd, h, x->header) != (ssize_t) x->header;
    if (fd >= 0 && close(fd) != 0) bad = 1;
    free(h);
    if (bad) {
      fprintf(stderr, "redset_hip_rebuild: write header %s: %s\n", x->red, strerror(errno));
      goto out;
    }
  }

  /* one fileio over the whole set; the missing members' data files are
   * (re)created at their recorded sizes */
  nfiles = calloc((size_t) ranks, sizeof(int));
  writable = calloc((size_t) ranks, sizeof(int));
  red = calloc((size_t) ranks, sizeof(char*));
  hdr = calloc((size_t) ranks, sizeof(unsigned long long));
  int total = 0;
  for (int r = 0; r < ranks; ++r) total += m[r].nfiles;
  paths = calloc((size_t) total + 1, sizeof(char*));
  sizes = calloc((size_t) total + 1, sizeof(unsigned long long));
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
    goto out;
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
  int meta_ok = 1;
  if (hdr_mode && rc == 0) {
    char kb[16];
    for (int i = 0; i < nmissing; ++i) {
      const member* x = &m[missing[i]];
      const htree* ft = ht_get(x->hash, "FILE");
      for (int k = 0; k < x->nfiles; ++k) {
        const htree* e = ht_get(ft, key_of(k, kb));
        if (apply_meta(x->paths[k], e->kids[0]) != 0) meta_ok = 0;
      }
    }
  }

  printf("{\"scheme\": \"%s\", \"ranks\": %d, \"encoding\": %d, \"missing\": [", scheme_name, ranks, encoding);
  for (int i = 0; i < nmissing; ++i) printf("%s%d", i ? ", " : "", missing[i]);
  printf("], \"ok\": %s, \"metadata_ok\": %s, \"seconds\": %.6f, \"bytes_read\": %llu, \"bytes_written\": %llu, \"GBps\": %.3f}\n",
         rc == 0 ? "true" : "false", meta_ok ? "true" : "false", st.seconds, st.bytes_read, st.bytes_written,
         st.seconds > 0 ? (double) (st.bytes_read + st.bytes_written) / st.seconds / 1e9 : 0.0);
  status = rc == 0 ? 0 : 1;
out:
  free(nfiles);
  free(writable);
  free(red);
  free(hdr);
  free(paths);
  free(sizes);
  free(missing);
  free_set(m, ranks, group);
  return status;
}
