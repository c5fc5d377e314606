/*
 * rank_mpi.c -- per-rank MPI backends (include/redset_hip_mpi.h): the
 * reference's backend-slot functions, host code in C, with the arithmetic on
 * the GPU through the codec's C ABI (include/redset_hip.h).
 *
 * Each function keeps the reference's slice loop and MPI exchange pattern and
 * replaces the per-step host multadds with one gf_mac / xor kernel call per
 * slice over all inputs that slice gathered. Host buffers are page-locked so
 * the H2D / D2H copies run at PCIe rate; MPI sees host memory (no GPU-aware
 * MPI needed). The only HIP calls made here are the runtime's C API for
 * pinned memory, copies and one stream; every kernel is reached through
 * redset_hip_gf_combine / redset_hip_xor_combine.
 */
#define _GNU_SOURCE
#include "redset_hip_mpi.h"

#include <errno.h>
#include <limits.h>
#include <pthread.h>
#include <hip/hip_runtime_api.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define DEFAULT_BUF ((size_t) 1 << 20) /* redset_mpi_buf_size default, src/redset.c:45 */
#define MAX_SCRATCH 12
#define MAX_STAGE ((size_t) 96 << 20) /* RS encode: bytes of ring slices staged per window (x2 buffers) */
/* REDSET_HIP_TEST_KNOBS=1: the test twin build (redset_amd/lib_test), whose
 * backends honour the suite's injection and A/B variables; the product reads
 * none */
#ifndef REDSET_HIP_TEST_KNOBS
#define REDSET_HIP_TEST_KNOBS 0
#endif

/* Bytes each step of the RS host-MPI exchange moves per cell: the slice. The
 * reference moves redset_mpi_buf_size B per message (src/redset.c:45,
 * default 1 MiB). Here B is raised to SLICE_MIN: on one box's shared-memory
 * MPI, RS(8+3) over 11 ranks with 64 MiB chunks and a 1 MiB buffer rebuilds
 * in 0.34-0.41 s against 0.61-0.62 s, and encodes (whole ring windows) in
 * 0.78-0.86 s against 1.02-1.07 s; 16 MiB chunks with a 16 MiB buffer (cut
 * to 1 MiB slices) 0.19 against 0.35 s and 0.23-0.26 against 0.31-0.32 s
 * (median of 6 warm calls, two alternating runs each,
 * profiles/r04s9_rank_slice.txt). The XOR backends keep B: larger slices
 * measured slower there. Two caps keep it
 * from growing past what pays: at least SLICES_MIN slices per chunk, so the
 * exchange of slice n still overlaps slice n-1's GPU work and writes (a 16
 * MiB buffer over a 64 MiB chunk leaves 4, too few to pipeline), and at most
 * SLICE_BUDGET of page-locked slice buffers per call (`cells` = the
 * slice-sized host buffers the backend holds); a cut never goes below B or 1
 * MiB, whichever is smaller (small chunks keep the caller's B). Every member
 * derives the same slice from the same arguments. */
#define SLICE_MIN ((size_t) 4 << 20)
#define SLICES_MIN 16
#define SLICE_BUDGET ((size_t) 256 << 20)
static size_t slice_bytes(size_t B, size_t chunk_size, size_t cells) {
#if REDSET_HIP_TEST_KNOBS
  /* test builds: REDSET_HIP_TEST_RANK_SLICE=raw moves B per step (A/B runs) */
  const char* v = getenv("REDSET_HIP_TEST_RANK_SLICE");
  if (v && strcmp(v, "raw") == 0) return B;
#endif
  const size_t mib = (size_t) 1 << 20;
  const size_t least = B < mib ? B : mib; /* a cut never goes below this */
  size_t s = B > SLICE_MIN ? B : SLICE_MIN;
  size_t per = (chunk_size + SLICES_MIN - 1) / SLICES_MIN;
  per = (per + 4095) / 4096 * 4096;
  size_t fit = SLICE_BUDGET / (cells ? cells : 1) / 4096 * 4096;
  if (s > per) s = per;
  if (s > fit) s = fit;
  return s > least ? s : least;
}

static int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
static int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return redset_hip_record_error(buf); /* REDSET_FAILURE */
}

static size_t min_sz(size_t a, size_t b) { return a < b ? a : b; }

/* ---- per-call accounting (redset_hip_rank_last_stats) -------------------- */
/* What a backend call moved and where its host thread waited: the time
 * blocked in logical-file / redundancy-file I/O, in MPI waits, and on the
 * GPU's copies, kernels and (sharded) exchanges. The phases overlap only
 * across the host/device boundary, so their sum is at most the call. */
static __thread redset_hip_rank_stats g_stats;

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double) t.tv_sec + 1e-9 * (double) t.tv_nsec;
}

int redset_hip_rank_last_stats(redset_hip_rank_stats* out) {
  if (!out) return fail("rank_last_stats: null argument");
  *out = g_stats;
  return REDSET_SUCCESS;
}

/* The kernels' hang word (include/redset_hip.h redset_hip_hang_faults) at the
 * start of the calling thread's backend call: a call during which it moved
 * fails, because a kernel wait with no fallback gave up and some launch's
 * outputs are wrong. The failure is this member's alone, after every
 * collective of the call has run; the caller's AND-reduce of the backends'
 * results fails redset_apply / redset_recover as a whole
 * (src/redset_reedsolomon.c:336-341, :1132). */
static __thread unsigned g_hang0;
static __thread int g_hang_read;

static double stats_begin(void) {
  memset(&g_stats, 0, sizeof(g_stats));
  g_hang_read = redset_hip_hang_faults(NULL, &g_hang0, 0) == REDSET_SUCCESS;
  return now_s();
}
static int stats_end(double t0, int rc) {
  unsigned h = 0;
  if (!rc && (!g_hang_read || redset_hip_hang_faults(NULL, &h, 0) != REDSET_SUCCESS))
    rc = fail("cannot read the kernels' hang count");
  else if (!rc && h != g_hang0)
    rc = fail("a kernel wait hit its hang cap during this call (%u): outputs not trusted", h - g_hang0);
  g_stats.seconds = now_s() - t0;
  return rc;
}

/* the logical file (index = segment) */
static int io_read(const redset_hip_io* io, int seg, unsigned long long off, size_t len, void* dst) {
  const double t0 = now_s();
  const int rc = io->read(io->ctx, 0, REDSET_HIP_CELL_DATA, seg, off, len, dst);
  g_stats.read_seconds += now_s() - t0;
  g_stats.read_bytes += len;
  return rc;
}
static int io_write(const redset_hip_io* io, int seg, unsigned long long off, size_t len, const void* src) {
  if (!io->write) return -1;
  const double t0 = now_s();
  const int rc = io->write(io->ctx, 0, REDSET_HIP_CELL_DATA, seg, off, len, src);
  g_stats.write_seconds += now_s() - t0;
  g_stats.write_bytes += len;
  return rc;
}
static void isend(const void* buf, int n, int peer, int tag, MPI_Comm comm, MPI_Request* req) {
  g_stats.sent_bytes += (unsigned long long) n;
  MPI_Isend(buf, n, MPI_BYTE, peer, tag, comm, req);
}
static void irecv(void* buf, int n, int peer, int tag, MPI_Comm comm, MPI_Request* req) {
  g_stats.recv_bytes += (unsigned long long) n;
  MPI_Irecv(buf, n, MPI_BYTE, peer, tag, comm, req);
}
static void mpi_waitall(int k, MPI_Request* req) {
  const double t0 = now_s();
  MPI_Waitall(k, req, MPI_STATUSES_IGNORE);
  g_stats.mpi_seconds += now_s() - t0;
}

/* ---- page-locked host + device scratch and one stream ------------------- */
/*
 * The reference allocates its slice buffers per call (src/redset_reedsolomon.c:
 * 298-302). Here a call's pinned host buffers, device buffers and stream go
 * back to a small process-wide cache when the call succeeds and the next call
 * takes them from there: pinning costs ~0.15 ms per MiB to allocate and free
 * and a stream ~2.7 ms to create and destroy (profiles/r02_alloc_probe.jsonl),
 * which is a large share of a small set's call. REDSET_HIP_SCRATCH_CACHE=0
 * restores allocate-and-free per call; redset_hip_rank_scratch_release()
 * frees the cache (e.g. at redset_finalize). A failed call frees its scratch.
 */
#define POOL_MAX 32
#define POOL_HOST_LIMIT ((size_t) 256 << 20)
#define POOL_DEV_LIMIT ((size_t) 1 << 30)

typedef struct {
  void* p;
  size_t n;
  int dev;    /* device memory (else pinned host) */
  int device; /* current device when it was made: handed out only to calls on it */
} pooled;

static pthread_mutex_t pool_mu = PTHREAD_MUTEX_INITIALIZER;
static pooled pool[POOL_MAX];
static int npool;
static size_t pool_bytes[2]; /* host, device */
static hipStream_t pool_stream;
static int pool_stream_device = -1;

static int current_device(void) {
  int d = -1;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

static int cache_on(void) {
  const char* v = getenv("REDSET_HIP_SCRATCH_CACHE");
  return !v || atoi(v) != 0;
}

typedef struct {
  pooled buf[2 * MAX_SCRATCH];
  int nbuf;
  hipStream_t stream;
  int device;
  int rc;
} scratch;

static void scratch_init(scratch* S) {
  const double t0 = now_s();
  memset(S, 0, sizeof(*S));
  S->device = current_device();
  if (cache_on()) {
    pthread_mutex_lock(&pool_mu);
    if (pool_stream && pool_stream_device == S->device) {
      S->stream = pool_stream;
      pool_stream = NULL;
    }
    pthread_mutex_unlock(&pool_mu);
  }
  if (!S->stream && hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking) != hipSuccess) {
    S->stream = NULL;
    S->rc = fail("hipStreamCreate failed");
  }
  g_stats.setup_seconds += now_s() - t0;
}

/* the smallest cached buffer of the kind that holds n bytes, or a new one */
static uint8_t* scratch_take(scratch* S, size_t n, int dev);
static uint8_t* scratch_get(scratch* S, size_t n, int dev) {
  const double t0 = now_s();
  uint8_t* p = scratch_take(S, n, dev);
  g_stats.setup_seconds += now_s() - t0;
  return p;
}
static uint8_t* scratch_take(scratch* S, size_t n, int dev) {
  void* p = NULL;
  if (S->rc || S->nbuf == 2 * MAX_SCRATCH) return NULL;
  if (n == 0) n = 1;
  size_t have = 0;
  if (cache_on()) {
    pthread_mutex_lock(&pool_mu);
    int best = -1;
    for (int i = 0; i < npool; ++i)
      if (pool[i].dev == dev && pool[i].device == S->device && pool[i].n >= n && (best < 0 || pool[i].n < pool[best].n))
        best = i;
    if (best >= 0) {
      p = pool[best].p;
      have = pool[best].n;
      pool_bytes[dev] -= have;
      pool[best] = pool[--npool];
    }
    pthread_mutex_unlock(&pool_mu);
  }
  if (!p) {
    if ((dev ? hipMalloc(&p, n) : hipHostMalloc(&p, n, hipHostMallocDefault)) != hipSuccess) {
      S->rc = fail("%s(%zu) failed", dev ? "hipMalloc" : "hipHostMalloc", n);
      return NULL;
    }
    have = n;
  }
  S->buf[S->nbuf].p = p;
  S->buf[S->nbuf].n = have;
  S->buf[S->nbuf].dev = dev;
  S->buf[S->nbuf].device = S->device;
  ++S->nbuf;
  return (uint8_t*) p;
}

static uint8_t* scratch_host(scratch* S, size_t n) { return scratch_get(S, n, 0); }
static uint8_t* scratch_dev(scratch* S, size_t n) { return scratch_get(S, n, 1); }

static void release(const pooled* b) {
  if (b->dev) (void) hipFree(b->p);
  else (void) hipHostFree(b->p);
}

/* ok: the call succeeded, its scratch may be cached */
static void scratch_release(scratch* S, int ok);
static void scratch_free(scratch* S, int ok) {
  const double t0 = now_s();
  scratch_release(S, ok);
  g_stats.setup_seconds += now_s() - t0;
}
static void scratch_release(scratch* S, int ok) {
  if (S->stream && hipStreamSynchronize(S->stream) != hipSuccess) ok = 0;
  ok = ok && cache_on();
  pthread_mutex_lock(&pool_mu);
  for (int i = 0; i < S->nbuf; ++i) {
    const pooled* b = &S->buf[i];
    const size_t limit = b->dev ? POOL_DEV_LIMIT : POOL_HOST_LIMIT;
    if (ok && npool < POOL_MAX && pool_bytes[b->dev] + b->n <= limit) {
      pool[npool++] = *b;
      pool_bytes[b->dev] += b->n;
    } else {
      release(b);
    }
  }
  if (S->stream && ok && !pool_stream) {
    pool_stream = S->stream;
    pool_stream_device = S->device;
    S->stream = NULL;
  }
  pthread_mutex_unlock(&pool_mu);
  if (S->stream) (void) hipStreamDestroy(S->stream);
  S->stream = NULL;
  S->nbuf = 0;
}

static void exch_release_all(void);
void redset_hip_rank_scratch_release(void) {
  exch_release_all();
  pthread_mutex_lock(&pool_mu);
  for (int i = 0; i < npool; ++i) release(&pool[i]);
  npool = 0;
  pool_bytes[0] = pool_bytes[1] = 0;
  if (pool_stream) (void) hipStreamDestroy(pool_stream);
  pool_stream = NULL;
  pthread_mutex_unlock(&pool_mu);
  redset_hip_release_scratch(); /* the streaming pipeline's cache too */
}

static int h2d(scratch* S, void* dst, const void* src, size_t n) {
  g_stats.h2d_bytes += n;
  return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, S->stream) == hipSuccess ? 0 : fail("H2D copy failed");
}

static int d2h(scratch* S, void* dst, const void* src, size_t n) {
  g_stats.d2h_bytes += n;
  return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, S->stream) == hipSuccess ? 0 : fail("D2H copy failed");
}


/* ---- file I/O: full pread / pwrite (redset_read_attempt /
 * redset_write_attempt, src/redset_io.c:234-310) --------------------------- */

static int pread_full(int fd, void* buf, size_t n, off_t off) {
  const double t0 = now_s();
  g_stats.read_bytes += n;
  char* p = (char*) buf;
  int rc = 0;
  while (n) {
    ssize_t k = pread(fd, p, n, off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) {
      rc = -1;
      break;
    }
    p += k;
    n -= (size_t) k;
    off += k;
  }
  g_stats.read_seconds += now_s() - t0;
  return rc;
}

static int pwrite_full(int fd, const void* buf, size_t n, off_t off) {
  const double t0 = now_s();
  g_stats.write_bytes += n;
  const char* p = (const char*) buf;
  int rc = 0;
  while (n) {
    ssize_t k = pwrite(fd, p, n, off);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) {
      rc = -1;
      break;
    }
    p += k;
    n -= (size_t) k;
    off += k;
  }
  g_stats.write_seconds += now_s() - t0;
  return rc;
}

/* Every member must enter the exchange loop or none may: a member whose
 * setup failed (scratch allocation, decode map) would otherwise leave its
 * peers blocked in the ring. One MPI_Allreduce(LAND) over the setup result,
 * as redset's callers AND-reduce a backend's rc (redset_alltrue,
 * src/redset_reedsolomon.c:1132). */
static int agree_setup(MPI_Comm comm, int rc) {
  int ok = rc == 0, all = 0;
  if (MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_LAND, comm) != MPI_SUCCESS) return fail("MPI_Allreduce failed");
  if (!all) return rc ? rc : fail("a peer's setup failed");
  return 0;
}

/* Test builds only (-DREDSET_HIP_TEST_KNOBS, the twin library the test suite
 * loads for it): REDSET_HIP_INJECT_DEVICE_FAILURE=<rank> makes that rank's
 * first device step report a failure (tests/mpi/rank_test.c drives it), so
 * the keep-the-collective-going path below is exercised without a broken
 * GPU. The product library reads no such variable. */
static int injected_device_failure(MPI_Comm comm) {
  if (!REDSET_HIP_TEST_KNOBS) return 0;
  static int fired = 0;
  const char* v = getenv("REDSET_HIP_INJECT_DEVICE_FAILURE");
  int r = -1;
  if (!v || fired) return 0;
  MPI_Comm_rank(comm, &r);
  if (atoi(v) != r) return 0;
  fired = 1;
  return fail("injected device failure (REDSET_HIP_INJECT_DEVICE_FAILURE)");
}

static int comm_geometry(MPI_Comm comm, int* ranks, int* rank) {
  if (MPI_Comm_size(comm, ranks) != MPI_SUCCESS || MPI_Comm_rank(comm, rank) != MPI_SUCCESS)
    return fail("MPI_Comm_size/rank failed");
  /* the codec library's struct layouts are the ones this file was built
   * against (every member loads the same library, so every member returns
   * here alike, before any collective) */
  if (redset_hip_abi_version() != REDSET_HIP_ABI_VERSION)
    return fail("libredset_hip has ABI version %d, the backends were built for %d", redset_hip_abi_version(),
                REDSET_HIP_ABI_VERSION);
  return 0;
}

/* header size = where the caller left fd_chunk (src/redset_reedsolomon.c:295, :588) */
static int header_size(int fd_chunk, const char* chunk_file, off_t* header) {
  *header = lseek(fd_chunk, 0, SEEK_CUR);
  if (*header < 0) return fail("lseek(%s) failed", chunk_file ? chunk_file : "chunk file");
  return 0;
}

/* member t's logical-file segment in XOR stripe c (src/redset_xor.c:251-266) */
static int xor_segment(int t, int c) { return c < t ? c : c - 1; }

/* ---- RS encode (replaces redset_reedsolomon_encode, src/redset_reedsolomon.c:280-402) */

/* record / wait an event of the scratch stream; a failure marks the device as gone */
static int ev_record(scratch* S, hipEvent_t ev) {
  return hipEventRecord(ev, S->stream) == hipSuccess ? 0 : fail("hipEventRecord failed");
}
static int ev_wait(hipEvent_t ev) {
  const double t0 = now_s();
  const int ok = hipEventSynchronize(ev) == hipSuccess;
  g_stats.gpu_seconds += now_s() - t0;
  return ok ? 0 : fail("device work failed (hipEventSynchronize)");
}

static int rs_encode_impl(const redset_hip_rs* rs, MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file,
                          int fd_chunk, size_t chunk_size, size_t buf_size) {
  int p, r, rp, e;
  off_t header;
  if (!rs || !lofi || !lofi->read) return fail("rs_encode_rank: null argument");
  if (comm_geometry(comm, &p, &r) || redset_hip_rs_shape(rs, &rp, &e)) return REDSET_FAILURE;
  if (p != rp) return fail("communicator has %d ranks, codec %d", p, rp);
  /* a bad fd on one member is agreed on below, not returned early: its
   * peers would wait for it in the first collective */
  const int hrc = header_size(fd_chunk, chunk_file, &header);
  const int d = p - e;
  const size_t buf = buf_size ? buf_size : DEFAULT_BUF;
  if (buf > (size_t) INT_MAX) return fail("buf_size %zu exceeds an MPI count", buf); /* same on every rank */
  /* the call's page-locked buffers, in slices of B: the window's own
   * segments (G), two receive windows (2*G*e) and two parity buffers (2*e).
   * The slice is cut so that even one-step windows (G = 1) fit SLICE_BUDGET:
   * (4e + 1) slices */
  const size_t B = slice_bytes(buf, chunk_size, (size_t) 4 * e + 1);
  /* ring steps staged per window: the d*e slices of a slice's whole ring
   * would need d*e*B of pinned and device memory (O(p*e)); windows of G steps
   * bound each receive window to MAX_STAGE, and all of the call's slice
   * buffers together to SLICE_BUDGET -- (2e + 1)*G + 2e slices (the
   * reference's own scratch is e+e+1 slices). RS(8+3) at the default 4 MiB
   * slice: G = 8 = d, 248 MiB pinned (and as much device memory) */
  size_t stage = MAX_STAGE;
#if REDSET_HIP_TEST_KNOBS
  /* test builds: the staging bound, for A/B runs (tools/rank_bench.py) */
  if (getenv("REDSET_HIP_TEST_RANK_STAGE_MIB")) stage = (size_t) atoll(getenv("REDSET_HIP_TEST_RANK_STAGE_MIB")) << 20;
#endif
  int G = (int) (stage / ((size_t) e * B));
  const size_t fit = SLICE_BUDGET > (size_t) 2 * e * B ? (SLICE_BUDGET - (size_t) 2 * e * B) / ((size_t) (2 * e + 1) * B) : 1;
  if ((size_t) G > fit) G = (int) fit;
  if (G < 1) G = 1;
  if (G > d) G = d;

  unsigned char* mat = malloc((size_t) (p + e) * p);
  unsigned char* coef = malloc((size_t) e * d);       /* [slot i][ring step s] */
  const unsigned char** ins = malloc(sizeof(*ins) * (size_t) G);
  MPI_Request* req = malloc(sizeof(*req) * 2 * (size_t) e * (size_t) G);
  scratch S;
  scratch_init(&S);
  /* two of everything the GPU touches: window w+1's exchange fills one
   * receive buffer while the GPU copies and combines window w from the other,
   * and slice n's parity is written while slice n+1 is exchanged */
  uint8_t* h_send = scratch_host(&S, (size_t) G * B); /* the window's own segments, one per step */
  uint8_t* h_recv[2] = {scratch_host(&S, (size_t) G * e * B), scratch_host(&S, (size_t) G * e * B)};
  uint8_t* h_par[2] = {scratch_host(&S, (size_t) e * B), scratch_host(&S, (size_t) e * B)};
  uint8_t* d_recv[2] = {scratch_dev(&S, (size_t) G * e * B), scratch_dev(&S, (size_t) G * e * B)};
  uint8_t* d_par[2] = {scratch_dev(&S, (size_t) e * B), scratch_dev(&S, (size_t) e * B)};
  hipEvent_t ev_recv[2] = {NULL, NULL}, ev_par[2] = {NULL, NULL};
  int rc = S.rc ? S.rc : hrc;
  for (int k = 0; k < 2 && !rc; ++k)
    if (hipEventCreateWithFlags(&ev_recv[k], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_par[k], hipEventDisableTiming) != hipSuccess)
      rc = fail("hipEventCreate failed");
  if (!rc && (!mat || !coef || !ins || !req)) rc = fail("out of host memory");
  if (!rc) rc = redset_hip_rs_matrix(rs, mat);
  if ((rc = agree_setup(comm, rc))) goto out;

  /* slot i's coefficients over the d slices it receives, in ring-step order:
   * at step s (chunk_step p-1-s) slot i receives from r + (p - chunk_step + i) */
  for (int i = 0; i < e; ++i)
    for (int s = 0; s < d; ++s) {
      const int step = p - 1 - s;
      const int sender = (r + (p - step + i)) % p;
      coef[(size_t) i * d + s] = mat[(size_t) (p + i) * p + sender];
    }

  /* after a device failure the loop keeps every MPI call (peers must not
   * hang, src/redset_reedsolomon.c:338-342) but skips GPU work and writes */
  int dev_failed = 0;
  long wcount = 0;                  /* windows so far (receive buffer = wcount & 1) */
  int have_prev = 0, prev_sp = 0;   /* a slice whose parity is still to be written */
  size_t prev_nread = 0, prev_count = 0;
  size_t n = 0;
  for (size_t nread = 0; nread < chunk_size; nread += B, ++n) {
    const size_t count = min_sz(B, chunk_size - nread);
    const int sp = (int) (n & 1);
    for (int s0 = 0; s0 < d; s0 += G) {
      const int gs = d - s0 < G ? d - s0 : G;
      const int bb = (int) (wcount & 1);
      /* the copy that read this receive buffer two windows ago is done */
      if (!dev_failed && wcount >= 2 && ev_wait(ev_recv[bb])) {
        rc = REDSET_FAILURE;
        dev_failed = 1;
      }
      /* the window's steps (chunk_step = p-1 .. e, src/redset_reedsolomon.c:
       * 329-377) exchanged together: at step s this rank sends its segment of
       * stripe r + chunk_step to the e parity holders of that stripe and
       * receives, for each of its own parity slots, one segment of stripe
       * r - ... (the same pairs as the reference's ring, which forwards
       * partial sums instead). Tag = step within the window, so a pair that
       * meets at several steps matches them one to one. */
      for (int s = s0; s < s0 + gs; ++s) {
        const int chunk_id = (r + p - 1 - s) % p;
        const int seg = redset_hip_rs_get_data_id(p, e, r, chunk_id);
        uint8_t* mine = h_send + (size_t) (s - s0) * B;
        if (io_read(lofi, seg, nread, count, mine) != 0) {
          rc = fail("lofi read failed");
          memset(mine, 0, count);
        }
      }
      int k = 0;
      for (int s = s0; s < s0 + gs; ++s) {
        const int step = p - 1 - s;
        for (int i = 0; i < e; ++i) {
          const int dist = p - step + i;
          irecv(h_recv[bb] + ((size_t) (s - s0) * e + i) * B, (int) count, (r + dist) % p, s - s0,
                    comm, &req[k++]);
          isend(h_send + (size_t) (s - s0) * B, (int) count, (r - dist + p) % p, s - s0, comm,
                    &req[k++]);
        }
      }
      mpi_waitall(k, req);
      ++wcount;
      if (dev_failed) continue;
      /* the window's gs*e slices: one H2D, one kernel per slot accumulating
       * over the window's steps -- enqueued, not waited for */
      int grc = injected_device_failure(comm);
      if (!grc) grc = h2d(&S, d_recv[bb], h_recv[bb], (size_t) gs * e * B);
      if (!grc) grc = ev_record(&S, ev_recv[bb]);
      for (int i = 0; i < e && !grc; ++i) {
        for (int s = 0; s < gs; ++s) ins[s] = d_recv[bb] + ((size_t) s * e + i) * B;
        unsigned char* o = d_par[sp] + (size_t) i * B;
        grc = redset_hip_gf_combine(ins, gs, &o, 1, coef + (size_t) i * d + s0, count, s0 > 0, S.stream);
      }
      if (grc) {
        rc = grc;
        dev_failed = 1;
      }
    }
    if (!dev_failed) {
      int grc = d2h(&S, h_par[sp], d_par[sp], (size_t) e * B);
      if (!grc) grc = ev_record(&S, ev_par[sp]);
      if (grc) {
        rc = grc;
        dev_failed = 1;
      }
    }
    /* the previous slice's parity, while this slice's GPU work runs (:379-388) */
    if (have_prev && !dev_failed) {
      if (ev_wait(ev_par[prev_sp])) {
        rc = REDSET_FAILURE;
        dev_failed = 1;
      } else {
        for (int i = 0; i < e; ++i) {
          const off_t off = header + (off_t) i * (off_t) chunk_size + (off_t) prev_nread;
          if (pwrite_full(fd_chunk, h_par[prev_sp] + (size_t) i * B, prev_count, off) != 0)
            rc = fail("write %s failed", chunk_file);
        }
      }
    }
    have_prev = 1;
    prev_sp = sp;
    prev_nread = nread;
    prev_count = count;
  }
  if (have_prev && !dev_failed) {
    if (ev_wait(ev_par[prev_sp])) {
      rc = REDSET_FAILURE;
    } else {
      for (int i = 0; i < e; ++i) {
        const off_t off = header + (off_t) i * (off_t) chunk_size + (off_t) prev_nread;
        if (pwrite_full(fd_chunk, h_par[prev_sp] + (size_t) i * B, prev_count, off) != 0)
          rc = fail("write %s failed", chunk_file);
      }
    }
  }
out:
  scratch_free(&S, rc == 0);
  for (int k = 0; k < 2; ++k) {
    if (ev_recv[k]) (void) hipEventDestroy(ev_recv[k]);
    if (ev_par[k]) (void) hipEventDestroy(ev_par[k]);
  }
  free(mat);
  free(coef);
  free(ins);
  free(req);
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}


/* ---- RS decode (replaces redset_reedsolomon_decode, src/redset_reedsolomon.c:570-785) */

#define TAG_RING 0
#define TAG_GATHER 1

/* the host-MPI exchange of the RS decode (members sharing GPUs, several
 * nodes, or no RCCL): the reference's message pattern through pinned host
 * memory */
static int rs_decode_host(const redset_hip_rs* rs, MPI_Comm comm, int p, int r, int e, int missing,
                          const int* rebuild_ranks, int need_rebuild, const redset_hip_io* lofi, const char* chunk_file,
                          int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t B) {

  unsigned char* D = malloc((size_t) missing * p); /* decode map of stripe r: missing x p */
  unsigned char* coef = malloc((size_t) missing * p);
  int* cols = malloc(sizeof(int) * (size_t) p);
  const unsigned char** ins = malloc(sizeof(*ins) * (size_t) p);
  unsigned char** outs = malloc(sizeof(*outs) * (size_t) missing);
  MPI_Request* req = malloc(sizeof(*req) * (size_t) (2 * p + missing + 2));
  scratch S;
  scratch_init(&S);
  /* two sets of slice buffers: slice n's ring exchange and GPU solve overlap
   * slice n-1's gather to the erased members and its writes */
  uint8_t* h_send = scratch_host(&S, (size_t) p * B); /* my cell of stripe c, for solver c */
  uint8_t* h_cells[2] = {scratch_host(&S, (size_t) p * B), scratch_host(&S, (size_t) p * B)};
  uint8_t* h_out[2] = {scratch_host(&S, (size_t) missing * B), scratch_host(&S, (size_t) missing * B)};
  uint8_t* h_gather = scratch_host(&S, (size_t) p * B); /* rebuilt cells from every solver */
  unsigned char* send_to = calloc((size_t) p, 1);    /* solver c's decode reads my cell of stripe c */
  unsigned char* Dc = malloc((size_t) missing * p);
  uint8_t* d_cells[2] = {scratch_dev(&S, (size_t) p * B), scratch_dev(&S, (size_t) p * B)};
  uint8_t* d_out[2] = {scratch_dev(&S, (size_t) missing * B), scratch_dev(&S, (size_t) missing * B)};
  hipEvent_t ev_done[2] = {NULL, NULL};
  int rc = S.rc ? S.rc : hrc;
  for (int k = 0; k < 2 && !rc; ++k)
    if (hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming) != hipSuccess) rc = fail("hipEventCreate failed");
  if (!rc && (!D || !coef || !cols || !ins || !outs || !req || !send_to || !Dc)) rc = fail("out of host memory");
  /* member r solves stripe r (decode_chunk_id = rank, :607-611): one linear
   * map equal to redset_rs_reduce_decode + redset_rs_gaussian_solve */
  if (!rc) rc = redset_hip_rs_decode_matrix(rs, missing, rebuild_ranks, r, D);
  /* every member derives every stripe's map the same way, so it knows which
   * solvers read its cells: the erased members' cells, and survivors' cells a
   * map does not use, are never sent (the reference's ring forwards them all) */
  for (int c = 0; c < p && !rc; ++c) {
    rc = redset_hip_rs_decode_matrix(rs, missing, rebuild_ranks, c, Dc);
    for (int i = 0; i < missing && !rc; ++i) send_to[c] |= Dc[(size_t) i * p + r] != 0;
  }
  if ((rc = agree_setup(comm, rc))) goto out;
  int ncols = 0;
  for (int s = 0; s < p; ++s) {
    int used = 0;
    for (int i = 0; i < missing; ++i) used |= D[(size_t) i * p + s] != 0;
    if (used) cols[ncols++] = s;
  }
  for (int i = 0; i < missing; ++i)
    for (int k = 0; k < ncols; ++k) coef[(size_t) i * ncols + k] = D[(size_t) i * p + cols[k]];

  /* after a device failure every MPI call of the loop still runs (peers must
   * not hang, src/redset_reedsolomon.c:666-681 keep going on read errors);
   * this member then sends zeros as its solved cells and fails the call */
  int dev_failed = 0;
  int have_prev = 0, prev_b = 0;
  size_t prev_nread = 0, prev_count = 0;
  size_t n = 0;
  for (size_t nread = 0;; nread += B, ++n) {
    const int more = nread < chunk_size;
    const size_t count = more ? min_sz(B, chunk_size - nread) : 0;
    const int bb = (int) (n & 1);
    if (more) {
      /* the slice's cells straight to their solvers, all at once (the
       * reference passes them round a ring, one step at a time, :646-703):
       * my cell of stripe c to member c, stripe r's used cells to me */
      for (int c = 0; c < p; ++c) {
        if (!send_to[c]) continue;
        uint8_t* mine = h_send + (size_t) c * B;
        const int enc = redset_hip_rs_get_encoding_id(p, e, r, c);
        int bad;
        if (enc < p) {
          const int seg = redset_hip_rs_get_data_id(p, e, r, c);
          bad = io_read(lofi, seg, nread, count, mine) != 0;
          if (bad) rc = fail("lofi read failed");
        } else {
          const off_t off = header + (off_t) (enc - p) * (off_t) chunk_size + (off_t) nread;
          bad = pread_full(fd_chunk, mine, count, off) != 0;
          if (bad) rc = fail("read %s failed", chunk_file);
        }
        if (bad) memset(mine, 0, count);
      }
      /* stripe r's used cells land packed, input j at j * B, so one copy of
       * ncols cells moves them to the GPU */
      int k = 0;
      for (int j = 0; j < ncols; ++j) {
        if (cols[j] != r) irecv(h_cells[bb] + (size_t) j * B, (int) count, cols[j], TAG_RING, comm, &req[k++]);
        else memcpy(h_cells[bb] + (size_t) j * B, h_send + (size_t) r * B, count);
      }
      for (int c = 0; c < p; ++c)
        if (c != r && send_to[c])
          isend(h_send + (size_t) c * B, (int) count, c, TAG_RING, comm, &req[k++]);
      mpi_waitall(k, req);
      /* enqueue this slice's solve; it runs while the previous slice is gathered */
      if (!dev_failed) {
        for (int k = 0; k < ncols; ++k) ins[k] = d_cells[bb] + (size_t) k * B;
        for (int i = 0; i < missing; ++i) outs[i] = d_out[bb] + (size_t) i * B;
        int grc = injected_device_failure(comm);
        if (!grc && ncols > 0) grc = h2d(&S, d_cells[bb], h_cells[bb], (size_t) ncols * B);
        if (!grc && ncols > 0) grc = redset_hip_gf_combine(ins, ncols, outs, missing, coef, count, 0, S.stream);
        if (!grc) grc = d2h(&S, h_out[bb], d_out[bb], (size_t) missing * B);
        if (!grc) grc = ev_record(&S, ev_done[bb]);
        if (grc) {
          rc = grc;
          dev_failed = 1;
        }
      }
    }
    if (have_prev) {
      /* previous slice: its solved cells to the erased members, :713-733 */
      if (!dev_failed && ev_wait(ev_done[prev_b])) {
        rc = REDSET_FAILURE;
        dev_failed = 1;
      }
      if (dev_failed) memset(h_out[prev_b], 0, (size_t) missing * B);
      int k = 0;
      if (need_rebuild)
        for (int step = 0; step < p; ++step) {
          const int lhs = (r - step + p) % p;
          irecv(h_gather + (size_t) lhs * B, (int) prev_count, lhs, TAG_GATHER, comm, &req[k++]);
        }
      for (int i = 0; i < missing; ++i)
        isend(h_out[prev_b] + (size_t) i * B, (int) prev_count, rebuild_ranks[i], TAG_GATHER, comm,
                  &req[k++]);
      mpi_waitall(k, req);
      if (need_rebuild) { /* :736-765 */
        for (int step = 0; step < p; ++step) {
          const int lhs = (r - step + p) % p;
          const int enc = redset_hip_rs_get_encoding_id(p, e, r, lhs);
          const uint8_t* cell = h_gather + (size_t) lhs * B;
          if (enc < p) {
            const int seg = redset_hip_rs_get_data_id(p, e, r, lhs);
            if (io_write(lofi, seg, prev_nread, prev_count, cell) != 0)
              rc = fail("lofi write failed");
          } else {
            const off_t off = header + (off_t) (enc - p) * (off_t) chunk_size + (off_t) prev_nread;
            if (pwrite_full(fd_chunk, cell, prev_count, off) != 0) rc = fail("write %s failed", chunk_file);
          }
        }
      }
    }
    if (!more) break;
    have_prev = 1;
    prev_b = bb;
    prev_nread = nread;
    prev_count = count;
  }
out:
  scratch_free(&S, rc == 0);
  for (int k = 0; k < 2; ++k)
    if (ev_done[k]) (void) hipEventDestroy(ev_done[k]);
  free(D);
  free(coef);
  free(cols);
  free(send_to);
  free(Dc);
  free(ins);
  free(outs);
  free(req);
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}

/* ---- XOR encode (replaces redset_xor_encode, src/redset_xor.c:220-295) */

static int xor_encode_impl(MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                           size_t chunk_size, size_t buf_size) {
  int p, r;
  off_t header;
  if (!lofi || !lofi->read) return fail("xor_encode_rank: null argument");
  if (comm_geometry(comm, &p, &r)) return REDSET_FAILURE;
  if (p < 2) return fail("XOR needs at least 2 ranks");
  /* a bad fd on one member is agreed on below, not returned early: its
   * peers would wait for it in the first collective */
  const int hrc = header_size(fd_chunk, chunk_file, &header);
  /* the caller's buffer as the slice: the RS rule (slice_bytes) measured
   * slower here (r04s9: 0.24-0.26 s against 0.17-0.23 s, XOR p = 8, 64 MiB) */
  const size_t B = buf_size ? buf_size : DEFAULT_BUF;
  if (B > (size_t) INT_MAX) return fail("buf_size %zu exceeds an MPI count", B); /* same on every rank */

  const unsigned char** ins = malloc(sizeof(*ins) * (size_t) p);
  MPI_Request* req = malloc(sizeof(*req) * 2 * (size_t) p);
  scratch S;
  scratch_init(&S);
  /* two sets of receive / result buffers: slice n's exchange runs while the
   * GPU combines slice n-1, whose result is written after it */
  uint8_t* h_send = scratch_host(&S, (size_t) p * B); /* my cell of stripe t, for t != r */
  uint8_t* h_recv[2] = {scratch_host(&S, (size_t) p * B), scratch_host(&S, (size_t) p * B)};
  uint8_t* h_out[2] = {scratch_host(&S, B), scratch_host(&S, B)};
  uint8_t* d_recv[2] = {scratch_dev(&S, (size_t) p * B), scratch_dev(&S, (size_t) p * B)};
  uint8_t* d_out[2] = {scratch_dev(&S, B), scratch_dev(&S, B)};
  hipEvent_t ev_done[2] = {NULL, NULL};
  int rc = S.rc ? S.rc : hrc;
  for (int k = 0; k < 2 && !rc; ++k)
    if (hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming) != hipSuccess) rc = fail("hipEventCreate failed");
  if (!rc && (!ins || !req)) rc = fail("out of host memory");
  if ((rc = agree_setup(comm, rc))) goto out;
  int dev_failed = 0; /* then keep exchanging, skip GPU work and writes */
  int have_prev = 0, prev_b = 0;
  size_t prev_nread = 0, prev_count = 0, n = 0;

  for (size_t nread = 0;; nread += B, ++n) {
    const int more = nread < chunk_size;
    const size_t count = more ? min_sz(B, chunk_size - nread) : 0;
    const int bb = (int) (n & 1);
    if (more) {
      /* the copy that read this receive buffer (slice n-2) is done: waited
       * for below when slice n-2's result was written */
      int k = 0;
      /* the ring of src/redset_xor.c:251-285 leaves member r with the XOR of
       * every other member's cell of stripe r; exchange those cells directly */
      for (int t = 0; t < p; ++t) {
        if (t == r) continue;
        if (io_read(lofi, xor_segment(r, t), nread, count,
                       h_send + (size_t) t * B) != 0) {
          rc = fail("lofi read failed");
          memset(h_send + (size_t) t * B, 0, count);
        }
        irecv(h_recv[bb] + (size_t) t * B, (int) count, t, 0, comm, &req[k++]);
        isend(h_send + (size_t) t * B, (int) count, t, 0, comm, &req[k++]);
      }
      mpi_waitall(k, req);
      if (!dev_failed) {
        int nin = 0;
        for (int t = 0; t < p; ++t)
          if (t != r) ins[nin++] = d_recv[bb] + (size_t) t * B;
        int grc = injected_device_failure(comm);
        if (!grc) grc = h2d(&S, d_recv[bb], h_recv[bb], (size_t) p * B);
        if (!grc) grc = redset_hip_xor_combine(ins, nin, d_out[bb], count, 0, S.stream);
        if (!grc) grc = d2h(&S, h_out[bb], d_out[bb], count);
        if (!grc) grc = ev_record(&S, ev_done[bb]);
        if (grc) {
          rc = grc;
          dev_failed = 1;
        }
      }
    }
    if (have_prev && !dev_failed) {
      if (ev_wait(ev_done[prev_b])) {
        rc = REDSET_FAILURE;
        dev_failed = 1;
      } else if (pwrite_full(fd_chunk, h_out[prev_b], prev_count, header + (off_t) prev_nread) != 0) { /* :280-284 */
        rc = fail("write %s failed", chunk_file);
      }
    }
    if (!more) break;
    have_prev = 1;
    prev_b = bb;
    prev_nread = nread;
    prev_count = count;
  }
out:
  scratch_free(&S, rc == 0);
  for (int k = 0; k < 2; ++k)
    if (ev_done[k]) (void) hipEventDestroy(ev_done[k]);
  free(ins);
  free(req);
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}


/* ---- XOR decode (replaces redset_xor_decode, src/redset_xor.c:441-531) */

#define XOR_CHAIN_SLICES_PER_HOP 4 /* the chain: at least this many slices per hop ... */
#define XOR_CHAIN_MIN_RANKS 6      /* ... and this many members (xor_decode_host) */

/* The XOR decode's gather to the root: every survivor sends its cell of
 * stripe c straight to the root (blocking sends, stripe by stripe), the root
 * XORs them on the GPU and writes its own cell of stripe c. One message per
 * cell, no hops: the shorter call when the chunk spans few slices. */
static int xor_decode_gather(MPI_Comm comm, int p, int r, int root, const redset_hip_io* lofi, const char* chunk_file,
                           int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t B) {

  const unsigned char** ins = malloc(sizeof(*ins) * (size_t) p);
  MPI_Request* req = malloc(sizeof(*req) * (size_t) p);
  scratch S;
  scratch_init(&S);
  /* the root double-buffers: unit n's cells arrive while the GPU XORs unit
   * n-1, whose result is written after */
  uint8_t* h_cells[2] = {scratch_host(&S, (size_t) p * B), scratch_host(&S, (size_t) p * B)};
  uint8_t* h_out[2] = {scratch_host(&S, B), scratch_host(&S, B)};
  uint8_t* d_cells[2] = {scratch_dev(&S, (size_t) p * B), scratch_dev(&S, (size_t) p * B)};
  uint8_t* d_out[2] = {scratch_dev(&S, B), scratch_dev(&S, B)};
  hipEvent_t ev_done[2] = {NULL, NULL};
  int rc = S.rc ? S.rc : hrc;
  for (int k = 0; k < 2 && !rc; ++k)
    if (hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming) != hipSuccess) rc = fail("hipEventCreate failed");
  if (!rc && (!ins || !req)) rc = fail("out of host memory");
  if ((rc = agree_setup(comm, rc))) goto out;
  int dev_failed = 0; /* root: keep receiving every cell, skip GPU work and writes */
  int have_prev = 0, prev_b = 0, prev_c = 0;
  size_t prev_nread = 0, prev_count = 0;
  long n = 0;

  /* stripe by stripe, as the reference's pipelined reduce to the root
   * (src/redset_xor.c:466-524): every survivor sends its cell of stripe c,
   * the root XORs them on the GPU and writes its own cell of stripe c */
  for (int c = 0; c <= p; ++c) {
    for (size_t nread = 0; c == p ? nread == 0 : nread < chunk_size; nread += B, ++n) {
      const int more = c < p;  /* c == p: one last pass to write the final unit */
      const size_t count = more ? min_sz(B, chunk_size - nread) : 0;
      const int bb = (int) (n & 1);
      if (more && r != root) {
        uint8_t* mine = h_cells[0] + (size_t) r * B;
        int bad;
        if (c != r) {
          bad = io_read(lofi, xor_segment(r, c), nread, count, mine) != 0;
          if (bad) rc = fail("lofi read failed");
        } else {
          bad = pread_full(fd_chunk, mine, count, header + (off_t) nread) != 0;
          if (bad) rc = fail("read %s failed", chunk_file);
        }
        if (bad) memset(mine, 0, count);
        const double t0 = now_s();
        MPI_Send(mine, (int) count, MPI_BYTE, root, 0, comm);
        g_stats.mpi_seconds += now_s() - t0;
        g_stats.sent_bytes += count;
        continue;
      }
      if (r != root) continue;
      if (more) {
        /* h_cells[bb] was last read by unit n-2's copy, waited for when
         * unit n-2 was written (below, during unit n-1) */
        int k = 0;
        for (int t = 0; t < p; ++t)
          if (t != root) irecv(h_cells[bb] + (size_t) t * B, (int) count, t, 0, comm, &req[k++]);
        mpi_waitall(k, req);
        if (!dev_failed) {
          int nin = 0;
          for (int t = 0; t < p; ++t)
            if (t != root) ins[nin++] = d_cells[bb] + (size_t) t * B;
          int grc = injected_device_failure(comm);
          if (!grc) grc = h2d(&S, d_cells[bb], h_cells[bb], (size_t) p * B);
          if (!grc) grc = redset_hip_xor_combine(ins, nin, d_out[bb], count, 0, S.stream);
          if (!grc) grc = d2h(&S, h_out[bb], d_out[bb], count);
          if (!grc) grc = ev_record(&S, ev_done[bb]);
          if (grc) {
            rc = grc;
            dev_failed = 1;
          }
        }
      }
      if (have_prev && !dev_failed) {
        if (ev_wait(ev_done[prev_b])) {
          rc = REDSET_FAILURE;
          dev_failed = 1;
        } else if (prev_c != root) {
          if (io_write(lofi, xor_segment(root, prev_c), prev_nread,
                                          prev_count, h_out[prev_b]) != 0)
            rc = fail("lofi write failed");
        } else if (pwrite_full(fd_chunk, h_out[prev_b], prev_count, header + (off_t) prev_nread) != 0) {
          rc = fail("write %s failed", chunk_file);
        }
      }
      have_prev = more;
      prev_b = bb;
      prev_c = c;
      prev_nread = nread;
      prev_count = count;
    }
  }
out:
  scratch_free(&S, rc == 0);
  for (int k = 0; k < 2; ++k)
    if (ev_done[k]) (void) hipEventDestroy(ev_done[k]);
  free(ins);
  free(req);
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}

/* The host-MPI exchange of the XOR decode: a chain through the survivors,
 * as the reference's pipelined reduce to the root (src/redset_xor.c:466-524),
 * but a slice of every stripe per message. Survivors in order root+1,
 * root+2, ..., root-1: the first sends its p cells of slice n (its data
 * segments and its parity, one per stripe) to the next; each following one
 * XORs what it receives with its own cells on the GPU and passes the result
 * on; the root receives, for every stripe, the XOR of every survivor's cell
 * -- its own lost cell -- and writes it. Every member sends and receives
 * p cells per slice, where a gather to the root would make the root receive
 * (p-1)*p. After a read or device error a member sends zeros and keeps the
 * chain going (src/redset_xor.c:466-524 keeps its loop going too), returning
 * failure. */
static int xor_decode_chain(MPI_Comm comm, int p, int r, int root, const redset_hip_io* lofi, const char* chunk_file,
                            int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t buf) {
  /* a message carries a slice of all p stripes: keep it within an MPI count
   * (the slice never changes the bytes written) */
  const size_t B = buf > (size_t) INT_MAX / (size_t) p ? (size_t) INT_MAX / (size_t) p : buf;
  const int pos = (r - root - 1 + p) % p; /* survivors 0 .. p-2, the root p-1 */
  const int prev = pos > 0 ? (r - 1 + p) % p : -1;
  const int next = pos < p - 1 ? (r + 1) % p : -1;
  const int survivor = next >= 0, compute = prev >= 0 && next >= 0;
  const size_t slab = (size_t) p * B; /* a slice of every stripe, cell c at c * count */
  scratch S;
  scratch_init(&S);
  uint8_t* h_own[2] = {NULL, NULL};
  uint8_t* h_in[2] = {NULL, NULL};
  uint8_t* h_res[2] = {NULL, NULL};
  uint8_t* d_own[2] = {NULL, NULL};
  uint8_t* d_in[2] = {NULL, NULL};
  for (int k = 0; k < 2; ++k) {
    if (survivor) h_own[k] = scratch_host(&S, slab);
    if (prev >= 0) h_in[k] = scratch_host(&S, slab);
    if (compute) {
      h_res[k] = scratch_host(&S, slab);
      d_own[k] = scratch_dev(&S, slab);
      d_in[k] = scratch_dev(&S, slab);
    }
  }
  hipEvent_t ev_done = NULL;
  int rc = S.rc ? S.rc : hrc;
  if (!rc && compute && hipEventCreateWithFlags(&ev_done, hipEventDisableTiming) != hipSuccess)
    rc = fail("hipEventCreate failed");
  if ((rc = agree_setup(comm, rc))) goto out;
  MPI_Request rreq[2] = {MPI_REQUEST_NULL, MPI_REQUEST_NULL}, sreq[2] = {MPI_REQUEST_NULL, MPI_REQUEST_NULL};
  int dev_failed = 0;
  const size_t nslice = (chunk_size + B - 1) / B;
  for (size_t n = 0; n < nslice; ++n) {
    const int b = (int) (n & 1);
    const size_t nread = n * B, count = min_sz(B, chunk_size - nread), bytes = (size_t) p * count;
    if (prev >= 0) irecv(h_in[b], (int) bytes, prev, 0, comm, &rreq[b]);
    if (survivor) {
      /* the first survivor sends h_own[b] itself: slice n-2's send is done */
      if (prev < 0) mpi_waitall(1, &sreq[b]);
      for (int c = 0; c < p; ++c) {
        uint8_t* mine = h_own[b] + (size_t) c * count;
        int bad;
        if (c != r) {
          bad = io_read(lofi, xor_segment(r, c), nread, count, mine) != 0;
          if (bad) rc = fail("lofi read failed");
        } else {
          bad = pread_full(fd_chunk, mine, count, header + (off_t) nread) != 0;
          if (bad) rc = fail("read %s failed", chunk_file);
        }
        if (bad) memset(mine, 0, count);
      }
    }
    if (prev < 0) {
      isend(h_own[b], (int) bytes, next, 0, comm, &sreq[b]);
      continue;
    }
    mpi_waitall(1, &rreq[b]);
    if (next < 0) {
      /* the root: stripe c's XOR of every survivor's cell is its own cell */
      for (int c = 0; c < p; ++c) {
        const uint8_t* cell = h_in[b] + (size_t) c * count;
        if (c != root) {
          if (io_write(lofi, xor_segment(root, c), nread, count, cell) != 0) rc = fail("lofi write failed");
        } else if (pwrite_full(fd_chunk, cell, count, header + (off_t) nread) != 0) {
          rc = fail("write %s failed", chunk_file);
        }
      }
      continue;
    }
    /* h_res[b] is free once slice n-2's send is done */
    mpi_waitall(1, &sreq[b]);
    int grc = dev_failed ? REDSET_FAILURE : injected_device_failure(comm);
    if (!grc) grc = h2d(&S, d_own[b], h_own[b], bytes);
    if (!grc) grc = h2d(&S, d_in[b], h_in[b], bytes);
    if (!grc) {
      const unsigned char* in1[1] = {d_in[b]};
      grc = redset_hip_xor_combine(in1, 1, d_own[b], bytes, 1, S.stream);
    }
    if (!grc) grc = d2h(&S, h_res[b], d_own[b], bytes);
    if (!grc) grc = ev_record(&S, ev_done);
    if (!grc) grc = ev_wait(ev_done);
    if (grc) {
      if (!dev_failed) rc = rc ? rc : grc;
      dev_failed = 1;
      memset(h_res[b], 0, bytes);
    }
    isend(h_res[b], (int) bytes, next, 0, comm, &sreq[b]);
  }
  mpi_waitall(2, sreq);
  mpi_waitall(2, rreq);
out:
  scratch_free(&S, rc == 0);
  if (ev_done) (void) hipEventDestroy(ev_done);
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}

/* The host-MPI exchange of the XOR decode: the chain for wide sets whose
 * chunk spans enough slices to fill it, else the gather. Measured on one box
 * (1 MiB buffers, profiles/r04s21_xor_decode_order.txt): at p = 4 the gather
 * wins at every chunk size (5.3-64 MiB: 2.2-2.5x), at p = 8 it wins at 8 MiB
 * (1.3x) and loses at 32 and 64 MiB (chain 1.45x and 1.75x faster), where
 * the root's (p-1)*p cells per slice swamp it. Every member derives the same
 * choice from the same arguments. */
static int xor_decode_host(MPI_Comm comm, int p, int r, int root, const redset_hip_io* lofi, const char* chunk_file,
                           int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t B) {
  const size_t nslice = (chunk_size + B - 1) / B;
  int chain = p >= XOR_CHAIN_MIN_RANKS && nslice >= (size_t) XOR_CHAIN_SLICES_PER_HOP * (size_t) (p - 1);
#if REDSET_HIP_TEST_KNOBS
  /* test builds: REDSET_HIP_TEST_XOR_DECODE=gather|chain forces one (A/B runs, tests) */
  const char* v = getenv("REDSET_HIP_TEST_XOR_DECODE");
  if (v) chain = strcmp(v, "chain") == 0;
#endif
  return chain ? xor_decode_chain(comm, p, r, root, lofi, chunk_file, fd_chunk, header, hrc, chunk_size, B)
               : xor_decode_gather(comm, p, r, root, lofi, chunk_file, fd_chunk, header, hrc, chunk_size, B);
}

/* ---- the multi-rank rebuild over the sharded plan (RCCL / xGMI) ---------- */
/*
 * When the members of the set each own a GPU of one node, the decode does
 * not pass cells between hosts at all: every member reads the cells some
 * stripe's decode needs into HBM, and the sharded plan (sharded.c) gathers
 * column slices of them onto every member's GPU over the transport -- RCCL
 * over xGMI --, runs gf_mac on each GPU's slice of every stripe, and returns
 * the rebuilt slices to the lost members, which write them after the header
 * as the host path does. This replaces the decode's ring and its gather to
 * the failed ranks (src/redset_reedsolomon.c:646-703, :713-733) and the XOR
 * decode's pipelined reduce to the root (src/redset_xor.c:466-524).
 *
 * The chunk goes in windows of at most kWindow bytes of staging per cell set
 * (double-buffered: the reads of window n+1 overlap the exchange and the
 * kernels of window n). Each window starts with one MPI_Allreduce(LAND) of
 * every member's state, so a read or device error on one member stops every
 * member before the next exchange: all return failure, none hangs (the
 * reference keeps its ring going instead, :666-681; the caller's AND-reduce
 * fails the call either way).
 */
#define SHARDED_WINDOW ((size_t) 96 << 20) /* host staging per window buffer, all cells */

static int g_exchange_mode = REDSET_HIP_EXCHANGE_AUTO;
static __thread int g_last_exchange = 0;

int redset_hip_rank_set_exchange(int mode) {
  if (mode < REDSET_HIP_EXCHANGE_AUTO || mode > REDSET_HIP_EXCHANGE_SHARDED_HOST)
    return fail("rank_set_exchange: unknown mode %d", mode);
  g_exchange_mode = mode;
  return REDSET_SUCCESS;
}

int redset_hip_rank_last_exchange(void) { return g_last_exchange; }

/* What the sharded slot keeps from one call to the next on a communicator
 * (a "slot context"): its pinned window images, device slabs, stream,
 * events and the sharded plans of every window, for one call shape. A
 * checkpoint loop calls the same shape again and again, and planning, the
 * plans' streams, the pinned images and the slabs are then set up once
 * instead of per call (round 5: they were ~20% of a warm call on one box,
 * profiles/r05s4_rank_roofline.jsonl). Another shape replaces it; a failed
 * call frees it; REDSET_HIP_SCRATCH_CACHE=0 or redset_hip_rank_scratch_release
 * frees it too. */
typedef struct {
  /* the shape it serves */
  int host, encode, xor_scheme, p, e, missing, lost[256], r, device;
  size_t chunk_size, win;
  redset_hip_transport tr;
  /* what it holds */
  size_t W, WW, nwin, tail, xbytes, xmsgs;
  unsigned char* want;
  /* device slabs, double-buffered over the windows, behind pinned window
   * images; host = 1 (_SHARDED_HOST): one set of slabs in pinned host
   * memory, no images */
  uint8_t *h_img[2], *hd[2], *hp[2], *gd[2], *gp[2];
  redset_hip_sharded* plan[2][2]; /* [buffer][tail window] */
  hipEvent_t ev[2];
  hipStream_t stream;
  hipStream_t xs; /* host slabs: the gathers' (idle) stream, so a gather never waits for a compute */
} slot_ctx;

static void slot_ctx_free(slot_ctx* C) {
  if (!C) return;
  if (C->stream) (void) hipStreamSynchronize(C->stream);
  for (int b = 0; b < 2; ++b) {
    for (int t = 0; t < 2; ++t) redset_hip_sharded_destroy(C->plan[b][t]);
    if (C->ev[b]) (void) hipEventDestroy(C->ev[b]);
    if (C->h_img[b]) (void) hipHostFree(C->h_img[b]);
    uint8_t* slab[4] = {C->hd[b], C->hp[b], C->gd[b], C->gp[b]};
    for (int k = 0; k < 4; ++k)
      if (slab[k]) (void) (C->host ? hipHostFree(slab[k]) : hipFree(slab[k]));
  }
  if (C->stream) (void) hipStreamDestroy(C->stream);
  if (C->xs) (void) hipStreamDestroy(C->xs);
  free(C->want);
  free(C);
}

/* per-communicator exchange, decided once and cached on the communicator
 * (an MPI attribute: the RCCL communicator, a _SHARDED_MPI transport and the
 * slot context are destroyed with it) */
typedef struct comm_exchange {
  int decided;             /* the RCCL decision has been made */
  int mode;                /* REDSET_HIP_EXCHANGE_HOST_MPI or _SHARDED_RCCL */
  redset_hip_transport tr;
  redset_hip_rccl* rccl;
  redset_hip_transport mt_tr;  /* _SHARDED_MPI: the MPI transport with device buffers */
  redset_hip_mpi_transport* mt;
  redset_hip_transport ht_tr;  /* _SHARDED_HOST: the MPI transport over host slabs */
  redset_hip_mpi_transport* ht;
  slot_ctx* ctx;
  int busy;                /* a sharded call is using mt / ctx (under exch_mu) */
  struct comm_exchange* next; /* the live list (exch_register) */
} comm_exchange;

/* every live comm_exchange, so redset_hip_rank_scratch_release can free
 * what they cache: an intrusive list, so no communicator is ever left out
 * (a fixed table of 64 dropped the 65th silently) */
static pthread_mutex_t exch_mu = PTHREAD_MUTEX_INITIALIZER;
static comm_exchange* exch_head;

static void exch_register(comm_exchange* X, int add) {
  pthread_mutex_lock(&exch_mu);
  if (add) {
    X->next = exch_head;
    exch_head = X;
  } else {
    for (comm_exchange** pp = &exch_head; *pp; pp = &(*pp)->next)
      if (*pp == X) {
        *pp = X->next;
        break;
      }
    X->next = NULL;
  }
  pthread_mutex_unlock(&exch_mu);
}

/* the communicator's cached sharded resources, freed (the RCCL communicator stays) */
static void exch_release(comm_exchange* X) {
  slot_ctx_free(X->ctx);
  X->ctx = NULL;
  redset_hip_mpi_transport_destroy(X->mt);
  X->mt = NULL;
  redset_hip_mpi_transport_destroy(X->ht);
  X->ht = NULL;
}

static int exch_keyval = MPI_KEYVAL_INVALID;

static int exch_delete(MPI_Comm comm, int keyval, void* attr, void* extra) {
  (void) comm, (void) keyval, (void) extra;
  comm_exchange* X = (comm_exchange*) attr;
  if (X) {
    exch_register(X, 0);
    exch_release(X);
    redset_hip_rccl_transport_destroy(X->rccl);
  }
  free(X);
  return MPI_SUCCESS;
}

/* the communicator's comm_exchange, made on first use (local) */
static int exch_get(MPI_Comm comm, comm_exchange** out) {
  *out = NULL;
  if (exch_keyval == MPI_KEYVAL_INVALID &&
      MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, exch_delete, &exch_keyval, NULL) != MPI_SUCCESS)
    return fail("MPI_Comm_create_keyval failed");
  comm_exchange* X = NULL;
  int found = 0;
  if (MPI_Comm_get_attr(comm, exch_keyval, &X, &found) != MPI_SUCCESS) return fail("MPI_Comm_get_attr failed");
  if (!found) {
    X = calloc(1, sizeof(*X));
    if (!X) return fail("out of host memory");
    X->mode = REDSET_HIP_EXCHANGE_HOST_MPI;
    if (MPI_Comm_set_attr(comm, exch_keyval, X) != MPI_SUCCESS) {
      free(X);
      return fail("MPI_Comm_set_attr failed");
    }
    exch_register(X, 1);
  }
  *out = X;
  return 0;
}

/* members on one node, each with its own GPU, and librccl loadable on every
 * member (collective; the same answer on every member) */
static int rccl_possible(MPI_Comm comm, int p, int r) {
  int ok = 1;
  MPI_Comm node;
  if (MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, r, MPI_INFO_NULL, &node) == MPI_SUCCESS) {
    int n = 0;
    MPI_Comm_size(node, &n);
    ok = n == p;
    MPI_Comm_free(&node);
  } else {
    ok = 0;
  }
  char bus[64];
  memset(bus, 0, sizeof(bus));
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(bus, (int) sizeof(bus) - 1, dev) != hipSuccess) ok = 0;
  char* all = malloc((size_t) p * sizeof(bus));
  if (!all) ok = 0;
  if (all && MPI_Allgather(bus, (int) sizeof(bus), MPI_CHAR, all, (int) sizeof(bus), MPI_CHAR, comm) == MPI_SUCCESS) {
    for (int a = 0; a < p && ok; ++a)
      for (int b = a + 1; b < p && ok; ++b)
        if (strncmp(all + (size_t) a * sizeof(bus), all + (size_t) b * sizeof(bus), sizeof(bus)) == 0) ok = 0;
  } else {
    ok = 0;
  }
  free(all);
  ok = ok && redset_hip_rccl_available();
  int all_ok = 0;
  if (MPI_Allreduce(&ok, &all_ok, 1, MPI_INT, MPI_LAND, comm) != MPI_SUCCESS) return 0;
  return all_ok;
}

/* a one-rank-per-GPU RCCL communicator over comm's members (collective) */
static int rccl_create(MPI_Comm comm, int p, int r, comm_exchange* X) {
  unsigned char id[129];
  memset(id, 0, sizeof(id));
  if (r == 0) id[128] = redset_hip_rccl_unique_id(id) == REDSET_SUCCESS;
  if (MPI_Bcast(id, (int) sizeof(id), MPI_BYTE, 0, comm) != MPI_SUCCESS) return fail("MPI_Bcast failed");
  if (!id[128]) return fail("RCCL unique id failed on member 0");
  int rc = redset_hip_rccl_transport_create(id, p, r, &X->tr, &X->rccl);
  int ok = rc == 0, all = 0;
  if (MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_LAND, comm) != MPI_SUCCESS) return fail("MPI_Allreduce failed");
  if (!all) {
    redset_hip_rccl_transport_destroy(X->rccl);
    X->rccl = NULL;
    return rc ? rc : fail("a peer's RCCL communicator failed");
  }
  return 0;
}

/* What AUTO means for a call (the same on every member):
 *   AUTO_DECODE       RCCL when the members each own a GPU of one node, else
 *                     the host path
 *   AUTO_ENCODE_SLABS the sharded plan over host slabs (_SHARDED_HOST): an RS
 *                     encode with d, e >= 2 and p <= AUTO_SLABS_MAX_P, where it
 *                     sends (d + e)(p - 1)/p cells per member against the
 *                     ring's d*e (RS(8+3): 10 against 24) and measured faster
 *                     on one box too (profiles/r05s12_rank_roofline.jsonl,
 *                     r05s26_rank_roofline_rs10p4.jsonl: p = 11, 14). Past
 *                     that a window's messages shrink as 1/p (its slices as
 *                     1/p^2), where the ring keeps whole slices
 *   AUTO_ENCODE_HOST  the host ring: XOR encodes and RS ones with e = 1 or
 *                     d = 1, where the two send the same bytes, and wider sets
 * AUTO never sends an encode over RCCL: north_star asks for RCCL "only for
 * the multi-rank rebuild case", and an encode over RCCL has not yet run on a
 * node with a GPU per member; forcing _SHARDED_RCCL still does. */
enum { AUTO_ENCODE_HOST = 0, AUTO_DECODE = 1, AUTO_ENCODE_SLABS = 2 };
#define AUTO_SLABS_MAX_P 32

/* The exchange of this call (collective): the process's mode -- every
 * member must set the same one -- or, for AUTO, what `autop` picks. For the
 * sharded modes *xo is the communicator's comm_exchange: its transport
 * (RCCL, or an MPI transport, made on first use and kept) and its slot
 * context. */
static int choose_exchange_now(MPI_Comm comm, int p, int r, int autop, int* mode, comm_exchange** xo);
static void exch_busy(comm_exchange* X, int busy);
static int choose_exchange(MPI_Comm comm, int p, int r, int autop, int* mode, comm_exchange** xo) {
  const double t0 = now_s();
  const int rc = choose_exchange_now(comm, p, r, autop, mode, xo);
  g_stats.setup_seconds += now_s() - t0;
  return rc;
}

static int choose_exchange_now(MPI_Comm comm, int p, int r, int autop, int* mode, comm_exchange** xo) {
  int m[2] = {g_exchange_mode, -g_exchange_mode}, mm[2];
  *xo = NULL;
  if (MPI_Allreduce(m, mm, 2, MPI_INT, MPI_MAX, comm) != MPI_SUCCESS) return fail("MPI_Allreduce failed");
  if (mm[0] != -mm[1]) return fail("members disagree on the rebuild exchange (redset_hip_rank_set_exchange)");
  *mode = m[0];
  if (*mode == REDSET_HIP_EXCHANGE_AUTO && autop == AUTO_ENCODE_HOST) *mode = REDSET_HIP_EXCHANGE_HOST_MPI;
  if (*mode == REDSET_HIP_EXCHANGE_AUTO && autop == AUTO_ENCODE_SLABS) *mode = REDSET_HIP_EXCHANGE_SHARDED_HOST;
  if (*mode == REDSET_HIP_EXCHANGE_HOST_MPI) return 0;
  comm_exchange* X = NULL;
  int rc = exch_get(comm, &X);
  if (*mode == REDSET_HIP_EXCHANGE_SHARDED_MPI || *mode == REDSET_HIP_EXCHANGE_SHARDED_HOST) {
    /* the sharded plan over MPI: with device buffers staged through pinned
     * memory (_SHARDED_MPI), or over slabs in pinned host memory that the
     * kernels read and write in place (_SHARDED_HOST); members may share a
     * GPU */
    if (!rc) exch_busy(X, 1);
    if (!rc && *mode == REDSET_HIP_EXCHANGE_SHARDED_MPI && !X->mt)
      rc = redset_hip_mpi_transport_create(comm, 1, &X->mt_tr, &X->mt);
    if (!rc && *mode == REDSET_HIP_EXCHANGE_SHARDED_HOST && !X->ht)
      rc = redset_hip_mpi_transport_create(comm, 2, &X->ht_tr, &X->ht);
    if ((rc = agree_setup(comm, rc))) {
      if (X) exch_busy(X, 0);
      return rc;
    }
    *xo = X;
    return 0;
  }
  if ((rc = agree_setup(comm, rc))) return rc;
  if (!X->decided) {
    if (*mode == REDSET_HIP_EXCHANGE_SHARDED_RCCL || rccl_possible(comm, p, r)) {
      if (rccl_create(comm, p, r, X) == 0) X->mode = REDSET_HIP_EXCHANGE_SHARDED_RCCL;
      else if (*mode == REDSET_HIP_EXCHANGE_SHARDED_RCCL) return REDSET_FAILURE;
    }
    X->decided = 1;
  }
  if (*mode == REDSET_HIP_EXCHANGE_SHARDED_RCCL && X->mode != REDSET_HIP_EXCHANGE_SHARDED_RCCL)
    return fail("RCCL exchange requested, but this communicator uses the host path");
  *mode = X->mode;
  if (*mode != REDSET_HIP_EXCHANGE_HOST_MPI) exch_busy(X, 1); /* until sharded_slot ends */
  *xo = X;
  return 0;
}

/* a communicator whose sharded call is running keeps its cache: that call
 * holds the transport and the context */
static void exch_release_all(void) {
  pthread_mutex_lock(&exch_mu);
  for (comm_exchange* X = exch_head; X; X = X->next)
    if (!X->busy) exch_release(X);
  pthread_mutex_unlock(&exch_mu);
}

static void exch_busy(comm_exchange* X, int busy) {
  pthread_mutex_lock(&exch_mu);
  X->busy = busy;
  pthread_mutex_unlock(&exch_mu);
}

/* member r's cell in stripe c: data cell x (0 <= x < d) or parity slot
 * d + i, as sharded.c cell_of numbers them */
static int member_cell(int p, int e, int xor_scheme, int r, int c) {
  if (xor_scheme) return c == r ? p - 1 : xor_segment(r, c);
  const int enc = redset_hip_rs_get_encoding_id(p, e, r, c);
  return enc < p ? redset_hip_rs_get_data_id(p, e, r, c) : (p - e) + (enc - p);
}

/* The slot context for this call: the communicator's cached one when it
 * serves this shape, else a new one -- buffers, stream, events, the cells of
 * mine the exchange reads, and the plans of every window (planning is
 * local: no communication, every member the same), with the MPI transport's
 * staging and requests sized for the largest exchange, so no exchange
 * allocates (a failed allocation there would leave the peers waiting).
 * Returns the context, or NULL with *rc set. */
static slot_ctx* slot_ctx_get(comm_exchange* X, int host_slabs, const redset_hip_transport* tr,
                              redset_hip_mpi_transport* mt, int encode, const redset_hip_rs* rs, int p, int r, int e,
                              int missing, const int* lost, int need_rebuild, size_t chunk_size, size_t win, int* rc) {
  const int xor_scheme = rs == NULL, d = p - e, ncell = p, world = p;
  int device = -1;
  (void) hipGetDevice(&device);
  slot_ctx* C = X->ctx;
  if (C) {
    int same = C->host == host_slabs && C->encode == encode && C->xor_scheme == xor_scheme && C->p == p && C->e == e &&
               C->missing == missing && C->r == r && C->device == device && C->chunk_size == chunk_size &&
               C->win == win && C->tr.exchange == tr->exchange && C->tr.ctx == tr->ctx;
    for (int i = 0; i < missing && same; ++i) same = C->lost[i] == lost[i];
    if (same) return C;
    X->ctx = NULL;
    slot_ctx_free(C);
  }
  C = calloc(1, sizeof(*C));
  if (!C) {
    *rc = fail("out of host memory");
    return NULL;
  }
  C->host = host_slabs, C->encode = encode, C->xor_scheme = xor_scheme, C->p = p, C->e = e, C->missing = missing, C->r = r;
  C->device = device, C->chunk_size = chunk_size, C->win = win, C->tr = *tr;
  for (int i = 0; i < missing; ++i) C->lost[i] = lost[i];
  /* every member computes a column slice. A decode computing on the
   * survivors only (redset_hip_rs_sharded_plan_on) cuts a lost member's
   * receive from 1208 to 738 MB (RS(8+3), two lost), but on one box the
   * host-slab decode then took 0.584 s against the host exchange's 0.359 s
   * in the same session (profiles/r05s30_*), where computing on every
   * member had been 0.372 against 0.318 s (r05s12) */
  const int* on = NULL;
  C->W = redset_hip_shard_slice_bytes(win, world);
  C->WW = C->W * (size_t) world; /* one cell's window in the host image */
  C->nwin = chunk_size ? (chunk_size + win - 1) / win : 0;
  C->tail = chunk_size - (C->nwin ? (C->nwin - 1) * win : 0);
  const double t0 = now_s();
  int err = 0;
  const size_t W = C->W;
  for (int b = 0; b < 2 && !err && host_slabs; ++b) {
    /* slabs in page-locked host memory: MPI sends and receives them
     * directly, the kernels read and write them over PCIe */
    if (hipHostMalloc((void**) &C->hd[b], (size_t) world * d * W, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**) &C->hp[b], (size_t) world * e * W, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**) &C->gd[b], (size_t) world * d * W, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**) &C->gp[b], (size_t) world * e * W, hipHostMallocDefault) != hipSuccess)
      err = fail("sharded slot: allocating %zu B of host slabs failed", (size_t) 2 * ncell * C->WW);
    if (!err && hipEventCreateWithFlags(&C->ev[b], hipEventDisableTiming) != hipSuccess) err = fail("hipEventCreate failed");
  }
  if (!err && host_slabs && hipStreamCreateWithFlags(&C->xs, hipStreamNonBlocking) != hipSuccess) {
    C->xs = NULL;
    err = fail("hipStreamCreate failed");
  }
  for (int b = 0; b < 2 && !err && !host_slabs; ++b) {
    if (hipHostMalloc((void**) &C->h_img[b], (size_t) ncell * C->WW, hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void**) &C->hd[b], (size_t) world * d * W) != hipSuccess ||
        hipMalloc((void**) &C->hp[b], (size_t) world * e * W) != hipSuccess ||
        hipMalloc((void**) &C->gd[b], (size_t) world * d * W) != hipSuccess ||
        hipMalloc((void**) &C->gp[b], (size_t) world * e * W) != hipSuccess)
      err = fail("sharded slot: allocating %zu B of window buffers failed", (size_t) ncell * C->WW);
    if (!err && hipEventCreateWithFlags(&C->ev[b], hipEventDisableTiming) != hipSuccess) err = fail("hipEventCreate failed");
  }
  if (!err && hipStreamCreateWithFlags(&C->stream, hipStreamNonBlocking) != hipSuccess) {
    C->stream = NULL;
    err = fail("hipStreamCreate failed");
  }
  C->want = calloc((size_t) ncell, 1); /* cells of mine some stripe's decode reads */
  unsigned char* D = malloc((size_t) (missing > 0 ? missing : 1) * p);
  int* host = malloc(sizeof(int) * (size_t) p);
  int* slot = calloc((size_t) p, sizeof(int));
  if (!err && (!C->want || !D || !host || !slot)) err = fail("out of host memory");
  g_stats.setup_seconds += now_s() - t0;
  /* which of my cells the exchange reads: the encode every data cell, the
   * decode those its maps read (the sharded plan sends exactly those) */
  for (int x = 0; x < d && encode && !err; ++x) C->want[x] = 1;
  for (int c = 0; c < p && !err && !need_rebuild && !encode; ++c) {
    int used = xor_scheme;
    if (!xor_scheme) {
      err = redset_hip_rs_decode_matrix(rs, missing, lost, c, D);
      for (int i = 0; i < missing && !err; ++i) used |= D[(size_t) i * p + r] != 0;
    }
    if (used) C->want[member_cell(p, e, xor_scheme, r, c)] = 1;
  }
  for (int m = 0; m < p && host; ++m) host[m] = m;
  /* the plans of buffers b = n & 1 of window n, whole or tail */
  const double tp = now_s();
  for (size_t n = 0; n < C->nwin && !err; ++n) {
    const size_t len = n + 1 == C->nwin ? C->tail : win;
    const int b = (int) (n & 1);
    redset_hip_sharded** P = &C->plan[b][len != win];
    if (*P) continue;
    redset_hip_shard_layout L = {1, host, slot, 1, len, W, C->hd[b], C->hp[b], C->gd[b], C->gp[b]};
    if (encode)
      err = xor_scheme ? redset_hip_xor_sharded_plan_on(p, REDSET_HIP_PLAN_XOR_ENCODE, 0, &L, on, tr, NULL, P)
                       : redset_hip_rs_sharded_plan_on(rs, REDSET_HIP_PLAN_RS_ENCODE, 0, NULL, &L, on, tr, NULL, P);
    else
      err = xor_scheme ? redset_hip_xor_sharded_plan_on(p, REDSET_HIP_PLAN_XOR_REBUILD, lost[0], &L, on, tr, NULL, P)
                       : redset_hip_rs_sharded_plan_on(rs, REDSET_HIP_PLAN_RS_REBUILD, missing, lost, &L, on, tr, NULL,
                                                       P);
    redset_hip_sharded_info info;
    if (!err && !(err = redset_hip_sharded_get_info(*P, &info))) {
      const size_t gb = info.gather_bytes_sent + info.gather_bytes_recv;
      const size_t rb = info.return_bytes_sent + info.return_bytes_recv;
      const size_t gm = (size_t) info.gather_messages + (size_t) info.gather_recv_messages;
      const size_t rm = (size_t) info.return_messages + (size_t) info.return_recv_messages;
      C->xbytes = gb > C->xbytes ? gb : C->xbytes;
      C->xbytes = rb > C->xbytes ? rb : C->xbytes;
      C->xmsgs = gm > C->xmsgs ? gm : C->xmsgs;
      C->xmsgs = rm > C->xmsgs ? rm : C->xmsgs;
    }
  }
  if (!err && mt) err = redset_hip_mpi_transport_reserve(mt, C->xbytes, C->xmsgs);
  g_stats.plan_seconds += now_s() - tp;
  free(D);
  free(host);
  free(slot);
  if (err) {
    slot_ctx_free(C);
    *rc = err;
    return NULL;
  }
  return C;
}

/* cell bytes per window of the sharded slot: `budget` over the p cells a
 * member holds (4 KiB multiples, at least 64 KiB), at most the chunk. The
 * caller's MPI buffer size does not raise it: the window sizes every pinned
 * image and slab of the call (host slabs: two sets of hosted + gathered
 * slabs, ~4 p win), and a window raised to a 64 MiB buffer pinned 2.8 GiB per
 * member for RS(8+3); the messages are the window's column
 * slices, not MPI buffers, so B has no say in them */
static size_t slot_window(size_t budget, size_t chunk_size, int ncell, size_t B) {
  (void) B;
  size_t win = budget / (size_t) ncell / 4096 * 4096;
  if (win < ((size_t) 64 << 10)) win = (size_t) 64 << 10;
#if REDSET_HIP_TEST_KNOBS
  /* test builds: small windows, so small sets take several (the mid-call stop) */
  if (getenv("REDSET_HIP_TEST_SHARDED_WINDOW")) win = (size_t) atoll(getenv("REDSET_HIP_TEST_SHARDED_WINDOW"));
#endif
  if (win > chunk_size) win = chunk_size;
  if (win == 0) win = 1;
  return win;
}

/* the context's epilogue of a sharded call: it serves the next call of this
 * shape; a failed call's, or every call's with the cache off, goes */
static int slot_done(comm_exchange* X, slot_ctx* C, int rc) {
  const double tt = now_s();
  if (C && C->stream && hipStreamSynchronize(C->stream) != hipSuccess && !rc) rc = fail("stream sync failed");
  if (C && (rc || !cache_on())) {
    slot_ctx_free(C);
    C = NULL;
  }
  X->ctx = C;
  exch_busy(X, 0);
  g_stats.setup_seconds += now_s() - tt;
  return rc ? REDSET_FAILURE : REDSET_SUCCESS;
}

/* _SHARDED_HOST: the sharded plan with every slab in page-locked host
 * memory. A member reads its cells' window slice by slice straight into its
 * hosted slabs, MPI sends and receives the slabs themselves, and the gf_mac
 * (or XOR) kernels read the gathered slices and write the results over PCIe
 * in place (as the zero-copy streaming path does), so nothing is staged or
 * copied. What crosses the network per member is the plan's column slices,
 * (d + e)(p - 1)/p cells for the encode, where the reference's ring sends
 * every data cell to each of the e parity holders, d*e cells
 * (src/redset_reedsolomon.c:329-363): RS(8+3) 10 cells instead of 24.
 * Windows alternate between two slab sets of SHARDED_WINDOW of cells each
 * (a member's p cells; each set holds the hosted and the gathered slabs, so
 * ~4 p win = 384 MiB pinned in all, whatever the MPI buffer: round 6 cut the
 * window from the buffer size, which had pinned 2.8 GiB at a 64 MiB buffer
 * (ADVICE r5), and measured the window at the default 1 MiB buffer, RS(8+3),
 * 64 MiB chunks, one box: 4 / 8 / 16 MiB windows encode in 0.715 / 0.524 /
 * 0.579 s against the host ring's 0.808 s, profiles/r06s5_*), and their
 * phases overlap: window n's
 * kernels run on the GPU while the host writes window n - 1, reads window
 * n + 1 and runs its gather; window n's return follows. Every member runs the
 * same collectives in the same order: agree(n), gather(n), return(n - 1). */
static int sharded_slot_host(int encode, const redset_hip_rs* rs, MPI_Comm comm, int p, int r, int e, int missing,
                             const int* lost, int need_rebuild, const redset_hip_io* lofi, const char* chunk_file,
                             int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t B, comm_exchange* X) {
  const int d = p - e, ncell = p, world = p;
  const size_t win = slot_window(SHARDED_WINDOW, chunk_size, ncell, B);
  int rc = hrc;
  if (!rc && need_rebuild && !lofi->write) rc = fail("lofi has no write callback");
  int crc = 0;
  slot_ctx* C = slot_ctx_get(X, 1, &X->ht_tr, X->ht, encode, rs, p, r, e, missing, lost, need_rebuild, chunk_size,
                             win, &crc);
  if (!rc) rc = crc;
  if ((rc = agree_setup(comm, rc))) return slot_done(X, C, rc);

  const size_t W = C->W, nwin = C->nwin, tail = C->tail;
  hipStream_t s = C->stream; /* the kernels, and the returns, which wait for them */
  const int writes = need_rebuild || encode;
  /* slice q of cell x in the hosted slabs b ([world][1][d][W], [world][1][e][W]) */
#define HOST_SLICE(b, x, q) ((x) < d ? C->hd[b] + ((size_t) (q) * d + (size_t) (x)) * W \
                                     : C->hp[b] + ((size_t) (q) * e + (size_t) ((x) - d)) * W)
#define WIN_LEN(n) ((n) + 1 == nwin ? tail : win)
  for (size_t n = 0; n <= nwin; ++n) {
    const int b = (int) (n & 1), pb = 1 - b;
    redset_hip_sharded* P = n < nwin ? C->plan[b][WIN_LEN(n) != win] : NULL;
    redset_hip_sharded* Pp = n >= 1 ? C->plan[pb][WIN_LEN(n - 1) != win] : NULL;
    if (n < nwin) {
      /* window n into slabs b, last used by window n - 2: its return and
       * writes are done (iteration n - 1), and its kernels are waited for
       * here, not left to the return's stream sync as a side effect (a
       * member with no return traffic never syncs it) */
      const size_t off = n * win, len = WIN_LEN(n);
      if (n >= 2 && !rc && ev_wait(C->ev[b])) rc = REDSET_FAILURE;
      for (int x = 0; x < ncell && !rc; ++x) {
        if (!C->want[x]) continue;
        for (size_t q = 0; q < (size_t) world && q * W < len && !rc; ++q) {
          const size_t lo = q * W, k = min_sz(W, len - lo);
          if (x < d) {
            if (io_read(lofi, x, off + lo, k, HOST_SLICE(b, x, q)) != 0) rc = fail("lofi read failed");
          } else if (pread_full(fd_chunk, HOST_SLICE(b, x, q), k,
                                header + (off_t) (x - d) * (off_t) chunk_size + (off_t) (off + lo)) != 0) {
            rc = fail("read %s failed", chunk_file);
          }
        }
      }
      /* every member's state before the window's exchanges: one failure
       * stops all (window n - 1's return is skipped by every member alike) */
      int ok = rc == 0, all = 0;
      const double ta = now_s();
      if (MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_LAND, comm) != MPI_SUCCESS) rc = fail("MPI_Allreduce failed");
      g_stats.mpi_seconds += now_s() - ta;
      if (!all) {
        if (!rc) rc = fail("a peer's read or device step failed");
        break;
      }
      if (!rc) rc = injected_device_failure(comm);
      if (!P && !rc) rc = fail("sharded window without a plan");
      /* the gather runs whatever this member's state since the agreement
       * (its peers are in it), on the idle stream: window n - 1's kernels
       * keep running */
      const double tx = now_s();
      if (P && redset_hip_sharded_execute_phase(P, REDSET_HIP_PHASE_GATHER, C->xs) != 0 && !rc) rc = REDSET_FAILURE;
      g_stats.exchange_seconds += now_s() - tx;
    }
    if (Pp) {
      /* window n - 1's results back to their holders, after its kernels (the
       * MPI transport waits for `s` before it posts) */
      const double tx = now_s();
      if (redset_hip_sharded_execute_phase(Pp, REDSET_HIP_PHASE_RETURN, s) != 0 && !rc) rc = REDSET_FAILURE;
      g_stats.exchange_seconds += now_s() - tx;
    }
    if (P) {
      /* window n's kernels, queued behind nothing: the host goes on */
      if (!rc && redset_hip_sharded_execute_phase(P, REDSET_HIP_PHASE_COMPUTE, s) != 0) rc = REDSET_FAILURE;
      if (!rc && hipEventRecord(C->ev[b], s) != hipSuccess) rc = fail("hipEventRecord failed");
      redset_hip_sharded_info info;
      if (redset_hip_sharded_get_info(P, &info) == 0) {
        g_stats.sent_bytes += info.gather_bytes_sent + info.return_bytes_sent;
        g_stats.recv_bytes += info.gather_bytes_recv + info.return_bytes_recv;
        /* the kernels' PCIe traffic: my slice of every stripe's inputs in,
         * of its outputs out */
        const unsigned long long out_b = (unsigned long long) p * (unsigned long long) (encode ? e : missing) *
                                         info.my_slice_len;
        g_stats.d2h_bytes += out_b;
        g_stats.h2d_bytes += info.compute_bytes > out_b ? info.compute_bytes - out_b : 0;
      }
    }
    if (Pp && writes && !rc) {
      /* window n - 1's rebuilt cells (encode: its parity cells), after the
       * header as the host path writes them; the slices computed in place
       * (my own) are done with its kernels */
      const size_t off = (n - 1) * win, len = WIN_LEN(n - 1);
      if (ev_wait(C->ev[pb])) rc = REDSET_FAILURE;
      for (int x = encode ? d : 0; x < ncell && !rc; ++x) {
        for (size_t q = 0; q < (size_t) world && q * W < len && !rc; ++q) {
          const size_t lo = q * W, k = min_sz(W, len - lo);
          if (x < d) {
            if (io_write(lofi, x, off + lo, k, HOST_SLICE(pb, x, q)) != 0) rc = fail("lofi write failed");
          } else if (pwrite_full(fd_chunk, HOST_SLICE(pb, x, q), k,
                                 header + (off_t) (x - d) * (off_t) chunk_size + (off_t) (off + lo)) != 0) {
            rc = fail("write %s failed", chunk_file);
          }
        }
      }
    }
  }
#undef WIN_LEN
#undef HOST_SLICE
  return slot_done(X, C, rc);
}

/* The encode (encode = 1: every member's data cells in, its parity cells
 * out) or the rebuild (the lost members' cells) as the sharded plan over the
 * communicator's transport (X: RCCL, or the _SHARDED_MPI transport; the
 * _SHARDED_HOST mode goes to sharded_slot_host). rs == NULL: XOR (e = 1;
 * rebuild: the root is lost[0]). */
static int sharded_slot(int encode, const redset_hip_rs* rs, MPI_Comm comm, int p, int r, int e, int missing,
                        const int* lost, int need_rebuild, const redset_hip_io* lofi, const char* chunk_file,
                        int fd_chunk, off_t header, int hrc, size_t chunk_size, size_t B, comm_exchange* X,
                        int mode) {
  if (mode == REDSET_HIP_EXCHANGE_SHARDED_HOST)
    return sharded_slot_host(encode, rs, comm, p, r, e, missing, lost, need_rebuild, lofi, chunk_file, fd_chunk,
                             header, hrc, chunk_size, B, X);
  const int d = p - e, ncell = p, world = p;
  const size_t win = slot_window(SHARDED_WINDOW, chunk_size, ncell, B);
  int rc = hrc;
  if (!rc && need_rebuild && !lofi->write) rc = fail("lofi has no write callback");
  int crc = 0;
  /* the mode's transport: RCCL, or the MPI transport with device buffers */
  const int over_mpi = mode == REDSET_HIP_EXCHANGE_SHARDED_MPI;
  slot_ctx* C = slot_ctx_get(X, 0, over_mpi ? &X->mt_tr : &X->tr, over_mpi ? X->mt : NULL, encode, rs, p, r, e,
                             missing, lost, need_rebuild, chunk_size, win, &crc);
  if (!rc) rc = crc;
  if ((rc = agree_setup(comm, rc))) goto out;

  const size_t W = C->W, WW = C->WW, nwin = C->nwin, tail = C->tail;
  for (size_t n = 0; n <= nwin; ++n) {
    const int b = (int) (n & 1);
    const size_t off = n * win, len = n + 1 == nwin ? tail : win;
    if (n < nwin) {
      /* buffers b were last used by window n - 2, written at window n - 1 */
      if (n >= 2 && !rc && ev_wait(C->ev[b])) rc = REDSET_FAILURE;
      /* the plan of buffers b for a whole window, or for the tail window */
      redset_hip_sharded* P = C->plan[b][len != win];
      uint8_t* img = C->h_img[b];
      for (int x = 0; x < ncell && !rc; ++x) {
        if (!C->want[x]) continue;
        uint8_t* dst = img + (size_t) x * WW;
        if (x < d) {
          if (io_read(lofi, x, off, len, dst) != 0) rc = fail("lofi read failed");
        } else if (pread_full(fd_chunk, dst, len, header + (off_t) (x - d) * (off_t) chunk_size + (off_t) off) != 0) {
          rc = fail("read %s failed", chunk_file);
        }
      }
      /* every member's state before the exchange: one failure stops all */
      int ok = rc == 0, all = 0;
      const double ta = now_s();
      if (MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_LAND, comm) != MPI_SUCCESS) rc = fail("MPI_Allreduce failed");
      g_stats.mpi_seconds += now_s() - ta;
      if (!all) {
        if (!rc) rc = fail("a peer's read or device step failed");
        break;
      }
      hipStream_t s = C->stream;
      if (!rc) rc = injected_device_failure(comm);
      double tc = now_s();
      for (int x = 0; x < ncell && !rc; ++x) {
        if (!C->want[x]) continue;
        uint8_t* dst = x < d ? C->hd[b] + (size_t) x * W : C->hp[b] + (size_t) (x - d) * W;
        const size_t dpitch = (size_t) (x < d ? d : e) * W;
        if (hipMemcpy2DAsync(dst, dpitch, img + (size_t) x * WW, W, W, (size_t) world, hipMemcpyHostToDevice, s) !=
            hipSuccess)
          rc = fail("H2D copy failed");
        g_stats.h2d_bytes += WW;
      }
      g_stats.copy_seconds += now_s() - tc;
      /* the exchange runs whatever this member's state since the agreement:
       * its peers are in it (a member whose copies failed sends what its
       * buffers hold, and every member stops at the next window's agreement) */
      const double tx = now_s();
      if (!P) {
        if (!rc) rc = fail("sharded window without a plan");
      } else if (redset_hip_sharded_execute(P, s) != 0 && !rc) {
        rc = REDSET_FAILURE;
      }
      g_stats.exchange_seconds += now_s() - tx;
      redset_hip_sharded_info info;
      if (!rc && redset_hip_sharded_get_info(P, &info) == 0) {
        g_stats.sent_bytes += info.gather_bytes_sent + info.return_bytes_sent;
        g_stats.recv_bytes += info.gather_bytes_recv + info.return_bytes_recv;
      }
      tc = now_s();
      for (int x = encode ? d : 0; x < ncell && !rc && (need_rebuild || encode); ++x) {
        const uint8_t* src = x < d ? C->hd[b] + (size_t) x * W : C->hp[b] + (size_t) (x - d) * W;
        const size_t spitch = (size_t) (x < d ? d : e) * W;
        if (hipMemcpy2DAsync(img + (size_t) x * WW, W, src, spitch, W, (size_t) world, hipMemcpyDeviceToHost, s) !=
            hipSuccess)
          rc = fail("D2H copy failed");
        g_stats.d2h_bytes += WW;
      }
      g_stats.copy_seconds += now_s() - tc;
      if (!rc && hipEventRecord(C->ev[b], s) != hipSuccess) rc = fail("hipEventRecord failed");
    }
    /* window n - 1's rebuilt cells (encode: parity cells), after the header
     * as the host path writes them */
    if (n >= 1 && (need_rebuild || encode) && !rc) {
      const int pb = 1 - b;
      const size_t poff = (n - 1) * win, plen = n == nwin ? tail : win;
      if (ev_wait(C->ev[pb])) rc = REDSET_FAILURE;
      for (int x = encode ? d : 0; x < ncell && !rc; ++x) {
        const uint8_t* cell = C->h_img[pb] + (size_t) x * WW;
        if (x < d) {
          if (io_write(lofi, x, poff, plen, cell) != 0) rc = fail("lofi write failed");
        } else if (pwrite_full(fd_chunk, cell, plen, header + (off_t) (x - d) * (off_t) chunk_size + (off_t) poff) != 0) {
          rc = fail("write %s failed", chunk_file);
        }
      }
    }
  }
out:;
  return slot_done(X, C, rc);
}

int redset_hip_rs_decode_rank(const redset_hip_rs* rs, MPI_Comm comm, int missing, const int* rebuild_ranks,
                              int need_rebuild, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                              size_t chunk_size, size_t buf_size) {
  int p, r, rp, e;
  off_t header;
  const double t0 = stats_begin();
  if (!rs || !lofi || !rebuild_ranks) return fail("rs_decode_rank: null argument");
  if (comm_geometry(comm, &p, &r) || redset_hip_rs_shape(rs, &rp, &e)) return REDSET_FAILURE;
  if (p != rp) return fail("communicator has %d ranks, codec %d", p, rp);
  if (missing < 1 || missing > e) return fail("cannot rebuild %d members with %d encoding blocks", missing, e);
  for (int i = 0; i < missing; ++i)
    if (rebuild_ranks[i] < 0 || rebuild_ranks[i] >= p || (i && rebuild_ranks[i] <= rebuild_ranks[i - 1]))
      return fail("rebuild ranks must be ascending members of 0..%d", p - 1); /* same on every rank */
  /* a bad fd on one member is agreed on later, not returned early: its
   * peers would wait for it in the first collective */
  const int hrc = header_size(fd_chunk, chunk_file, &header);
  const size_t B = buf_size ? buf_size : DEFAULT_BUF;
  if (B > (size_t) INT_MAX) return fail("buf_size %zu exceeds an MPI count", B); /* same on every rank */
  int mode;
  comm_exchange* X = NULL;
  if (choose_exchange(comm, p, r, AUTO_DECODE, &mode, &X)) return REDSET_FAILURE;
  g_last_exchange = mode;
  int rc = mode == REDSET_HIP_EXCHANGE_HOST_MPI
               ? rs_decode_host(rs, comm, p, r, e, missing, rebuild_ranks, need_rebuild, lofi, chunk_file, fd_chunk,
                                header, hrc, chunk_size, slice_bytes(B, chunk_size, (size_t) (4 * p + 2 * missing)))
               : sharded_slot(0, rs, comm, p, r, e, missing, rebuild_ranks, need_rebuild, lofi, chunk_file, fd_chunk,
                              header, hrc, chunk_size, B, X, mode);
  return stats_end(t0, rc);
}

int redset_hip_xor_decode_rank(MPI_Comm comm, int root, const redset_hip_io* lofi, const char* chunk_file,
                               int fd_chunk, size_t chunk_size, size_t buf_size) {
  int p, r;
  off_t header;
  const double t0 = stats_begin();
  if (!lofi || !lofi->read) return fail("xor_decode_rank: null argument");
  if (comm_geometry(comm, &p, &r)) return REDSET_FAILURE;
  if (p < 2) return fail("XOR needs at least 2 ranks");
  if (root < 0 || root >= p) return fail("root %d out of range", root);
  /* a bad fd on one member is agreed on later, not returned early: its
   * peers would wait for it in the first collective */
  const int hrc = header_size(fd_chunk, chunk_file, &header);
  const size_t B = buf_size ? buf_size : DEFAULT_BUF;
  if (B > (size_t) INT_MAX) return fail("buf_size %zu exceeds an MPI count", B); /* same on every rank */
  int mode;
  comm_exchange* X = NULL;
  if (choose_exchange(comm, p, r, AUTO_DECODE, &mode, &X)) return REDSET_FAILURE;
  g_last_exchange = mode;
  int rc = mode == REDSET_HIP_EXCHANGE_HOST_MPI
               ? xor_decode_host(comm, p, r, root, lofi, chunk_file, fd_chunk, header, hrc, chunk_size, B)
               : sharded_slot(0, NULL, comm, p, r, 1, 1, &root, r == root, lofi, chunk_file, fd_chunk, header, hrc,
                              chunk_size, B, X, mode);
  return stats_end(t0, rc);
}

/* The encodes: the sharded plan (every data cell's column slices gathered
 * onto the GPUs, gf_mac (or the XOR) there, the parity slices returned to
 * their holders) under a sharded mode and, over host slabs, under AUTO for RS
 * with e >= 2; else the host ring (src/redset_reedsolomon.c:329-377,
 * src/redset_xor.c:251-285). */
static int encode_rank(const redset_hip_rs* rs, MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file,
                       int fd_chunk, size_t chunk_size, size_t buf_size) {
  int p, r, e = 1;
  if (!lofi || !lofi->read) return fail("encode_rank: null argument");
  if (comm_geometry(comm, &p, &r)) return REDSET_FAILURE;
  if (rs) {
    int rp;
    if (redset_hip_rs_shape(rs, &rp, &e)) return REDSET_FAILURE;
    if (p != rp) return fail("communicator has %d ranks, codec %d", p, rp);
  } else if (p < 2) {
    return fail("XOR needs at least 2 ranks");
  }
  const size_t B = buf_size ? buf_size : DEFAULT_BUF;
  if (B > (size_t) INT_MAX) return fail("buf_size %zu exceeds an MPI count", B); /* same on every rank */
  int mode;
  comm_exchange* X = NULL;
  /* fewer bytes than the ring needs d >= 2 and e >= 2: (d + e)(p - 1)/p < d*e */
  const int slabs = rs && e >= 2 && p - e >= 2 && p <= AUTO_SLABS_MAX_P;
  if (choose_exchange(comm, p, r, slabs ? AUTO_ENCODE_SLABS : AUTO_ENCODE_HOST, &mode, &X))
    return REDSET_FAILURE;
  g_last_exchange = mode;
  int rc;
  if (mode == REDSET_HIP_EXCHANGE_HOST_MPI) {
    rc = rs ? rs_encode_impl(rs, comm, lofi, chunk_file, fd_chunk, chunk_size, buf_size)
            : xor_encode_impl(comm, lofi, chunk_file, fd_chunk, chunk_size, buf_size);
  } else {
    /* a bad fd on one member is agreed on inside, not returned early */
    off_t header;
    const int hrc = header_size(fd_chunk, chunk_file, &header);
    rc = sharded_slot(1, rs, comm, p, r, e, 0, NULL, 0, lofi, chunk_file, fd_chunk, header, hrc, chunk_size, B, X,
                      mode);
  }
  return rc;
}

int redset_hip_rs_encode_rank(const redset_hip_rs* rs, MPI_Comm comm, const redset_hip_io* lofi,
                              const char* chunk_file, int fd_chunk, size_t chunk_size, size_t buf_size) {
  const double t0 = stats_begin();
  if (!rs) return stats_end(t0, fail("rs_encode_rank: null argument"));
  return stats_end(t0, encode_rank(rs, comm, lofi, chunk_file, fd_chunk, chunk_size, buf_size));
}

int redset_hip_xor_encode_rank(MPI_Comm comm, const redset_hip_io* lofi, const char* chunk_file, int fd_chunk,
                               size_t chunk_size, size_t buf_size) {
  const double t0 = stats_begin();
  return stats_end(t0, encode_rank(NULL, comm, lofi, chunk_file, fd_chunk, chunk_size, buf_size));
}

/* ---- MPI transport of the sharded path (include/redset_hip_mpi.h) ------- */

#define MPI_PIECE ((size_t) 1 << 30) /* bytes per MPI message (int counts) */

struct redset_hip_mpi_transport {
  MPI_Comm comm;
  int world, rank, device;
  int hip_host;     /* host buffers that HIP kernels on `stream` read and write */
  uint8_t* stage;   /* staging (device mode): pinned, or malloc'd if pinning failed */
  size_t stage_len;
  int stage_pinned;
  MPI_Request* req;
  int req_cap;
};

/* staging and requests for `need` bytes and `nreq` MPI requests */
static int mpi_transport_size(struct redset_hip_mpi_transport* T, size_t need, size_t nreq) {
  if (T->device && need > T->stage_len) {
    if (T->stage) T->stage_pinned ? (void) hipHostFree(T->stage) : free(T->stage);
    T->stage = NULL;
    T->stage_len = 0;
    T->stage_pinned = hipHostMalloc((void**) &T->stage, need, hipHostMallocDefault) == hipSuccess;
    /* pageable memory carries the messages as well (its copies are slower) */
    if (!T->stage_pinned) T->stage = malloc(need);
    if (!T->stage) return fail("mpi transport: out of host memory (%zu)", need);
    T->stage_len = need;
  }
  if (nreq > (size_t) T->req_cap) {
    MPI_Request* r = realloc(T->req, sizeof(*r) * nreq);
    if (!r) return fail("mpi transport: out of host memory (%zu requests)", nreq);
    T->req = r;
    T->req_cap = (int) nreq;
  }
  return 0;
}

int redset_hip_mpi_transport_reserve(redset_hip_mpi_transport* T, size_t bytes, size_t messages) {
  if (!T) return fail("mpi_transport_reserve: null transport");
  /* messages above MPI_PIECE go in pieces: at most bytes / MPI_PIECE more */
  return mpi_transport_size(T, bytes, messages + bytes / MPI_PIECE + 1) ? REDSET_FAILURE : REDSET_SUCCESS;
}

/* Every message of the exchange is posted and waited for even after a HIP
 * error on this member (its peers are in the same exchange and would hang,
 * src/redset_reedsolomon.c:338-342): the error is returned at the end, and
 * the bytes this member sent are unspecified. Only buffers that were not
 * reserved (redset_hip_mpi_transport_reserve) and then fail to allocate
 * return before the messages are posted. Where the host thread waits goes to
 * the call's stats (redset_hip_rank_last_stats): the GPU work that feeds
 * the exchange (gpu_seconds), the staging copies (stage_seconds), MPI
 * (mpi_seconds). */
static int mpi_exchange(void* ctx, const redset_hip_xfer* x, int n, void* stream) {
  struct redset_hip_mpi_transport* T = (struct redset_hip_mpi_transport*) ctx;
  hipStream_t s = (hipStream_t) stream;
  int rc = 0;
  size_t need = 0, nreq = 0;
  for (int i = 0; i < n; ++i)
    if (x[i].peer != T->rank) {
      need += x[i].len;
      nreq += (x[i].len + MPI_PIECE - 1) / MPI_PIECE;
    }
  if (mpi_transport_size(T, need, nreq)) return REDSET_FAILURE;
  /* work already on the stream produced the send buffers -- in host mode
   * too, where a HIP compute over page-locked slabs may still be writing
   * them, on the null stream as well (device_buffers = 2); a host-only
   * caller (device_buffers = 0, no stream) needs no HIP runtime */
  double t0 = now_s();
  if ((T->device || T->hip_host || s) && hipStreamSynchronize(s) != hipSuccess)
    rc = fail("mpi transport: stream sync failed");
  g_stats.gpu_seconds += now_s() - t0;
  /* local copies, and (device mode) every send staged to host */
  t0 = now_s();
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    if (x[i].peer == T->rank) {
      if (i + 1 >= n || !x[i].send || x[i + 1].send || x[i + 1].peer != T->rank || x[i + 1].len != x[i].len)
        return fail("mpi transport: malformed local copy"); /* a plan bug, the same on every member */
      if (!rc && T->device) {
        if (hipMemcpyAsync(x[i + 1].buf, x[i].buf, x[i].len, hipMemcpyDeviceToDevice, s) != hipSuccess)
          rc = fail("mpi transport: local copy failed");
      } else if (!rc) {
        memmove(x[i + 1].buf, x[i].buf, x[i].len);
      }
      ++i;
      continue;
    }
    if (!rc && T->device && x[i].send &&
        hipMemcpyAsync(T->stage + off, x[i].buf, x[i].len, hipMemcpyDeviceToHost, s) != hipSuccess)
      rc = fail("mpi transport: D2H staging failed");
    off += x[i].len;
  }
  if (!rc && T->device && hipStreamSynchronize(s) != hipSuccess) rc = fail("mpi transport: stream sync failed");
  g_stats.stage_seconds += now_s() - t0;
  int k = 0;
  off = 0;
  for (int i = 0; i < n; ++i) {
    if (x[i].peer == T->rank) {
      ++i;
      continue;
    }
    uint8_t* base = T->device ? T->stage + off : (uint8_t*) x[i].buf;
    for (size_t done = 0; done < x[i].len; done += MPI_PIECE) {
      const int cnt = (int) min_sz(MPI_PIECE, x[i].len - done);
      if (x[i].send) MPI_Isend(base + done, cnt, MPI_BYTE, x[i].peer, 7, T->comm, &T->req[k++]);
      else MPI_Irecv(base + done, cnt, MPI_BYTE, x[i].peer, 7, T->comm, &T->req[k++]);
    }
    off += x[i].len;
  }
  t0 = now_s();
  const int mrc = MPI_Waitall(k, T->req, MPI_STATUSES_IGNORE);
  g_stats.mpi_seconds += now_s() - t0;
  if (mrc != MPI_SUCCESS) return fail("mpi transport: MPI_Waitall failed");
  if (!T->device || rc) return rc;
  t0 = now_s();
  off = 0;
  for (int i = 0; i < n && !rc; ++i) {
    if (x[i].peer == T->rank) {
      ++i;
      continue;
    }
    if (!x[i].send && hipMemcpyAsync(x[i].buf, T->stage + off, x[i].len, hipMemcpyHostToDevice, s) != hipSuccess)
      rc = fail("mpi transport: H2D failed");
    off += x[i].len;
  }
  /* the staging buffer is reused by the next exchange */
  if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = fail("mpi transport: stream sync failed");
  g_stats.stage_seconds += now_s() - t0;
  return rc;
}

int redset_hip_mpi_transport_create(MPI_Comm comm, int device_buffers, redset_hip_transport* out,
                                    redset_hip_mpi_transport** handle) {
  if (!out || !handle) return fail("mpi_transport_create: null argument");
  *handle = NULL;
  struct redset_hip_mpi_transport* T = calloc(1, sizeof(*T));
  if (!T) return fail("out of host memory");
  if (comm_geometry(comm, &T->world, &T->rank)) {
    free(T);
    return REDSET_FAILURE;
  }
  T->comm = comm;
  if (device_buffers < 0 || device_buffers > 2) {
    free(T);
    return fail("mpi_transport_create: device_buffers %d is not 0, 1 or 2", device_buffers);
  }
  T->device = device_buffers == 1;
  T->hip_host = device_buffers == 2;
  out->world = T->world;
  out->rank = T->rank;
  out->exchange = mpi_exchange;
  out->ctx = T;
  *handle = T;
  return REDSET_SUCCESS;
}

void redset_hip_mpi_transport_destroy(redset_hip_mpi_transport* T) {
  if (!T) return;
  if (T->stage && T->stage_pinned) (void) hipHostFree(T->stage);
  else free(T->stage);
  free(T->req);
  free(T);
}
