/* rcclstub.c -- TEST INFRASTRUCTURE ONLY: a stand-in for librccl.so.1 with
 * the eight entry points the sharded path's RCCL transport resolves
 * (redset_amd/csrc/transport_rccl.c rccl_open: ncclGetErrorString,
 * ncclGroupStart / ncclGroupEnd, ncclSend / ncclRecv, ncclGetUniqueId,
 * ncclCommInitRank, ncclCommDestroy), so that transport's code -- grouped
 * point-to-point sends and receives, local copies, the cached communicator of
 * the per-rank slot (rank_mpi.c) and dist.py's RcclTransport -- runs at
 * world > 1 on a box with ONE GPU, where the real RCCL refuses two ranks on
 * the same device ("Duplicate GPU"). It is built into tests/rcclstub/ and
 * loaded only by tests: through LD_LIBRARY_PATH for the C drivers (which
 * dlopen "librccl.so.1"), or through the test twin's
 * REDSET_HIP_TEST_RCCL_LIBRARY in torch processes (torch has already mapped
 * the real librccl.so.1 there). The product never names it.
 *
 * Semantics: a communicator is a POSIX shared-memory segment named by the
 * unique id, holding one single-producer / single-consumer byte ring per
 * directed pair of ranks. ncclSend / ncclRecv inside a group are recorded;
 * ncclGroupEnd synchronises the streams they were posted on (so the bytes a
 * send reads are final and a receive overwrites nothing still in use), then
 * moves every message through the rings with hipMemcpy, progressing all of
 * them at once (pairs exchanging in both directions never wait on each
 * other), and returns when all are done: a stream-ordered RCCL group, made
 * synchronous. Messages between a pair are framed with their length and
 * matched in posting order, as RCCL matches them; a length mismatch is an
 * ncclInvalidUsage error instead of a hang. No progress for 120 s is an
 * ncclSystemError (a peer that never posts its side). Any number of ranks
 * may share a GPU.
 */
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define STUB_MAGIC 0x52434353u /* "RCCS" */
#define STUB_TIMEOUT_S 120.0
#define MAX_OPS 65536

typedef struct {
  unsigned long long wpos; /* bytes the sender has written (release) */
  unsigned long long rpos; /* bytes the receiver has consumed (release) */
  char pad[48];
} chan_hdr;

typedef struct {
  int arrived, departed, world;
  int pad;
  unsigned long long chan_bytes;
} seg_hdr;

struct ncclComm {
  int world, rank;
  char name[64];
  size_t map_bytes, chan_bytes;
  unsigned char* base;
};

typedef struct {
  int send, peer;
  unsigned char* buf;
  size_t len;
  hipStream_t stream;
  struct ncclComm* comm;
  size_t done;      /* payload bytes moved */
  int hdr_done;     /* frame header moved */
} stub_op;

static __thread stub_op* g_ops;
static __thread int g_nops, g_cap, g_depth;
static __thread char g_err[256];

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double) t.tv_sec + 1e-9 * (double) t.tv_nsec;
}

const char* ncclGetErrorString(ncclResult_t r) {
  if (g_err[0]) return g_err;
  switch (r) {
    case ncclSuccess: return "no error";
    case ncclSystemError: return "rcclstub: system error";
    case ncclInvalidArgument: return "rcclstub: invalid argument";
    case ncclInvalidUsage: return "rcclstub: invalid usage";
    default: return "rcclstub: error";
  }
}

static ncclResult_t stub_fail(ncclResult_t r, const char* msg) {
  snprintf(g_err, sizeof(g_err), "rcclstub: %s", msg);
  return r;
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return stub_fail(ncclInvalidArgument, "null id");
  memset(id, 0, sizeof(*id));
  unsigned char rnd[16];
  int fd = open("/dev/urandom", O_RDONLY);
  if (fd < 0 || read(fd, rnd, sizeof(rnd)) != (ssize_t) sizeof(rnd)) {
    if (fd >= 0) close(fd);
    return stub_fail(ncclSystemError, "cannot read /dev/urandom");
  }
  close(fd);
  char* s = id->internal;
  int n = snprintf(s, 64, "/rcclstub_%d_", (int) getpid());
  for (int i = 0; i < 16 && n < 60; ++i) n += snprintf(s + n, 64 - (size_t) n, "%02x", rnd[i]);
  return ncclSuccess;
}

static chan_hdr* chan_of(struct ncclComm* c, int from, int to) {
  const size_t stride = sizeof(chan_hdr) + c->chan_bytes;
  return (chan_hdr*) (c->base + 4096 + ((size_t) from * (size_t) c->world + (size_t) to) * stride);
}
static unsigned char* chan_data(struct ncclComm* c, chan_hdr* h) { (void) c; return (unsigned char*) (h + 1); }

ncclResult_t ncclCommInitRank(ncclComm_t* out, int world, ncclUniqueId id, int rank) {
  if (!out || world < 1 || rank < 0 || rank >= world) return stub_fail(ncclInvalidArgument, "bad world / rank");
  if (strncmp(id.internal, "/rcclstub_", 10) != 0) return stub_fail(ncclInvalidArgument, "not a stub unique id");
  struct ncclComm* c = calloc(1, sizeof(*c));
  if (!c) return stub_fail(ncclSystemError, "out of memory");
  c->world = world;
  c->rank = rank;
  snprintf(c->name, sizeof(c->name), "%.60s", id.internal);
  /* ring bytes per directed pair: 4 MiB, less for wide worlds (64 MiB of rings) */
  size_t cb = ((size_t) 64 << 20) / ((size_t) world * (size_t) world);
  if (cb > ((size_t) 4 << 20)) cb = (size_t) 4 << 20;
  if (cb < ((size_t) 256 << 10)) cb = (size_t) 256 << 10;
  c->chan_bytes = cb;
  c->map_bytes = 4096 + (size_t) world * (size_t) world * (sizeof(chan_hdr) + cb);
  int fd = shm_open(c->name, O_CREAT | O_RDWR, 0600);
  if (fd < 0) {
    free(c);
    return stub_fail(ncclSystemError, "shm_open failed");
  }
  /* every rank sizes it alike; truncating to the same size changes nothing */
  if (ftruncate(fd, (off_t) c->map_bytes) != 0) {
    close(fd);
    free(c);
    return stub_fail(ncclSystemError, "ftruncate failed");
  }
  c->base = mmap(NULL, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (c->base == MAP_FAILED) {
    free(c);
    return stub_fail(ncclSystemError, "mmap failed");
  }
  seg_hdr* H = (seg_hdr*) c->base;
  __atomic_store_n(&H->world, world, __ATOMIC_RELAXED);
  __atomic_add_fetch(&H->arrived, 1, __ATOMIC_ACQ_REL);
  const double t0 = now_s();
  while (__atomic_load_n(&H->arrived, __ATOMIC_ACQUIRE) < world) {
    if (now_s() - t0 > STUB_TIMEOUT_S) {
      munmap(c->base, c->map_bytes);
      free(c);
      return stub_fail(ncclSystemError, "ranks did not all arrive");
    }
    usleep(200);
  }
  *out = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  seg_hdr* H = (seg_hdr*) c->base;
  if (__atomic_add_fetch(&H->departed, 1, __ATOMIC_ACQ_REL) == c->world) shm_unlink(c->name);
  munmap(c->base, c->map_bytes);
  free(c);
  return ncclSuccess;
}

ncclResult_t ncclGroupStart(void) {
  ++g_depth;
  return ncclSuccess;
}

static ncclResult_t post(int send, const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                         hipStream_t stream) {
  if (type != ncclUint8 && type != ncclInt8) return stub_fail(ncclInvalidArgument, "only byte messages");
  if (!comm || peer < 0 || peer >= comm->world || peer == comm->rank)
    return stub_fail(ncclInvalidArgument, "bad peer");
  if (g_nops == g_cap) {
    int cap = g_cap ? 2 * g_cap : 64;
    if (cap > MAX_OPS) return stub_fail(ncclInvalidUsage, "too many operations in one group");
    stub_op* v = realloc(g_ops, sizeof(*v) * (size_t) cap);
    if (!v) return stub_fail(ncclSystemError, "out of memory");
    g_ops = v;
    g_cap = cap;
  }
  stub_op o = {send, peer, (unsigned char*) buf, count, stream, comm, 0, 0};
  g_ops[g_nops++] = o;
  return g_depth > 0 ? ncclSuccess : ncclGroupEnd();
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
  return post(1, buf, count, type, peer, comm, stream);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
  return post(0, buf, count, type, peer, comm, stream);
}

/* move what the ring allows for op o; returns 1 if it progressed, -1 on error */
static int progress(stub_op* o) {
  struct ncclComm* c = o->comm;
  chan_hdr* h = o->send ? chan_of(c, c->rank, o->peer) : chan_of(c, o->peer, c->rank);
  unsigned char* data = chan_data(c, h);
  const unsigned long long cap = c->chan_bytes;
  int moved = 0;
  if (o->send) {
    unsigned long long w = __atomic_load_n(&h->wpos, __ATOMIC_RELAXED);
    const unsigned long long r = __atomic_load_n(&h->rpos, __ATOMIC_ACQUIRE);
    if (!o->hdr_done) {
      if (cap - (w - r) < 16) return 0;
      unsigned long long frame[2] = {STUB_MAGIC, o->len};
      for (int i = 0; i < 16; ++i) data[(w + (unsigned long long) i) % cap] = ((unsigned char*) frame)[i];
      w += 16;
      o->hdr_done = 1;
      moved = 1;
      __atomic_store_n(&h->wpos, w, __ATOMIC_RELEASE);
    }
    while (o->done < o->len) {
      const unsigned long long room = cap - (w - __atomic_load_n(&h->rpos, __ATOMIC_ACQUIRE));
      if (room == 0) break;
      const unsigned long long at = w % cap;
      size_t n = o->len - o->done;
      if (n > room) n = (size_t) room;
      if (n > cap - at) n = (size_t) (cap - at);
      if (hipMemcpy(data + at, o->buf + o->done, n, hipMemcpyDefault) != hipSuccess) return -1;
      o->done += n;
      w += n;
      moved = 1;
      __atomic_store_n(&h->wpos, w, __ATOMIC_RELEASE);
    }
    return moved;
  }
  unsigned long long r = __atomic_load_n(&h->rpos, __ATOMIC_RELAXED);
  if (!o->hdr_done) {
    const unsigned long long w = __atomic_load_n(&h->wpos, __ATOMIC_ACQUIRE);
    if (w - r < 16) return 0;
    unsigned long long frame[2];
    for (int i = 0; i < 16; ++i) ((unsigned char*) frame)[i] = data[(r + (unsigned long long) i) % cap];
    if (frame[0] != STUB_MAGIC || frame[1] != o->len) {
      snprintf(g_err, sizeof(g_err), "rcclstub: rank %d receives %zu B from %d, which sends %llu B", c->rank, o->len,
               o->peer, frame[1]);
      return -2;
    }
    r += 16;
    o->hdr_done = 1;
    moved = 1;
    __atomic_store_n(&h->rpos, r, __ATOMIC_RELEASE);
  }
  while (o->done < o->len) {
    const unsigned long long avail = __atomic_load_n(&h->wpos, __ATOMIC_ACQUIRE) - r;
    if (avail == 0) break;
    const unsigned long long at = r % cap;
    size_t n = o->len - o->done;
    if (n > avail) n = (size_t) avail;
    if (n > cap - at) n = (size_t) (cap - at);
    if (hipMemcpy(o->buf + o->done, data + at, n, hipMemcpyDefault) != hipSuccess) return -1;
    o->done += n;
    r += n;
    moved = 1;
    __atomic_store_n(&h->rpos, r, __ATOMIC_RELEASE);
  }
  return moved;
}

ncclResult_t ncclGroupEnd(void) {
  if (g_depth > 0) --g_depth;
  if (g_depth > 0) return ncclSuccess;
  ncclResult_t rc = ncclSuccess;
  g_err[0] = 0;
  /* the streams the operations were posted on: their earlier work first */
  for (int i = 0; i < g_nops; ++i) {
    int seen = 0;
    for (int k = 0; k < i && !seen; ++k) seen = g_ops[k].stream == g_ops[i].stream;
    if (!seen && hipStreamSynchronize(g_ops[i].stream) != hipSuccess) rc = stub_fail(ncclSystemError, "stream sync");
  }
  double last = now_s();
  for (int left = g_nops; left > 0 && rc == ncclSuccess;) {
    int any = 0;
    left = 0;
    for (int i = 0; i < g_nops && rc == ncclSuccess; ++i) {
      stub_op* o = &g_ops[i];
      if (o->hdr_done && o->done == o->len) continue;
      /* messages of one direction of a pair go in posting order */
      int first = 1;
      for (int k = 0; k < i && first; ++k) {
        const stub_op* q = &g_ops[k];
        if (q->send == o->send && q->peer == o->peer && q->comm == o->comm && !(q->hdr_done && q->done == q->len))
          first = 0;
      }
      ++left;
      if (!first) continue;
      const int m = progress(o);
      if (m == -1) rc = stub_fail(ncclSystemError, "hipMemcpy failed");
      if (m == -2) rc = ncclInvalidUsage;
      any |= m > 0;
    }
    if (rc != ncclSuccess || left == 0) break;
    if (any) {
      last = now_s();
    } else {
      if (now_s() - last > STUB_TIMEOUT_S) rc = stub_fail(ncclSystemError, "no progress for 120 s (a peer never posted)");
      usleep(20);
    }
  }
  g_nops = 0;
  return rc;
}
