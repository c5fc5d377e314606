/*
 * transport_rccl.c -- the sharded path's transport over RCCL / xGMI
 * (include/redset_hip.h: redset_hip_rccl_*). One exchange = one
 * ncclGroupStart/End of point-to-point ncclSend / ncclRecv on the caller's
 * stream (RCCL schedules them over the xGMI links), local copies as
 * hipMemcpyAsync on the same stream. This is what replaces the reference's
 * MPI_Irecv / MPI_Isend ring and gather (src/redset_reedsolomon.c:690-694,
 * :713-733) for the multi-rank rebuild.
 *
 * RCCL is opened with dlopen on the first redset_hip_rccl_* call, so the
 * codec library itself does not need librccl: single-GPU encode / rebuild,
 * the streaming pipeline and the MPI transport load without it.
 */
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "redset_hip.h"

/* the RCCL entry points this transport uses, resolved once */
static struct {
  const char* (*GetErrorString)(ncclResult_t);
  ncclResult_t (*GroupStart)(void);
  ncclResult_t (*GroupEnd)(void);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  int ok;
  char err[200];
} rccl;
static pthread_once_t rccl_once = PTHREAD_ONCE_INIT;

static void rccl_open(void) {
  static const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"};
  void* h = NULL;
#if REDSET_HIP_TEST_KNOBS
  /* test builds: a stand-in RCCL by path (tests/rcclstub), for processes
   * where the real librccl.so.1 is already mapped (torch's) and a library
   * search would return it */
  const char* stub = getenv("REDSET_HIP_TEST_RCCL_LIBRARY");
  if (stub && stub[0]) h = dlopen(stub, RTLD_NOW | RTLD_LOCAL);
#endif
  for (size_t i = 0; i < sizeof(names) / sizeof(names[0]) && !h; ++i) h = dlopen(names[i], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    snprintf(rccl.err, sizeof(rccl.err), "RCCL transport: cannot load librccl (%s)", dlerror());
    return;
  }
#define RCCL_SYM(field, name)                                                                   \
  do {                                                                                          \
    *(void**) (&rccl.field) = dlsym(h, name);                                                   \
    if (!rccl.field) {                                                                          \
      snprintf(rccl.err, sizeof(rccl.err), "RCCL transport: librccl lacks %s", name);           \
      return;                                                                                   \
    }                                                                                           \
  } while (0)
  RCCL_SYM(GetErrorString, "ncclGetErrorString");
  RCCL_SYM(GroupStart, "ncclGroupStart");
  RCCL_SYM(GroupEnd, "ncclGroupEnd");
  RCCL_SYM(Send, "ncclSend");
  RCCL_SYM(Recv, "ncclRecv");
  RCCL_SYM(GetUniqueId, "ncclGetUniqueId");
  RCCL_SYM(CommInitRank, "ncclCommInitRank");
  RCCL_SYM(CommDestroy, "ncclCommDestroy");
#undef RCCL_SYM
  rccl.ok = 1;
}

/* REDSET_SUCCESS once RCCL is loaded, else the recorded failure */
static int rccl_load(void) {
  pthread_once(&rccl_once, rccl_open);
  return rccl.ok ? REDSET_SUCCESS : redset_hip_record_error(rccl.err);
}

struct redset_hip_rccl {
  ncclComm_t comm;
  int world, rank;
};

static int rfail(const char* what, ncclResult_t r) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s: %s", what, rccl.GetErrorString(r));
  return redset_hip_record_error(buf);
}

static int rccl_exchange(void* ctx, const redset_hip_xfer* x, int n, void* stream) {
  struct redset_hip_rccl* R = (struct redset_hip_rccl*) ctx;
  hipStream_t s = (hipStream_t) stream;
  /* a failed local copy does not skip the peers' messages (they would wait
   * in their group forever): it is reported after the group */
  int rc = 0;
  for (int i = 0; i < n; ++i) {
    if (x[i].peer != R->rank) continue;
    /* local copy: the send entry (source) is followed by its receive (destination) */
    if (!x[i].send || i + 1 >= n || x[i + 1].peer != R->rank || x[i + 1].send || x[i + 1].len != x[i].len)
      return redset_hip_record_error("rccl exchange: malformed local copy"); /* a plan bug, on every member */
    if (!rc && hipMemcpyAsync(x[i + 1].buf, x[i].buf, x[i].len, hipMemcpyDeviceToDevice, s) != hipSuccess)
      rc = redset_hip_record_error("rccl exchange: local hipMemcpyAsync failed");
    ++i;
  }
  ncclResult_t r = rccl.GroupStart();
  if (r != ncclSuccess) return rfail("ncclGroupStart", r);
  for (int i = 0; i < n; ++i) {
    if (x[i].peer == R->rank) continue;
    r = x[i].send ? rccl.Send(x[i].buf, x[i].len, ncclUint8, x[i].peer, R->comm, s)
                  : rccl.Recv(x[i].buf, x[i].len, ncclUint8, x[i].peer, R->comm, s);
    if (r != ncclSuccess) {
      (void) rccl.GroupEnd();
      return rfail(x[i].send ? "ncclSend" : "ncclRecv", r);
    }
  }
  r = rccl.GroupEnd();
  if (r != ncclSuccess) return rfail("ncclGroupEnd", r);
  return rc;
}

int redset_hip_rccl_available(void) {
  pthread_once(&rccl_once, rccl_open);
  return rccl.ok;
}

int redset_hip_rccl_unique_id(unsigned char id_out[128]) {
  ncclUniqueId id;
  if (!id_out) return redset_hip_record_error("rccl_unique_id: null argument");
  if (rccl_load() != REDSET_SUCCESS) return REDSET_FAILURE;
  ncclResult_t r = rccl.GetUniqueId(&id);
  if (r != ncclSuccess) return rfail("ncclGetUniqueId", r);
  memcpy(id_out, &id, sizeof(id) < 128 ? sizeof(id) : 128);
  return REDSET_SUCCESS;
}

int redset_hip_rccl_transport_create(const unsigned char id[128], int world, int rank, redset_hip_transport* out,
                                     redset_hip_rccl** handle) {
  if (!id || !out || !handle) return redset_hip_record_error("rccl_transport_create: null argument");
  *handle = NULL;
  if (world < 1 || rank < 0 || rank >= world) return redset_hip_record_error("rccl_transport_create: bad world/rank");
  if (rccl_load() != REDSET_SUCCESS) return REDSET_FAILURE;
  struct redset_hip_rccl* R = calloc(1, sizeof(*R));
  if (!R) return redset_hip_record_error("out of host memory");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid) < 128 ? sizeof(uid) : 128);
  ncclResult_t r = rccl.CommInitRank(&R->comm, world, uid, rank);
  if (r != ncclSuccess) {
    free(R);
    return rfail("ncclCommInitRank", r);
  }
  R->world = world;
  R->rank = rank;
  out->world = world;
  out->rank = rank;
  out->exchange = rccl_exchange;
  out->ctx = R;
  *handle = R;
  return REDSET_SUCCESS;
}

void redset_hip_rccl_transport_destroy(redset_hip_rccl* R) {
  if (!R) return;
  (void) rccl.CommDestroy(R->comm);
  free(R);
}
