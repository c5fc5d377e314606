/* hipstub.c -- TEST INFRASTRUCTURE ONLY. CPU stand-ins for the HIP runtime
 * calls the per-rank backends (redset_amd/csrc/rank_mpi.c) make, and for the
 * two combine entry points they call (redset_hip_gf_combine /
 * redset_hip_xor_combine, include/redset_hip.h), so that
 * tests/test_mpi_hoststub.py can run rank_test's host-MPI path -- file reads,
 * the ring exchange, scratch pool, per-call stats, writes -- on this CPU-only
 * container under LD_PRELOAD. Its output is checked against the oracle like
 * the GPU suite's. It is never built into, linked by or loaded with the
 * product libraries, and never used on a GPU box: the GPU suite
 * (tests/test_gpu_mpi.py) runs the same driver on the real runtime.
 * GF(2^8) over x^8+x^4+x^3+x^2+1, the reference's field
 * (src/redset_reedsolomon.c gf_mult_table), by shift-and-add. */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int hipGetDevice(int* d) { *d = 0; return 0; }
int hipSetDevice(int d) { (void) d; return 0; }
int hipGetDeviceCount(int* n) { *n = 1; return 0; }
int hipStreamCreateWithFlags(void** s, unsigned f) { (void) f; *s = malloc(8); return 0; }
int hipStreamCreate(void** s) { *s = malloc(8); return 0; }
int hipStreamDestroy(void* s) { free(s); return 0; }
int hipStreamSynchronize(void* s) { (void) s; return 0; }
int hipStreamWaitEvent(void* s, void* e, unsigned f) { (void) s; (void) e; (void) f; return 0; }
int hipDeviceSynchronize(void) { return 0; }
int hipHostMalloc(void** p, size_t n, unsigned f) { (void) f; *p = malloc(n ? n : 1); return *p ? 0 : 2; }
int hipHostFree(void* p) { free(p); return 0; }
int hipMalloc(void** p, size_t n) { *p = malloc(n ? n : 1); return *p ? 0 : 2; }
int hipFree(void* p) { free(p); return 0; }
int hipMemcpyAsync(void* d, const void* s, size_t n, int k, void* st) { (void) k; (void) st; memmove(d, s, n); return 0; }
int hipMemcpy(void* d, const void* s, size_t n, int k) { (void) k; memmove(d, s, n); return 0; }
int hipMemset(void* d, int v, size_t n) { memset(d, v, n); return 0; }
int hipMemsetAsync(void* d, int v, size_t n, void* st) { (void) st; memset(d, v, n); return 0; }
int hipMemcpy2DAsync(void* d, size_t dp, const void* s, size_t sp, size_t w, size_t h, int k, void* st) {
  (void) k; (void) st;
  for (size_t i = 0; i < h; ++i) memmove((char*) d + i * dp, (const char*) s + i * sp, w);
  return 0;
}
int hipEventCreateWithFlags(void** e, unsigned f) { (void) f; *e = malloc(8); return 0; }
int hipEventCreate(void** e) { *e = malloc(8); return 0; }
int hipEventRecord(void* e, void* s) { (void) e; (void) s; return 0; }
int hipEventSynchronize(void* e) { (void) e; return 0; }
int hipEventDestroy(void* e) { free(e); return 0; }
int hipDeviceGetPCIBusId(char* b, int n, int d) { snprintf(b, (size_t) n, "0000:00:00.%d", d); return 0; }
const char* hipGetErrorString(int e) { (void) e; return "hipstub"; }

static uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t) ((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
    b >>= 1;
  }
  return r;
}

int redset_hip_gf_combine(const unsigned char* const* in, int nin, unsigned char* const* out, int nout,
                          const unsigned char* coef, size_t n, int acc, void* s) {
  (void) s;
  for (int j = 0; j < nout; ++j)
    for (size_t k = 0; k < n; ++k) {
      uint8_t r = acc ? out[j][k] : 0;
      for (int i = 0; i < nin; ++i) r ^= gf_mul(coef[j * nin + i], in[i][k]);
      out[j][k] = r;
    }
  return 0;
}

int redset_hip_xor_combine(const unsigned char* const* in, int nin, unsigned char* out, size_t n, int acc,
                           void* s) {
  (void) s;
  for (size_t k = 0; k < n; ++k) {
    uint8_t r = acc ? out[k] : 0;
    for (int i = 0; i < nin; ++i) r ^= in[i][k];
    out[k] = r;
  }
  return 0;
}

/* the kernels' hang count (include/redset_hip.h redset_hip_hang_faults):
 * 0, unless HIPSTUB_HANG_RANK names this process's MPI rank (PMI_RANK), whose
 * count then moves on every read -- a hang-capped kernel wait in every call,
 * which the backends must turn into REDSET_FAILURE */
int redset_hip_hang_faults(void* s, unsigned* count, int clear) {
  static unsigned reads;
  (void) s;
  (void) clear;
  const char* want = getenv("HIPSTUB_HANG_RANK");
  const char* me = getenv("PMI_RANK");
  *count = (want && me && atoi(want) == atoi(me)) ? reads++ : 0;
  return 0;
}

/* ---- whole-set plans, on the CPU ------------------------------------------
 * The sharded exchange (sharded.c, inside libredset_hip.so) computes each
 * set through redset_hip_{rs,xor}_plan_* + redset_hip_plan_execute, which
 * launch kernels. These stand-ins keep the plan's pointers and run the same
 * arithmetic on the CPU at execute, so the per-rank backends' sharded slot
 * (rank_mpi.c sharded_slot: windows, planning, staging, exchanges) runs here
 * too. The layout maps and decode maps come from the library itself
 * (redset_hip_rs_get_encoding_id / _get_data_id / _rs_matrix /
 * _rs_decode_matrix); the bytes are checked against the oracle by the tests. */
typedef struct redset_hip_rs redset_hip_rs;
int redset_hip_rs_shape(const redset_hip_rs* rs, int* ranks, int* encoding);
int redset_hip_rs_matrix(const redset_hip_rs* rs, unsigned char* mat_out);
int redset_hip_rs_get_encoding_id(int ranks, int encoding, int rank, int chunk_id);
int redset_hip_rs_get_data_id(int ranks, int encoding, int rank, int chunk_id);
int redset_hip_rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int chunk_id,
                                unsigned char* coef_out);

enum { STUB_RS_ENCODE = 1, STUB_RS_REBUILD = 2, STUB_XOR_ENCODE = 3, STUB_XOR_REBUILD = 4, STUB_COMBINE = 5 };
/* a combine plan's job (include/redset_hip.h redset_hip_combine_job), copied */
typedef struct {
  int nin, nout, acc;
  const unsigned char** in;
  unsigned char** out;
  unsigned char* coef;
} stub_job;
struct redset_hip_plan {
  int kind, p, e, missing, lost[256];
  stub_job* jobs; /* STUB_COMBINE */
  int njobs;
  /* the coefficients, copied at plan time as the library's plans do (the
   * caller may destroy its codec while the plan lives): the encoding matrix,
   * or every stripe's decode map */
  unsigned char* coef;
  unsigned char **lofi, **par;
  size_t n, stride;
};

static int stub_plan(int kind, const redset_hip_rs* rs, int p, int e, int missing, const int* lost,
                     unsigned char* const* lofi, unsigned char* const* par, size_t n, size_t stride,
                     struct redset_hip_plan** out) {
  struct redset_hip_plan* P = calloc(1, sizeof(*P));
  if (!P) return 1;
  P->kind = kind, P->p = p, P->e = e, P->missing = missing, P->n = n, P->stride = stride;
  for (int i = 0; i < missing; ++i) P->lost[i] = lost[i];
  if (kind == STUB_RS_ENCODE) {
    P->coef = malloc((size_t) (p + e) * p);
    redset_hip_rs_matrix(rs, P->coef);
  } else if (kind == STUB_RS_REBUILD) {
    P->coef = malloc((size_t) p * missing * p);
    for (int c = 0; c < p; ++c) redset_hip_rs_decode_matrix(rs, missing, lost, c, P->coef + (size_t) c * missing * p);
  }
  P->lofi = malloc(sizeof(*P->lofi) * (size_t) p);
  P->par = malloc(sizeof(*P->par) * (size_t) p);
  for (int r = 0; r < p; ++r) P->lofi[r] = lofi[r], P->par[r] = par[r];
  *out = P;
  return 0;
}

int redset_hip_rs_plan_encode(const redset_hip_rs* rs, unsigned char* const* lofi, unsigned char* const* parity,
                              size_t chunk, size_t stride, struct redset_hip_plan** out) {
  int p, e;
  redset_hip_rs_shape(rs, &p, &e);
  return stub_plan(STUB_RS_ENCODE, rs, p, e, 0, NULL, lofi, parity, chunk, stride, out);
}
int redset_hip_rs_plan_rebuild(const redset_hip_rs* rs, int missing, const int* lost, unsigned char* const* lofi,
                               unsigned char* const* parity, size_t chunk, size_t stride,
                               struct redset_hip_plan** out) {
  int p, e;
  redset_hip_rs_shape(rs, &p, &e);
  return stub_plan(STUB_RS_REBUILD, rs, p, e, missing, lost, lofi, parity, chunk, stride, out);
}
int redset_hip_xor_plan_encode(int p, unsigned char* const* lofi, unsigned char* const* xorc, size_t chunk,
                               size_t stride, struct redset_hip_plan** out) {
  return stub_plan(STUB_XOR_ENCODE, NULL, p, 1, 0, NULL, lofi, xorc, chunk, stride, out);
}
int redset_hip_xor_plan_rebuild(int p, int root, unsigned char* const* lofi, unsigned char* const* xorc,
                                size_t chunk, size_t stride, struct redset_hip_plan** out) {
  return stub_plan(STUB_XOR_REBUILD, NULL, p, 1, 1, &root, lofi, xorc, chunk, stride, out);
}
/* redset_hip_plan_combine on the CPU: the sharded plans' partial-sum shape
 * builds its combines through it (sharded.c plan_reduce); execute runs them
 * with the stand-in gf_combine above */
typedef struct {
  int nin, nout;
  const unsigned char* const* in;
  unsigned char* const* out;
  const unsigned char* coef;
  int accumulate;
} stub_combine_job;
int redset_hip_plan_combine(const stub_combine_job* jobs, int njobs, size_t nbytes, struct redset_hip_plan** out) {
  struct redset_hip_plan* P = calloc(1, sizeof(*P));
  if (!P) return 1;
  P->kind = STUB_COMBINE;
  P->n = nbytes;
  P->jobs = calloc((size_t) (njobs > 0 ? njobs : 1), sizeof(stub_job));
  P->njobs = njobs;
  for (int k = 0; k < njobs; ++k) {
    stub_job* J = &P->jobs[k];
    J->nin = jobs[k].nin, J->nout = jobs[k].nout, J->acc = jobs[k].accumulate;
    J->in = malloc(sizeof(*J->in) * (size_t) J->nin);
    J->out = malloc(sizeof(*J->out) * (size_t) J->nout);
    J->coef = malloc((size_t) J->nin * (size_t) J->nout);
    memcpy(J->in, jobs[k].in, sizeof(*J->in) * (size_t) J->nin);
    memcpy(J->out, jobs[k].out, sizeof(*J->out) * (size_t) J->nout);
    memcpy(J->coef, jobs[k].coef, (size_t) J->nin * (size_t) J->nout);
  }
  *out = P;
  return 0;
}

void redset_hip_plan_destroy(struct redset_hip_plan* P) {
  if (!P) return;
  for (int k = 0; k < P->njobs; ++k) {
    free(P->jobs[k].in);
    free(P->jobs[k].out);
    free(P->jobs[k].coef);
  }
  free(P->jobs);
  free(P->coef);
  free(P->lofi);
  free(P->par);
  free(P);
}

/* member r's cell of stripe c (src/redset_reedsolomon_common.c:822-853;
 * XOR: src/redset_xor.c:251-266) */
static unsigned char* stub_cell(const struct redset_hip_plan* P, int r, int c) {
  if (P->kind >= STUB_XOR_ENCODE) return c == r ? P->par[r] : P->lofi[r] + (size_t) (c < r ? c : c - 1) * P->stride;
  const int enc = redset_hip_rs_get_encoding_id(P->p, P->e, r, c);
  return enc < P->p ? P->lofi[r] + (size_t) redset_hip_rs_get_data_id(P->p, P->e, r, c) * P->stride
                    : P->par[r] + (size_t) (enc - P->p) * P->stride;
}

int redset_hip_plan_execute(const struct redset_hip_plan* P, void* stream) {
  (void) stream;
  if (P->kind == STUB_COMBINE) {
    for (int k = 0; k < P->njobs; ++k) {
      const stub_job* J = &P->jobs[k];
      redset_hip_gf_combine(J->in, J->nin, J->out, J->nout, J->coef, P->n, J->acc, stream);
    }
    return 0;
  }
  const int p = P->p, e = P->e;
  const unsigned char* mat = P->coef;
  for (int c = 0; c < p; ++c) {
    if (P->kind == STUB_RS_ENCODE) { /* parity slot i of stripe c = row p + i over its data holders */
      for (int r = 0; r < p; ++r) {
        const int enc = redset_hip_rs_get_encoding_id(p, e, r, c);
        if (enc < p) continue;
        unsigned char* out = stub_cell(P, r, c);
        memset(out, 0, P->n);
        for (int s = 0; s < p; ++s) {
          if (redset_hip_rs_get_encoding_id(p, e, s, c) >= p) continue;
          const uint8_t k = mat[(size_t) enc * p + s];
          const unsigned char* in = stub_cell(P, s, c);
          for (size_t b = 0; b < P->n; ++b) out[b] ^= gf_mul(k, in[b]);
        }
      }
    } else if (P->kind == STUB_RS_REBUILD) {
      const unsigned char* D = P->coef + (size_t) c * P->missing * p;
      for (int i = 0; i < P->missing; ++i) {
        unsigned char* out = stub_cell(P, P->lost[i], c);
        memset(out, 0, P->n);
        for (int s = 0; s < p; ++s) {
          const uint8_t k = D[(size_t) i * p + s];
          if (!k) continue;
          const unsigned char* in = stub_cell(P, s, c);
          for (size_t b = 0; b < P->n; ++b) out[b] ^= gf_mul(k, in[b]);
        }
      }
    } else { /* XOR: the target of stripe c is member c's chunk (encode) or the root's cell */
      const int t = P->kind == STUB_XOR_ENCODE ? c : P->lost[0];
      unsigned char* out = stub_cell(P, t, c);
      memset(out, 0, P->n);
      for (int s = 0; s < p; ++s) {
        if (s == t) continue;
        const unsigned char* in = stub_cell(P, s, c);
        for (size_t b = 0; b < P->n; ++b) out[b] ^= in[b];
      }
    }
  }
  return 0;
}
