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
