// streambench: HBM rate of multi-stream read/write patterns on one MI355X,
// to find what limits the codec's 8-read / 3-write stripe pattern.
// Every job reads NIN streams and writes NOUT streams of `n` bytes each
// (out[o] = xor of the inputs ^ o), grid-stride within the job like gf_mac.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/streambench tools/streambench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Job {
  const uint4* in[8];
  uint4* out[4];
};

// global (address space 1) views: global_load/store, never flat (flat ops
// also count on lgkmcnt and would tie LDS waits to HBM traffic)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gcv4;
typedef __attribute__((address_space(1))) v4u gv4;
__device__ __forceinline__ uint4 gld(const uint4* p, size_t i) {
  v4u t = ((gcv4*) p)[i];
  return make_uint4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ void gst(uint4* p, size_t i, uint4 r) {
  ((gv4*) p)[i] = v4u{r.x, r.y, r.z, r.w};
}

template <int NIN, int NOUT, int U>
__global__ void __launch_bounds__(256) kstream(const Job* jobs, size_t nvec, int bpj, size_t omask) {
  const Job J = jobs[blockIdx.x / bpj];  // by value: pointers stay in registers
  const int part = blockIdx.x % bpj;
  const size_t stride = (size_t) bpj * 256 * U;
  for (size_t v = (size_t) part * 256 * U + threadIdx.x; v < nvec; v += stride) {
    uint4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = make_uint4(0, 0, 0, 0);
    uint4 x[NIN > 0 ? NIN : 1][U];
#pragma unroll
    for (int i = 0; i < NIN; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v + u * 256 < nvec) x[i][u] = gld(J.in[i], v + u * 256);
#pragma unroll
    for (int i = 0; i < NIN; ++i)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u].x ^= x[i][u].x;
        acc[u].y ^= x[i][u].y;
        acc[u].z ^= x[i][u].z;
        acc[u].w ^= x[i][u].w;
      }
#pragma unroll
    for (int o = 0; o < NOUT; ++o)
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (v + u * 256 < nvec) {
          uint4 r = acc[u];
          r.x ^= o + (unsigned) v;
          gst(J.out[o], (v + u * 256) & omask, r);
        }
    if constexpr (NOUT == 0) {
      // keep the loads live without a store per iteration
      if ((acc[0].x ^ acc[0].y ^ acc[0].z ^ acc[0].w) == 0x9e3779b9u && v == 7) J.out[0][0] = acc[0];
    }
  }
}

// Split roles: waves 0-3 of a 512-thread block load + combine and hand the
// results to waves 4-7 through a double-buffered LDS ring; only those store.
// The loading waves then never wait on store acknowledgements (gfx9 vmcnt
// counts stores too), and the barrier is a raw s_barrier (no vmcnt drain).
template <int NIN, int NOUT>
__global__ void __launch_bounds__(512) ksplit(const Job* jobs, size_t nvec, int bpj) {
  __shared__ uint4 ring[2][NOUT][256];
  const Job J = jobs[blockIdx.x / bpj];
  const int part = blockIdx.x % bpj;
  const int t = threadIdx.x & 255;
  const bool loader = threadIdx.x < 256;
  const size_t vstep = (size_t) bpj * 256;
  const size_t T = (nvec + vstep - 1) / vstep;
  size_t v = (size_t) part * 256 + t;
  for (size_t k = 0; k < T; ++k, v += vstep) {
    const int b = k & 1;
    if (loader) {
      uint4 acc = make_uint4(0, 0, 0, 0);
      if (v < nvec) {
        uint4 x[NIN];
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[i] = gld(J.in[i], v);
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          acc.x ^= x[i].x; acc.y ^= x[i].y; acc.z ^= x[i].z; acc.w ^= x[i].w;
        }
      }
#pragma unroll
      for (int o = 0; o < NOUT; ++o) {
        uint4 r = acc;
        r.x ^= o + (unsigned) v;
        ring[b][o][t] = r;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only: LDS traffic done, vm untouched
    __builtin_amdgcn_s_barrier();
    if (!loader && v < nvec) {
#pragma unroll
      for (int o = 0; o < NOUT; ++o) gst(J.out[o], v, ring[b][o][t]);
    }
  }
}

// Interleaved cells: the NIN + NOUT cells of a job stored block-interleaved
// at granularity G vectors (cell k's block b at ((b * ncell) + k) * G), so
// one position of every cell of a stripe lies in one contiguous region.
template <int NIN, int NOUT>
__global__ void __launch_bounds__(256) kinter(uint4* const* bases, size_t nvec, int bpj, size_t G) {
  constexpr int NC = NIN + NOUT;
  const int job = blockIdx.x / bpj;
  const int part = blockIdx.x % bpj;
  const gcv4* base = (const gcv4*) bases[job];
  gv4* wbase = (gv4*) bases[job];
  const size_t stride = (size_t) bpj * 256;
  for (size_t v = (size_t) part * 256 + threadIdx.x; v < nvec; v += stride) {
    const size_t blk = v / G, off = v % G;
    v4u x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = base[(blk * NC + i) * G + off];
    v4u acc = x[0];
#pragma unroll
    for (int i = 1; i < NIN; ++i) acc ^= x[i];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) wbase[(blk * NC + NIN + o) * G + off] = acc + (unsigned) o;
  }
}

struct Arena {
  char* base;
  size_t size, used;
  void* take(size_t n) {
    size_t a = (used + 4095) & ~(size_t) 4095;
    if (a + n > size) {
      fprintf(stderr, "arena full\n");
      exit(1);
    }
    used = a + n;
    return base + a;
  }
};

template <int NIN, int NOUT, int U>
void run(const char* name, Arena& A, int njobs, size_t n, int bpc, int cus, size_t gap, size_t omask = ~(size_t) 0) {
  A.used = 0;
  std::vector<Job> h(njobs);
  for (int j = 0; j < njobs; ++j) {
    for (int i = 0; i < 8; ++i) h[j].in[i] = nullptr;
    for (int o = 0; o < 4; ++o) h[j].out[o] = nullptr;
    for (int i = 0; i < NIN; ++i) h[j].in[i] = (const uint4*) A.take(n + gap);
    for (int o = 0; o < (NOUT > 0 ? NOUT : 1); ++o) h[j].out[o] = (uint4*) A.take(n + gap);
  }
  Job* d;
  CK(hipMalloc(&d, sizeof(Job) * njobs));
  CK(hipMemcpy(d, h.data(), sizeof(Job) * njobs, hipMemcpyHostToDevice));
  size_t nvec = n / 16;
  int total = bpc * cus;
  int bpj = total / njobs;
  if (bpj < 1) bpj = 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) kstream<NIN, NOUT, U><<<bpj * njobs, 256>>>(d, nvec, bpj, omask);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) kstream<NIN, NOUT, U><<<bpj * njobs, 256>>>(d, nvec, bpj, omask);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  double bytes = (double) njobs * (NIN + NOUT) * n;
  printf("%-34s jobs=%3d in=%d out=%d U=%d bpc=%d gap=%6zu  %8.4f ms  %7.1f GB/s\n", name, njobs, NIN, NOUT, U, bpc,
         gap, ms, bytes / ms / 1e6);
  CK(hipFree(d));
}

template <int NIN, int NOUT>
void run_split(const char* name, Arena& A, int njobs, size_t n, int bpc, int cus) {
  A.used = 0;
  std::vector<Job> h(njobs);
  for (int j = 0; j < njobs; ++j) {
    for (int i = 0; i < 8; ++i) h[j].in[i] = nullptr;
    for (int o = 0; o < 4; ++o) h[j].out[o] = nullptr;
    for (int i = 0; i < NIN; ++i) h[j].in[i] = (const uint4*) A.take(n);
    for (int o = 0; o < (NOUT > 0 ? NOUT : 1); ++o) h[j].out[o] = (uint4*) A.take(n);
  }
  Job* d;
  CK(hipMalloc(&d, sizeof(Job) * njobs));
  CK(hipMemcpy(d, h.data(), sizeof(Job) * njobs, hipMemcpyHostToDevice));
  size_t nvec = n / 16;
  int bpj = bpc * cus / njobs;
  if (bpj < 1) bpj = 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  constexpr int NO = NOUT > 0 ? NOUT : 1;
  for (int w = 0; w < 3; ++w) ksplit<NIN, NO><<<bpj * njobs, 512>>>(d, nvec, bpj);
  CK(hipDeviceSynchronize());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) ksplit<NIN, NO><<<bpj * njobs, 512>>>(d, nvec, bpj);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  double bytes = (double) njobs * (NIN + NOUT) * n;
  printf("%-34s jobs=%3d in=%d out=%d bpc=%d  %8.4f ms  %7.1f GB/s\n", name, njobs, NIN, NOUT, bpc, ms,
         bytes / ms / 1e6);
  CK(hipFree(d));
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  const size_t n = (size_t) 64 << 20;
  Arena A;
  A.size = (size_t) 12 << 30;
  if (getenv("STREAMBENCH_ALLOC")) {
    // allocation-to-allocation variance: fresh allocation per round, each
    // timed twice; flags from the env (0 default, 4 = hipDeviceMallocContiguous)
    const unsigned flags = (unsigned) atoi(getenv("STREAMBENCH_ALLOC"));
    A.size = (size_t) 8 << 30;
    for (int round = 0; round < 6; ++round) {
      if (flags == 0) CK(hipMalloc(&A.base, A.size));
      else CK(hipExtMallocWithFlags((void**) &A.base, A.size, flags));
      CK(hipMemset(A.base, 0x5a, A.size));
      char name[64];
      snprintf(name, sizeof(name), "alloc %d flags %u", round, flags);
      run<8, 3, 1>(name, A, 11, n, 2, cus, 0);
      run<8, 3, 1>(name, A, 11, n, 2, cus, 0);
      run<8, 0, 1>(name, A, 11, n, 2, cus, 0);
      CK(hipFree(A.base));
    }
    return 0;
  }
  CK(hipMalloc(&A.base, A.size));
  CK(hipMemset(A.base, 0x5a, A.size));
  A.used = 0;
  printf("device %s, %d CUs, stream %zu MiB\n", prop.gcnArchName, cus, n >> 20);
  if (getenv("STREAMBENCH_SLIDE")) {
    // same layout (11 stripes x 11 cells of 64 MiB, 7.6 GiB) at different
    // offsets inside one 40 GiB allocation: does the physical region matter?
    CK(hipFree(A.base));
    const size_t G = (size_t) 1 << 30;
    char* big;
    CK(hipMalloc(&big, 40 * G));
    CK(hipMemset(big, 0x5a, 40 * G));
    for (int rep = 0; rep < 2; ++rep)
      for (size_t off = 0; off + 8 * G <= 40 * G; off += 4 * G) {
        Arena B{big + off, 8 * G, 0};
        char name[64];
        snprintf(name, sizeof(name), "8r3w at +%zu GiB", off / G);
        run<8, 3, 1>(name, B, 11, n, 2, cus, 0);
      }
    return 0;
  }
  if (getenv("STREAMBENCH_GAPS")) {
    // separate cells with a pad after each: does the relative placement of a
    // stripe's cells matter?
    const size_t M = 1 << 20;
    if (getenv("STREAMBENCH_BIG")) {
      CK(hipFree(A.base));
      A.size = (size_t) atoi(getenv("STREAMBENCH_BIG")) << 30;
      CK(hipMalloc(&A.base, A.size));
      CK(hipMemset(A.base, 0x5a, A.size));
    }
    for (int rep = 0; rep < 2; ++rep)
      for (size_t gap : {(size_t) 0, 16 * M, 32 * M, 0 * M, 16 * M, 32 * M})
        run<8, 3, 1>("8r3w cells + gap", A, 11, n, 2, cus, gap);
    return 0;
  }
  if (getenv("STREAMBENCH_INTER")) {
    const int njobs = 11;
    std::vector<uint4*> hb(njobs);
    for (int j = 0; j < njobs; ++j) hb[j] = (uint4*) (A.base + (size_t) j * 11 * n);
    uint4** db;
    CK(hipMalloc(&db, sizeof(uint4*) * njobs));
    CK(hipMemcpy(db, hb.data(), sizeof(uint4*) * njobs, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 2; ++rep) {
      run<8, 3, 1>("8r3w separate cells", A, 11, n, 2, cus, 0);
      for (size_t Gb : {(size_t) 1024, (size_t) 4096, (size_t) 16384, (size_t) 65536, (size_t) 1 << 20})
        for (int bpc : {2, 4}) {
          const size_t G = Gb / 16, nvec = n / 16;
          const int bpj = bpc * cus / njobs;
          for (int w = 0; w < 3; ++w) kinter<8, 3><<<bpj * njobs, 256>>>(db, nvec, bpj, G);
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0));
          for (int r = 0; r < 10; ++r) kinter<8, 3><<<bpj * njobs, 256>>>(db, nvec, bpj, G);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          ms /= 10;
          printf("8r3w interleaved G=%7zu B bpc=%d  %8.4f ms  %7.1f GB/s\n", Gb, bpc, ms, 11.0 * 11 * n / ms / 1e6);
        }
    }
    return 0;
  }
  if (getenv("STREAMBENCH_SPLIT")) {
    for (int rep = 0; rep < 2; ++rep)
      for (int bpc : {1, 2}) {
        run<8, 3, 1>("8r3w same waves (bpc = 256-thr)", A, 11, n, 2 * bpc, cus, 0);
        run_split<8, 3>("8r3w split roles (bpc = 512-thr)", A, 11, n, bpc, cus);
        run_split<8, 2>("8r2w split roles (bpc = 512-thr)", A, 11, n, bpc, cus);
      }
    return 0;
  }
  const size_t small = ((size_t) 1 << 20) / 16 - 1;  // 1 MiB window: stores stay in L2
  for (int rep = 0; rep < 2; ++rep)
    for (int bpc : {2, 4}) {
      run<8, 0, 1>("8r0w", A, 11, n, bpc, cus, 0);
      run<8, 1, 1>("8r1w", A, 11, n, bpc, cus, 0);
      run<8, 2, 1>("8r2w", A, 11, n, bpc, cus, 0);
      run<8, 3, 1>("8r3w", A, 11, n, bpc, cus, 0);
      run<8, 4, 1>("8r4w", A, 11, n, bpc, cus, 0);
      run<8, 1, 1>("8r1w stores into 1 MiB (L2)", A, 11, n, bpc, cus, 0, small);
      run<8, 3, 1>("8r3w stores into 1 MiB (L2)", A, 11, n, bpc, cus, 0, small);
      run<4, 3, 1>("4r3w", A, 22, n, bpc, cus, 0);
      run<0, 3, 1>("0r3w", A, 11, n, bpc, cus, 0);
    }
  CK(hipFree(A.base));
  return 0;
}
