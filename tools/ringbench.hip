// ringbench: does a loader-wave LDS-DMA ring move the codec's 8-read /
// 3-write stripe pattern faster than the plain VGPR sweep?
//
// Both kernels compute out[o] = xor(in[0..7]) ^ o over 16-B vectors of 64 MiB
// cells, one stripe (8 input cells, 3 output cells) per launch, 11 stripes in
// sequence like the bench's RS(8+3) encode, 512-thread blocks, one per CU.
//  kplain: every wave loads a position of the 8 inputs into VGPRs, waits,
//          combines and stores (the codec's sweep).
//  kring<L, D, S>: L loader waves stream 8 KiB items (one 1 KiB row per
//          input, 64 lanes x 16 B) with global_load_lds_dwordx4 nt into a ring
//          of S slots in LDS, keep D items in flight each and publish an item
//          behind a counted vmcnt (FULL word per slot); 8 - L consumer waves
//          read a published item with ds_read_b128, release the slot (FREE
//          word), combine and store. Consumers never wait on a store
//          acknowledgement and loaders never on arithmetic.
// Deadlock freedom: a loader drains and publishes everything it holds before
// it waits for a free slot, so every issued item is eventually published.
// Every spin is bounded (kSpinCap); a capped spin sets an error flag.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/ringbench tools/ringbench.hip
//   (-DRB_NIN=16 -DRB_NOUT=4 -DRB_BLOCK=1024: the RS(16+4) stripe at the
//   codec's block shape; the ring gets as many slots as 144 KiB of LDS hold)
// Run: ringbench [reps] [rand]
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

#ifndef RB_NIN
#define RB_NIN 8
#endif
#ifndef RB_NOUT
#define RB_NOUT 3
#endif
#ifndef RB_BLOCK
#define RB_BLOCK 512
#endif
constexpr int NIN = RB_NIN, NOUT = RB_NOUT, kBlock = RB_BLOCK, kWaves = kBlock / 64;
constexpr int kSlots = 144 / NIN > 16 ? 16 : 144 / NIN;  // slots of NIN KiB in 144 KiB
constexpr unsigned kSpinCap = 1u << 24;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gcv4;
typedef __attribute__((address_space(1))) v4u gv4;
typedef __attribute__((address_space(3))) v4u lv4;
typedef __attribute__((address_space(3))) volatile unsigned lvu;  // LDS, never flat

struct Stripe {
  gcv4* in[NIN];
  gv4* out[NOUT];
};

__device__ __forceinline__ void store_nt(gv4* p, size_t v, v4u r) { __builtin_nontemporal_store(r, p + v); }

__global__ void __launch_bounds__(kBlock) kplain(Stripe J, size_t nvec) {
  const size_t step = (size_t) gridDim.x * kBlock;
  for (size_t v = (size_t) blockIdx.x * kBlock + threadIdx.x; v < nvec; v += step) {
    v4u x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = __builtin_nontemporal_load(J.in[i] + v);
    v4u a = x[0];
#pragma unroll
    for (int i = 1; i < NIN; ++i) a ^= x[i];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) store_nt(J.out[o], v, a ^ (unsigned) o);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// flags through LDS-typed pointers: flat accesses would also count on vmcnt
__device__ __forceinline__ unsigned lds_ld(unsigned* p) { return *(lvu*) p; }
__device__ __forceinline__ void lds_st(unsigned* p, unsigned v) { *(lvu*) p = v; }

template <int L, int D, int S = kSlots>
__global__ void __launch_bounds__(kBlock) kring(Stripe J, size_t nvec, unsigned* err) {
  static_assert(L >= 1 && L < kWaves && D >= 1 && (D - 1) * L < S, "ring shape");
  constexpr int C = kWaves - L;
  __shared__ v4u ring[S * NIN * 64];
  __shared__ unsigned full[S], freed[S];
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane((int) threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t G = gridDim.x, rows = (nvec + 63) / 64;
  const size_t K = rows > blockIdx.x ? (rows - blockIdx.x + G - 1) / G : 0;  // this block's items
  auto vec_of = [&](size_t k) { return (k * G + blockIdx.x) * 64 + lane; };
  const unsigned ring0 = __builtin_amdgcn_readfirstlane((unsigned) (uintptr_t) (lv4*) ring);

  if (wave < L) {
    // loader: items k = wave, wave + L, ...; pend = items issued, not yet published
    size_t pend[D];
    int npend = 0;
    auto publish_oldest = [&]() {
      const size_t k = pend[0];
      if (lane == 0) lds_st(&full[k % S], (unsigned) (k / S) + 1);
      for (int j = 1; j < npend; ++j) pend[j - 1] = pend[j];
      --npend;
    };
    for (size_t k = wave; k < K; k += L) {
      const unsigned use = (unsigned) (k / S);
      if (lds_ld(&freed[k % S]) < use) {
        // drain and publish what we hold, then wait for the slot
        wait_vm<0>();
        while (npend > 0) publish_oldest();
        unsigned spins = 0;
        while (lds_ld(&freed[k % S]) < use) {
          if (++spins > kSpinCap) {
            if (lane == 0) atomicOr(err, 1u);
            return;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      const size_t v = vec_of(k);
      const size_t vc = v < nvec ? v : nvec - 1;
      const unsigned slot = ring0 + (unsigned) ((k % S) * NIN * 1024);
#pragma unroll
      for (int i = 0; i < NIN; ++i) {
        unsigned keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(J.in[i] + vc), "s"(slot + (unsigned) (i * 1024))
            : "memory");
      }
      pend[npend++] = k;
      if (npend == D) {
        wait_vm<((D - 1) * NIN > 63 ? 63 : (D - 1) * NIN)>();  // the oldest item has landed (D within vmcnt: see main)
        publish_oldest();
      }
    }
    wait_vm<0>();
    while (npend > 0) publish_oldest();
    return;
  }
  // consumer c: items k = c, c + C, ...
  const int c = wave - L;
  for (size_t k = c; k < K; k += C) {
    const unsigned want = (unsigned) (k / S) + 1;
    unsigned spins = 0;
    while (lds_ld(&full[k % S]) < want) {
      if (++spins > kSpinCap) {
        if (lane == 0) atomicOr(err, 2u);
        return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const lv4* s = (const lv4*) ring + (k % S) * NIN * 64;
    v4u x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = s[i * 64 + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(&freed[k % S], want);
    v4u a = x[0];
#pragma unroll
    for (int i = 1; i < NIN; ++i) a ^= x[i];
    const size_t v = vec_of(k);
    if (v < nvec) {
#pragma unroll
      for (int o = 0; o < NOUT; ++o) store_nt(J.out[o], v, a ^ (unsigned) o);
    }
  }
}

// uniform random bytes (splitmix64 of the dword index), like the bench's cells
__global__ void kfill_random(unsigned* p, size_t n, unsigned long long seed) {
  for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
    unsigned long long z = (seed + i) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (unsigned) (z ^ (z >> 31));
  }
}

__global__ void kcount_diff(const v4u* a, const v4u* b, size_t n, unsigned long long* bad) {
  unsigned long long local = 0;
  for (size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
    const v4u d = a[i] ^ b[i];
    local += (d.x | d.y | d.z | d.w) != 0;
  }
  if (local) atomicAdd(bad, local);
}

int main(int argc, char** argv) {
  const size_t cell = 64ull << 20, stride = 80ull << 20, nvec = cell / 16;
  const int nstripe = 11, reps = argc > 1 ? atoi(argv[1]) : 10;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t ncell = (size_t) nstripe * (NIN + NOUT);
  unsigned char* base = nullptr;
  CK(hipMalloc(&base, ncell * stride + NOUT * cell));  // + the reference copy of stripe 0's NOUT outputs
  CK(hipMemset(base, 0x5A, ncell * stride));
  // distinct input contents: byte pattern per cell, or (argv[2] = "rand")
  // uniform random bytes in every cell, as the codec bench uses
  const bool rnd = argc > 2 && argv[2][0] == 'r';
  for (size_t c = 0; c < ncell; ++c) {
    if (rnd) kfill_random<<<1024, 256>>>((unsigned*) (base + c * stride), cell / 4, c << 40);
    else CK(hipMemset(base + c * stride, (int) (c * 37 + 11) & 0xFF, cell / 2));
  }
  CK(hipDeviceSynchronize());
  printf("inputs: %s\n", rnd ? "uniform random" : "constant halves");
  std::vector<Stripe> js(nstripe);
  for (int s = 0; s < nstripe; ++s) {
    for (int i = 0; i < NIN; ++i) js[s].in[i] = (gcv4*) (base + ((size_t) s * (NIN + NOUT) + i) * stride);
    for (int o = 0; o < NOUT; ++o) js[s].out[o] = (gv4*) (base + ((size_t) s * (NIN + NOUT) + NIN + o) * stride);
  }
  unsigned char* ref = base + ncell * stride;
  unsigned* err = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(err, 0, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double) nstripe * (NIN + NOUT) * cell;

  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 2; ++w)
      for (int s = 0; s < nstripe; ++s) launch(js[s]);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
      for (int s = 0; s < nstripe; ++s) launch(js[s]);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    // stripe 0's outputs against the plain kernel's (the first plain run has
    // no reference yet)
    CK(hipMemset(bad, 0, 8));
    for (int o = 0; o < NOUT; ++o)
      kcount_diff<<<1024, 256>>>((const v4u*) js[0].out[o], (const v4u*) (ref + o * cell), nvec, bad);
    unsigned long long hbad = 0;
    CK(hipMemcpy(&hbad, bad, 8, hipMemcpyDeviceToHost));
    const double per = ms / (reps * nstripe);
    printf("%-16s %8.1f us/launch  %7.1f GB/s  err=%u mismatched_vectors=%llu\n", name, per * 1e3,
           bytes * reps / (ms * 1e-3) / 1e9, herr, hbad);
    fflush(stdout);
  };
  const int grid = cus;
  run("plain", [&](const Stripe& J) { kplain<<<grid, kBlock>>>(J, nvec); });
  for (int o = 0; o < NOUT; ++o) CK(hipMemcpy(ref + o * cell, (void*) js[0].out[o], cell, hipMemcpyDeviceToDevice));
  for (int round = 0; round < 2; ++round) {
    run("plain", [&](const Stripe& J) { kplain<<<grid, kBlock>>>(J, nvec); });
    run("ring L1 D2", [&](const Stripe& J) { kring<1, 2><<<grid, kBlock>>>(J, nvec, err); });
    run("ring L1 D3", [&](const Stripe& J) { kring<1, 3><<<grid, kBlock>>>(J, nvec, err); });
    if (3 * NIN <= 63) run("ring L1 D4", [&](const Stripe& J) { kring<1, 4><<<grid, kBlock>>>(J, nvec, err); });
    if (4 * NIN <= 63) run("ring L1 D5", [&](const Stripe& J) { kring<1, 5><<<grid, kBlock>>>(J, nvec, err); });
    run("ring L2 D2", [&](const Stripe& J) { kring<2, 2><<<grid, kBlock>>>(J, nvec, err); });
  }
  return 0;
}
