// gfbench.hip -- microbenchmark of gf_mac kernel variants on the bench
// workload (11 stripes x (8 inputs + 3 outputs) x 64 MiB). Standalone:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gfbench.hip -o tools/gfbench
// Prints one line per variant: avg ms, GB/s of algorithmic bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kMaxIn = 16, kMaxOut = 4;
struct Job {
  const uint8_t* in[kMaxIn];
  uint8_t* out[kMaxOut];
  uint8_t coef[kMaxOut][kMaxIn];
};

enum Mode { PROD = 0, MEMONLY = 1, FULLTAB = 2, NOOUT = 3 };

__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r ^= (b & 1u) ? a : 0u;
    b >>= 1;
    a <<= 1;
    a ^= (a & 0x100u) ? 0x11Du : 0u;
  }
  return r;
}

template <int OFF>
__device__ __forceinline__ uint32_t byte_of(uint32_t x) {
  if constexpr (OFF == 0) return x & 0xFFu;
  else if constexpr (OFF == 24) return x >> 24;
  else {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(r) : "v"(x), "i"(OFF));
    return r;
  }
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

__device__ __forceinline__ uint32_t lds_at(const uint32_t* lds, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + off);
}

__device__ __forceinline__ uint32_t gather_byte(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int j) {
  const uint32_t sel_lo = 0x0c0c0000u | (static_cast<uint32_t>(4 + j) << 8) | static_cast<uint32_t>(j);
  const uint32_t sel_hi = 0x00000c0cu | (static_cast<uint32_t>(4 + j) << 24) | (static_cast<uint32_t>(j) << 16);
  return __builtin_amdgcn_perm(a1, a0, sel_lo) | __builtin_amdgcn_perm(a3, a2, sel_hi);
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4* p) {
  if constexpr (NT) {
    v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(t.x, t.y, t.z, t.w);
  } else {
    return *p;
  }
}
template <bool NT>
__device__ __forceinline__ void st(uint4* p, uint4 v) {
  if constexpr (NT) {
    v4u t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<v4u*>(p));
  } else {
    *p = v;
  }
}

__constant__ int g_skew;
template <int NIN, int MODE, bool NT, int U, int BLOCK, bool GS = false>
__global__ void __launch_bounds__(BLOCK) kvar(const Job* jobs, size_t nvec, int bpj, int nout) {
  __shared__ uint32_t lds[MODE == FULLTAB ? NIN * 256 : NIN * 32];
  const int job = blockIdx.x / bpj;
  const int part = blockIdx.x - job * bpj;
  const Job& J = jobs[job];
  if constexpr (MODE == FULLTAB) {
    for (int e = threadIdx.x; e < NIN * 256; e += BLOCK) {
      const int i = e >> 8;
      uint32_t v = 0;
      for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], e & 255) << (8 * j);
      lds[e] = v;
    }
  } else {
    for (int e = threadIdx.x; e < NIN * 32; e += BLOCK) {
      const int i = e >> 5, h = (e >> 4) & 1;
      const uint32_t x = static_cast<uint32_t>(e & 15) << (4 * h);
      uint32_t v = 0;
      for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], x) << (8 * j);
      lds[e] = v;
    }
  }
  __syncthreads();
  // GS: the job's blocks sweep the cells together (block-interleaved), so at
  // any moment they share a contiguous window of every cell; else each block
  // owns one contiguous range
  const size_t per = GS ? nvec : (nvec + bpj - 1) / bpj;
  const size_t v0 = GS ? (size_t)part * BLOCK * U : per * part;
  const size_t v1 = GS ? nvec : ((v0 + per < nvec) ? v0 + per : nvec);
  const size_t vstep = GS ? (size_t)bpj * BLOCK * U : (size_t)BLOCK * U;
  const uint4* in[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) in[i] = reinterpret_cast<const uint4*>(J.in[i]);
  uint4* out[kMaxOut];
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) out[j] = reinterpret_cast<uint4*>(J.out[j]);

  // skew: job j starts its sweep j/njobs of the way into the cells (wraps)
  const size_t shift = g_skew ? (nvec / gridDim.x * bpj) * job : 0;
  for (size_t vb0 = v0 + threadIdx.x; vb0 < v1; vb0 += vstep) {
    size_t vb = vb0 + shift;
    if (vb >= nvec) vb -= nvec;
    uint4 x[U][NIN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t v = vb + (size_t)u * BLOCK;
#pragma unroll
      for (int i = 0; i < NIN; ++i) x[u][i] = (v < v1) ? ld<NT>(in[i] + v) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t v = vb + (size_t)u * BLOCK;
      (void)v1;
      uint32_t acc[16];
#pragma unroll
      for (int b = 0; b < 16; ++b) acc[b] = 0;
      if constexpr (MODE == MEMONLY || MODE == NOOUT) {
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          acc[0] ^= x[u][i].x; acc[1] ^= x[u][i].y; acc[2] ^= x[u][i].z; acc[3] ^= x[u][i].w;
          acc[4 + (i & 3)] ^= x[u][i].x * 3u;
        }
      } else if constexpr (MODE == FULLTAB) {
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          const uint32_t w[4] = {x[u][i].x, x[u][i].y, x[u][i].z, x[u][i].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t lo = (w[q] << 2) & 0x03FC03FCu;
            const uint32_t hi = (w[q] >> 6) & 0x03FC03FCu;
            acc[4 * q + 0] ^= lds_at(lds, i * 1024 + (lo & 0xFFFFu));
            acc[4 * q + 2] ^= lds_at(lds, i * 1024 + (lo >> 16));
            acc[4 * q + 1] ^= lds_at(lds, i * 1024 + (hi & 0xFFFFu));
            acc[4 * q + 3] ^= lds_at(lds, i * 1024 + (hi >> 16));
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          const uint32_t w[4] = {x[u][i].x, x[u][i].y, x[u][i].z, x[u][i].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
            const uint32_t hi4 = (w[q] >> 2) & 0x3C3C3C3Cu;
            const uint32_t ol[4] = {byte_of<0>(lo4), byte_of<8>(lo4), byte_of<16>(lo4), byte_of<24>(lo4)};
            const uint32_t oh[4] = {byte_of<0>(hi4), byte_of<8>(hi4), byte_of<16>(hi4), byte_of<24>(hi4)};
#pragma unroll
            for (int b = 0; b < 4; ++b)
              acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, i * 128 + ol[b]), lds_at(lds, i * 128 + 64 + oh[b]));
          }
        }
      }
      if (v < v1) {
        if constexpr (MODE == NOOUT) {
          if ((acc[0] ^ acc[5]) == 0x12345678u) out[0][v] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        } else {
#pragma unroll
          for (int j = 0; j < kMaxOut; ++j) {
            if (j < nout) {
              uint4 r;
              r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
              r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
              r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
              r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
              st<NT>(out[j] + v, r);
            }
          }
        }
      }
    }
  }
}

// plain copy / read-only references for the HBM ceiling of this pattern
__global__ void __launch_bounds__(256) kcopy(const uint4* a, uint4* b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

struct Setup {
  std::vector<Job> jobs;
  Job* d_jobs;
  size_t nvec;
  int nout;
};

template <int NIN, int MODE, bool NT, int U, int BLOCK, bool GS = false>
float run(const Setup& S, int blocks_per_cu, int cus, int reps, const char* name, double bytes) {
  const int njobs = (int)S.jobs.size();
  int bpj = (cus * blocks_per_cu) / njobs;
  if (bpj < 1) bpj = 1;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((kvar<NIN, MODE, NT, U, BLOCK, GS>), dim3(njobs * bpj), dim3(BLOCK), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((kvar<NIN, MODE, NT, U, BLOCK, GS>), dim3(njobs * bpj), dim3(BLOCK), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-44s bpc=%d blk=%4d  %8.4f ms  %8.1f GB/s\n", name, blocks_per_cu, BLOCK, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  return ms;
}


// FLAT: the whole grid sweeps job 0, then job 1, ... (vector index space is
// job-major); LDS holds every job's tables so a block can serve any job.
template <int NIN, int BLOCK>
__global__ void __launch_bounds__(BLOCK) kflat(const Job* jobs, int njobs, size_t nvec, int nout) {
  __shared__ uint32_t lds[16 * NIN * 32];
  for (int e = threadIdx.x; e < njobs * NIN * 32; e += BLOCK) {
    const int jb = e / (NIN * 32), r = e % (NIN * 32);
    const int i = r >> 5, h = (r >> 4) & 1;
    const uint32_t x = static_cast<uint32_t>(r & 15) << (4 * h);
    uint32_t v = 0;
    for (int j = 0; j < nout; ++j) v |= gf_mul_dev(jobs[jb].coef[j][i], x) << (8 * j);
    lds[e] = v;
  }
  __syncthreads();
  const size_t total = nvec * njobs;   // nvec is a multiple of BLOCK here
  for (size_t t0 = (size_t)blockIdx.x * BLOCK; t0 < total; t0 += (size_t)gridDim.x * BLOCK) {
    const int job = __builtin_amdgcn_readfirstlane((int)(t0 / nvec));
    const size_t v = t0 - (size_t)job * nvec + threadIdx.x;
    const Job& J = jobs[job];
    const uint32_t* T = lds + job * NIN * 32;
    uint4 x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = reinterpret_cast<const uint4*>(J.in[i])[v];
    uint32_t acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      const uint32_t w[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
        const uint32_t hi4 = (w[q] >> 2) & 0x3C3C3C3Cu;
        const uint32_t ol[4] = {byte_of<0>(lo4), byte_of<8>(lo4), byte_of<16>(lo4), byte_of<24>(lo4)};
        const uint32_t oh[4] = {byte_of<0>(hi4), byte_of<8>(hi4), byte_of<16>(hi4), byte_of<24>(hi4)};
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(T, i * 128 + ol[b]), lds_at(T, i * 128 + 64 + oh[b]));
      }
    }
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      if (j < nout) {
        uint4 r;
        r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
        r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
        r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
        r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
        reinterpret_cast<uint4*>(J.out[j])[v] = r;
      }
    }
  }
}

float run_flat(const Setup& S, int blocks_per_cu, int cus, int reps, double bytes) {
  const int njobs = (int)S.jobs.size();
  const int grid = cus * blocks_per_cu;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kflat<8, 256>), dim3(grid), dim3(256), 0, 0, S.d_jobs, njobs, S.nvec, S.nout);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((kflat<8, 256>), dim3(grid), dim3(256), 0, 0, S.d_jobs, njobs, S.nvec, S.nout);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-44s bpc=%d blk= 256  %8.4f ms  %8.1f GB/s\n", "prod FLAT (job-major sweep)", blocks_per_cu, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  return ms;
}


// PIPE: GS sweep with the next iteration's loads issued before this
// iteration's lookups and stores (2 vectors of every input in flight per lane)
template <int NIN, int BLOCK>
__global__ void __launch_bounds__(BLOCK) kpipe(const Job* jobs, size_t nvec, int bpj, int nout) {
  __shared__ uint32_t lds[NIN * 32];
  const int job = blockIdx.x / bpj;
  const int part = blockIdx.x - job * bpj;
  const Job& J = jobs[job];
  for (int e = threadIdx.x; e < NIN * 32; e += BLOCK) {
    const int i = e >> 5, h = (e >> 4) & 1;
    const uint32_t x = static_cast<uint32_t>(e & 15) << (4 * h);
    uint32_t v = 0;
    for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], x) << (8 * j);
    lds[e] = v;
  }
  __syncthreads();
  const uint4* in[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) in[i] = reinterpret_cast<const uint4*>(J.in[i]);
  const size_t vstep = (size_t)bpj * BLOCK;
  size_t v = (size_t)part * BLOCK + threadIdx.x;
  uint4 x[NIN];
  if (v < nvec) {
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = in[i][v];
  }
  for (; v < nvec; v += vstep) {
    const size_t vn = v + vstep;
    uint4 xn[NIN];
    if (vn < nvec) {
#pragma unroll
      for (int i = 0; i < NIN; ++i) xn[i] = in[i][vn];
    }
    uint32_t acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      const uint32_t w[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
        const uint32_t hi4 = (w[q] >> 2) & 0x3C3C3C3Cu;
        const uint32_t ol[4] = {byte_of<0>(lo4), byte_of<8>(lo4), byte_of<16>(lo4), byte_of<24>(lo4)};
        const uint32_t oh[4] = {byte_of<0>(hi4), byte_of<8>(hi4), byte_of<16>(hi4), byte_of<24>(hi4)};
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, i * 128 + ol[b]), lds_at(lds, i * 128 + 64 + oh[b]));
      }
    }
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      if (j < nout) {
        uint4 r;
        r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
        r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
        r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
        r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
        reinterpret_cast<uint4*>(J.out[j])[v] = r;
      }
    }
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = xn[i];
  }
}

float run_pipe(const Setup& S, int blocks_per_cu, int cus, int reps, double bytes) {
  const int njobs = (int)S.jobs.size();
  int bpj = (cus * blocks_per_cu) / njobs;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kpipe<8, 256>), dim3(njobs * bpj), dim3(256), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((kpipe<8, 256>), dim3(njobs * bpj), dim3(256), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-44s bpc=%d blk= 256  %8.4f ms  %8.1f GB/s\n", "prod PIPE (GS + prefetch)", blocks_per_cu, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  return ms;
}


// PIPE with buffer loads/stores carrying explicit cache-policy bits
// (aux: 1 = sc0, 2 = nt, 16 = sc1)
template <int NIN, int LAUX, int SAUX>
__global__ void __launch_bounds__(256) kpipe_aux(const Job* jobs, size_t nvec, int bpj, int nout) {
  __shared__ uint32_t lds[NIN * 32];
  const int job = blockIdx.x / bpj;
  const int part = blockIdx.x - job * bpj;
  const Job& J = jobs[job];
  for (int e = threadIdx.x; e < NIN * 32; e += 256) {
    const int i = e >> 5, h = (e >> 4) & 1;
    const uint32_t x = static_cast<uint32_t>(e & 15) << (4 * h);
    uint32_t v = 0;
    for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], x) << (8 * j);
    lds[e] = v;
  }
  __syncthreads();
  const int nrec = (int)(nvec * 16 > 0x7fffffffull ? 0x7fffffff : nvec * 16);
  __amdgpu_buffer_rsrc_t rin[NIN], rout[kMaxOut];
#pragma unroll
  for (int i = 0; i < NIN; ++i) rin[i] = __builtin_amdgcn_make_buffer_rsrc((void*)J.in[i], 0, nrec, 0x00020000);
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) rout[j] = __builtin_amdgcn_make_buffer_rsrc((void*)J.out[j], 0, nrec, 0x00020000);
  const size_t vstep = (size_t)bpj * 256;
  size_t v = (size_t)part * 256 + threadIdx.x;
  v4u x[NIN];
  if (v < nvec) {
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rin[i], (int)(v * 16), 0, LAUX);
  }
  for (; v < nvec; v += vstep) {
    const size_t vn = v + vstep;
    v4u xn[NIN];
    if (vn < nvec) {
#pragma unroll
      for (int i = 0; i < NIN; ++i) xn[i] = __builtin_amdgcn_raw_buffer_load_b128(rin[i], (int)(vn * 16), 0, LAUX);
    }
    uint32_t acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      const uint32_t w[4] = {x[i].x, x[i].y, x[i].z, x[i].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
        const uint32_t hi4 = (w[q] >> 2) & 0x3C3C3C3Cu;
        const uint32_t ol[4] = {byte_of<0>(lo4), byte_of<8>(lo4), byte_of<16>(lo4), byte_of<24>(lo4)};
        const uint32_t oh[4] = {byte_of<0>(hi4), byte_of<8>(hi4), byte_of<16>(hi4), byte_of<24>(hi4)};
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, i * 128 + ol[b]), lds_at(lds, i * 128 + 64 + oh[b]));
      }
    }
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      if (j < nout) {
        v4u r;
        r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
        r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
        r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
        r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
        __builtin_amdgcn_raw_buffer_store_b128(r, rout[j], (int)(v * 16), 0, SAUX);
      }
    }
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = xn[i];
  }
}

template <int LAUX, int SAUX>
float run_aux(const Setup& S, int blocks_per_cu, int cus, int reps, double bytes) {
  const int njobs = (int)S.jobs.size();
  int bpj = (cus * blocks_per_cu) / njobs;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((kpipe_aux<8, LAUX, SAUX>), dim3(njobs * bpj), dim3(256), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((kpipe_aux<8, LAUX, SAUX>), dim3(njobs * bpj), dim3(256), 0, 0, S.d_jobs, S.nvec, bpj, S.nout);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-30s laux=%2d saux=%2d bpc=%d  %8.4f ms  %8.1f GB/s\n", "PIPE buffer-op", LAUX, SAUX, blocks_per_cu, ms, bytes / (ms * 1e-3) / 1e9);
  fflush(stdout);
  return ms;
}

int main(int argc, char** argv) {
  const size_t C = (argc > 1 ? atol(argv[1]) : 64) << 20;
  const size_t pad = argc > 2 ? atol(argv[2]) : 0;        // bytes between consecutive cells
  const int skew = argc > 3 ? atoi(argv[3]) : 0;          // 1: jobs start their sweep at staggered offsets
  const int stripes = 11, nin = 8, nout = 3;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s, %d CUs, chunk %zu MiB\n", prop.name, cus, C >> 20);
  const size_t cstride = C + pad;
  const size_t total = (size_t)stripes * (nin + nout) * cstride;
  const int nalloc = argc > 4 ? atoi(argv[4]) : 1;
  for (int alloc = 0; alloc < nalloc; ++alloc) {
  uint8_t* buf;
  CHECK(hipMalloc(&buf, total));
  printf("== allocation %d at %p\n", alloc, (void*)buf);
  // random fill via a simple LCG kernel substitute: memset pattern then host init of a few MB is enough?
  {
    std::vector<uint8_t> h(64 << 20);
    uint64_t s = 88172645463325252ull;
    for (size_t i = 0; i < h.size(); i += 8) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      memcpy(&h[i], &s, 8);
    }
    for (size_t off = 0; off < total; off += h.size())
      CHECK(hipMemcpy(buf + off, h.data(), std::min(h.size(), total - off), hipMemcpyHostToDevice));
  }
  Setup S;
  S.nvec = C / 16;
  S.nout = nout;
  for (int c = 0; c < stripes; ++c) {
    Job J;
    memset(&J, 0, sizeof(J));
    uint8_t* base = buf + (size_t)c * (nin + nout) * cstride;
    for (int i = 0; i < nin; ++i) J.in[i] = base + (size_t)i * cstride;
    for (int j = 0; j < nout; ++j) J.out[j] = base + (size_t)(nin + j) * cstride;
    for (int j = 0; j < nout; ++j)
      for (int i = 0; i < nin; ++i) J.coef[j][i] = (uint8_t)(17 * j + 29 * i + 3);
    S.jobs.push_back(J);
  }
  CHECK(hipMalloc(&S.d_jobs, S.jobs.size() * sizeof(Job)));
  CHECK(hipMemcpy(S.d_jobs, S.jobs.data(), S.jobs.size() * sizeof(Job), hipMemcpyHostToDevice));
  const double bytes = (double)stripes * (nin + nout) * C;
  CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_skew), &skew, sizeof(int)));
  printf("cell pad %zu B, skew %d\n", pad, skew);
  const int reps = 10;

  // ceilings
  if (getenv("GFBENCH_COPY")) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const size_t n = total / 2 / 16;
    for (int g : {1024, 2048, 4096}) {
      hipLaunchKernelGGL(kcopy, dim3(g), dim3(256), 0, 0, (const uint4*)buf, (uint4*)(buf + total / 2), n);
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(a));
      for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(kcopy, dim3(g), dim3(256), 0, 0, (const uint4*)buf, (uint4*)(buf + total / 2), n);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      ms /= reps;
      printf("%-44s grid=%d  %8.4f ms  %8.1f GB/s\n", "copy (1 in -> 1 out, float4)", g, ms, (double)total / (ms * 1e-3) / 1e9);
    }
  }
  for (int round = 0; round < (getenv("GFBENCH_ROUNDS") ? atoi(getenv("GFBENCH_ROUNDS")) : 1); ++round) {
    printf("round %d\n", round);
    run<8, MEMONLY, false, 1, 256, true>(S, 2, cus, reps, "memonly GS", bytes);
    run_pipe(S, 4, cus, reps, bytes);
    run_aux<0, 0>(S, 4, cus, reps, bytes);
    run_aux<2, 0>(S, 4, cus, reps, bytes);
    run_aux<0, 2>(S, 4, cus, reps, bytes);
    run_aux<0, 19>(S, 4, cus, reps, bytes);
    run_aux<2, 19>(S, 4, cus, reps, bytes);
    run_aux<0, 17>(S, 4, cus, reps, bytes);
    run_aux<16, 0>(S, 4, cus, reps, bytes);
  }
  }  // allocations (kept live so each one gets new physical pages)
  return 0;
}
