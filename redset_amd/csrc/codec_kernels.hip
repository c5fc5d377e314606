// codec_kernels.hip -- CDNA4 (gfx950) kernels for redset's RS / XOR codec.
//
// gf_mac: out[j] = sum_i coef[j][i] * in[i] over GF(2^8)/0x11D, byte-wise.
//   Replaces the reference's e*d separate read-modify-write passes of
//   redset_rs_reduce_buffer_multadd (src/redset_reedsolomon_common.c:786-819;
//   CUDA multadd_gpu, src/redset_reedsolomon_gpu.cu:29-48) with ONE pass that
//   reads every input once and writes every output once.
//
//   Multiplication by a constant is GF(2)-linear, so c*x = c*(x & 0x0F) ^
//   c*(x & 0xF0). For every input i the block builds two 16-entry nibble
//   tables in LDS whose entries pack the products for all (<= 4) outputs into
//   one dword: T_i,h[n] = sum_j (coef[j][i] * (n << 4h)) << 8j. A byte then
//   costs two ds_read_b32 and two XORs for all outputs at once. A 16-entry
//   dword table spans 16 distinct banks, so whatever the data a wave's reads
//   of it are conflict-free (equal nibbles broadcast); no replication needed.
//   Inputs stream in as 16-B loads (1 KiB per wave instruction); the 16
//   packed accumulators are transposed back to per-output bytes with v_perm.
//
// xor_reduce: out = XOR of inputs (reference reduce_xor, src/redset_xor.c:35-42;
//   CUDA xor_gpu, src/redset_xor_gpu.cu:20-26), one pass, 16-B vectors.
#include <hip/hip_runtime.h>

#include "codec_kernels.h"

namespace redset_hip {

namespace {

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

// LDS image: [input][half][nibble] dwords = 128 B per input.
constexpr int kTableBytes = 2 * 16 * 4;

__device__ __forceinline__ void build_tables(uint32_t* lds, const GfJob& J, int nin, int nout) {
  const int entries = nin * 32;  // (input, half, nibble)
  for (int e = threadIdx.x; e < entries; e += blockDim.x) {
    const int i = e >> 5;
    const int h = (e >> 4) & 1;
    const uint32_t x = static_cast<uint32_t>(e & 15) << (4 * h);
    uint32_t v = 0;
    for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], x) << (8 * j);
    lds[e] = v;
  }
}

// v_bfe_u32 x, off, 8 -- emitted directly: hipcc rewrites a constant-offset
// extract into a shift + and, which costs one more VALU op per table lookup
template <int OFF>
__device__ __forceinline__ uint32_t byte_of(uint32_t x) {
  if constexpr (OFF == 0) {
    return x & 0xFFu;
  } else if constexpr (OFF == 24) {
    return x >> 24;
  } else {
    uint32_t r;
    asm("v_bfe_u32 %0, %1, %2, 8" : "=v"(r) : "v"(x), "i"(OFF));
    return r;
  }
}

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96); gfx950 has no
// v_xor3_b32 and hipcc does not form bitop3 from plain XORs
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// dword at byte offset `off` of the LDS image
__device__ __forceinline__ uint32_t lds_at(const uint32_t* lds, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + off);
}

// gather byte j of a[0..3] into one dword
__device__ __forceinline__ uint32_t gather_byte(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int j) {
  const uint32_t sel_lo = 0x0c0c0000u | (static_cast<uint32_t>(4 + j) << 8) | static_cast<uint32_t>(j);
  const uint32_t sel_hi = 0x00000c0cu | (static_cast<uint32_t>(4 + j) << 24) | (static_cast<uint32_t>(j) << 16);
  return __builtin_amdgcn_perm(a1, a0, sel_lo) | __builtin_amdgcn_perm(a3, a2, sel_hi);
}

template <int NIN>
__device__ __forceinline__ void gf_mac_body(const GfLaunch& L, const GfJob& J, int part) {
  // static (not extern) so the table offsets fold into ds_read's immediate
  __shared__ uint32_t lds[kMaxIn * kTableBytes / 4];
  const int nout = L.nout;

  build_tables(lds, J, NIN, nout);
  __syncthreads();

  // The job's blocks sweep its cells together, block-interleaved: at any
  // moment they cover one contiguous window of every cell, which keeps HBM
  // row locality across the ~100 concurrent cell streams (measured +8% over
  // one contiguous range per block, tools/gfbench.hip "GS").
  const size_t nvec = L.bytes_only ? 0 : L.nbytes / 16;
  const size_t vstep = static_cast<size_t>(L.blocks_per_job) * kBlock;

  const uint4* in[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) in[i] = reinterpret_cast<const uint4*>(J.in[i]);
  uint4* out[kMaxOut];
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) out[j] = reinterpret_cast<uint4*>(J.out[j]);

  // software pipeline: the next sweep position's loads are issued before
  // this one's table lookups and stores, so every lane keeps two vectors of
  // each input in flight (+4% at 4 blocks/CU, tools/gfbench.hip "PIPE")
  size_t v = static_cast<size_t>(part) * kBlock + threadIdx.x;
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
        // byte b of lo4 / hi4 = 4 * (low / high nibble of byte b) = table offset
        const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
        const uint32_t hi4 = (w[q] >> 2) & 0x3C3C3C3Cu;
        const uint32_t ol[4] = {byte_of<0>(lo4), byte_of<8>(lo4), byte_of<16>(lo4), byte_of<24>(lo4)};
        const uint32_t oh[4] = {byte_of<0>(hi4), byte_of<8>(hi4), byte_of<16>(hi4), byte_of<24>(hi4)};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, i * kTableBytes + ol[b]),
                                lds_at(lds, i * kTableBytes + 64 + oh[b]));
        }
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
        if (L.accumulate) {
          const uint4 o = out[j][v];
          r.x ^= o.x; r.y ^= o.y; r.z ^= o.z; r.w ^= o.w;
        }
        out[j][v] = r;
      }
    }
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = xn[i];
  }

  // byte path: the tail after the last whole 16-B vector, or everything when
  // some pointer is not 16-B aligned; spread over the job's blocks
  const size_t tail0 = nvec * 16;
  for (size_t k = tail0 + static_cast<size_t>(part) * kBlock + threadIdx.x; k < L.nbytes;
       k += static_cast<size_t>(L.blocks_per_job) * kBlock) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      const uint32_t b = J.in[i][k];
      acc ^= lds[i * 32 + (b & 15u)] ^ lds[i * 32 + 16 + (b >> 4)];
    }
    for (int j = 0; j < nout; ++j) {
      uint8_t r = static_cast<uint8_t>(acc >> (8 * j));
      if (L.accumulate) r ^= J.out[j][k];
      J.out[j][k] = r;
    }
  }
}

template <int NIN>
__device__ __forceinline__ void xor_body(const XorLaunch& L, const XorJob& J, int part) {
  const size_t nvec = L.bytes_only ? 0 : L.nbytes / 16;
  const size_t vstep = static_cast<size_t>(L.blocks_per_job) * kBlock;
  const uint4* in[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) in[i] = reinterpret_cast<const uint4*>(J.in[i]);
  uint4* out = reinterpret_cast<uint4*>(J.out);
  for (size_t v = static_cast<size_t>(part) * kBlock + threadIdx.x; v < nvec; v += vstep) {
    uint4 x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = in[i][v];
    uint4 r = x[0];
#pragma unroll
    for (int i = 1; i < NIN; ++i) {
      r.x ^= x[i].x; r.y ^= x[i].y; r.z ^= x[i].z; r.w ^= x[i].w;
    }
    if (L.accumulate) {
      const uint4 o = out[v];
      r.x ^= o.x; r.y ^= o.y; r.z ^= o.z; r.w ^= o.w;
    }
    out[v] = r;
  }
  const size_t tail0 = nvec * 16;
  for (size_t k = tail0 + static_cast<size_t>(part) * kBlock + threadIdx.x; k < L.nbytes;
       k += static_cast<size_t>(L.blocks_per_job) * kBlock) {
    uint8_t r = L.accumulate ? J.out[k] : 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) r ^= J.in[i][k];
    J.out[k] = r;
  }
}

// entry points: jobs from a device array (plans), or one job passed by
// value in the kernel arguments (stripe primitives, no device descriptor)
template <int NIN>
__global__ void __launch_bounds__(kBlock) gf_mac_kernel(GfLaunch L) {
  const int job = blockIdx.x / L.blocks_per_job;
  gf_mac_body<NIN>(L, L.jobs[job], blockIdx.x - job * L.blocks_per_job);
}

template <int NIN>
__global__ void __launch_bounds__(kBlock) gf_mac_kernel_arg(GfLaunch L, GfJob J) {
  gf_mac_body<NIN>(L, J, blockIdx.x);
}

template <int NIN>
__global__ void __launch_bounds__(kBlock) xor_kernel(XorLaunch L) {
  const int job = blockIdx.x / L.blocks_per_job;
  xor_body<NIN>(L, L.jobs[job], blockIdx.x - job * L.blocks_per_job);
}

template <int NIN>
__global__ void __launch_bounds__(kBlock) xor_kernel_arg(XorLaunch L, XorJob J) {
  xor_body<NIN>(L, J, blockIdx.x);
}

using GfKernel = void (*)(GfLaunch);
using XorKernel = void (*)(XorLaunch);
using GfKernelArg = void (*)(GfLaunch, GfJob);
using XorKernelArg = void (*)(XorLaunch, XorJob);

template <int... N>
struct KernelTables {
  static constexpr GfKernel gf[sizeof...(N)] = {&gf_mac_kernel<N>...};
  static constexpr XorKernel xr[sizeof...(N)] = {&xor_kernel<N>...};
  static constexpr GfKernelArg gf_arg[sizeof...(N)] = {&gf_mac_kernel_arg<N>...};
  static constexpr XorKernelArg xr_arg[sizeof...(N)] = {&xor_kernel_arg<N>...};
};
using Tables = KernelTables<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;

}  // namespace

int device_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 256;
    cus = prop.multiProcessorCount;
  }
  return cus;
}

int gf_blocks_per_cu(int nin) {
  if (nin < 1 || nin > kMaxIn) return 1;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(Tables::gf[nin - 1]), kBlock,
                                                   0) != hipSuccess ||
      n < 1)
    n = 1;
  return n;
}

int launch_gf(const GfLaunch& L, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn || L.nout < 1 || L.nout > kMaxOut) return hipErrorInvalidValue;
  if (L.njobs == 0 || L.nbytes == 0) return hipSuccess;
  const dim3 grid(static_cast<unsigned>(L.njobs * L.blocks_per_job));
  hipLaunchKernelGGL(Tables::gf[L.nin - 1], grid, dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), L);
  return hipGetLastError();
}

int launch_gf_single(const GfLaunch& L, const GfJob& J, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn || L.nout < 1 || L.nout > kMaxOut) return hipErrorInvalidValue;
  if (L.nbytes == 0) return hipSuccess;
  hipLaunchKernelGGL(Tables::gf_arg[L.nin - 1], dim3(static_cast<unsigned>(L.blocks_per_job)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), L, J);
  return hipGetLastError();
}

int launch_xor_single(const XorLaunch& L, const XorJob& J, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn) return hipErrorInvalidValue;
  if (L.nbytes == 0) return hipSuccess;
  hipLaunchKernelGGL(Tables::xr_arg[L.nin - 1], dim3(static_cast<unsigned>(L.blocks_per_job)), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), L, J);
  return hipGetLastError();
}

int launch_xor(const XorLaunch& L, void* stream) {
  if (L.nin < 1 || L.nin > kMaxIn) return hipErrorInvalidValue;
  if (L.njobs == 0 || L.nbytes == 0) return hipSuccess;
  const dim3 grid(static_cast<unsigned>(L.njobs * L.blocks_per_job));
  hipLaunchKernelGGL(Tables::xr[L.nin - 1], grid, dim3(kBlock), 0, static_cast<hipStream_t>(stream), L);
  return hipGetLastError();
}

}  // namespace redset_hip
