// codec_device.h -- CDNA4 (gfx950) kernels for redset's RS / XOR codec.
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
//
// Kernel templates only; every codec_sets_*.hip instantiates them for a
// range of input counts (split so the instantiations compile in parallel)
// and exposes them through a KernelSet table (codec_kernels.h).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "codec_kernels.h"

// 0 (default): plain sweep -- load a position of every input, wait,
// combine, store. 1: the software-pipelined sweep below. Measured A/B on one
// box (bench.py RS(8+3), tools/ab_bench.sh, profiles/r01_ab_pipeline.txt):
// plain 5.02 TB/s at 2 blocks/CU, pipelined 4.82; the HBM side prefers fewer
// requests in flight (2 blocks/CU beat 3 and 4 for both), so the extra
// prefetch only adds DRAM row contention.
#ifndef REDSET_PIPELINE
#define REDSET_PIPELINE 0
#endif
// 1: timing-only build with the GF arithmetic replaced by XOR (never shipped)
#ifndef REDSET_MEMONLY
#define REDSET_MEMONLY 0
#endif
// Table offsets of the GF lookups: 0 = packed shift + mask, then one extract
// per offset (12 VALU ops per input dword); 1 (default) = one SDWA-byte-select
// AND per offset (10 ops); 2 = SDWA only in kernels with <= 2 outputs. Round
// 1 measured 2 best (+1.9% on the RS step; SDWA cost the 3-output encode
// 0.6%, profiles/r01_ab_sdwa_offsets.txt) -- while every lookup also paid a
// v_add of the tables' LDS base. With the tables at the bottom of LDS
// (gf_mac_body), 1 is ahead: +0.7% encode, +0.6% step over 2
// (profiles/r03_ab_tables_first.txt).
#ifndef REDSET_SDWA_OFFSETS
#define REDSET_SDWA_OFFSETS 1
#endif
// knob 2: the SDWA parts (sdwa_parts) of the kernels with > 2 outputs
#ifndef REDSET_SDWA_WIDE_PARTS
#define REDSET_SDWA_WIDE_PARTS 0
#endif
// Cache policy of the cell streams. Every cell byte is read or written
// exactly once, so both directions are marked non-temporal (`nt`): +3% on
// the RS step and +7% on XOR against the default policy, while either one
// alone gains nothing (nt loads alone lose 2%) -- profiles/r01_ab_cache_policy.txt.
// A/B knobs (tools/build_ab_variant.sh): stores 0 = default, 1 = nt; loads
// 0 = default, 1 = nt. (Round 1 also tried sc0/sc1 variants as inline-asm
// stores; with the ring kernels those builds failed the bench's round trip,
// profiles/r03_ab_cache_policy.txt -- the compiler does not protect an asm
// store's data registers -- so they are gone.)
#ifndef REDSET_STORE_POLICY
#define REDSET_STORE_POLICY 1
#endif
#if REDSET_STORE_POLICY != 0 && REDSET_STORE_POLICY != 1
#error "REDSET_STORE_POLICY: 0 (default) or 1 (nt)"
#endif
#ifndef REDSET_LOAD_POLICY
#define REDSET_LOAD_POLICY 1
#endif

// Register budget of the kernels: N > 0 compiles them for at most N waves
// per SIMD (amdgpu_waves_per_eu), i.e. up to 512 / N VGPRs; 0 lets the
// compiler aim for 4 waves (<= 128 VGPRs). The codec runs one block per CU,
// so the default -- the block's own waves per SIMD (4 for the ring's 1024
// threads, 2 for the plain sweep's 512) -- costs no occupancy; for the plain
// sweep it lets gf_mac<8,3> issue all 8 input loads of a position before its
// first wait (+1.0% on the RS step, profiles/r01_ab_waves_per_eu.txt).
#ifndef REDSET_WAVES_PER_EU
#define REDSET_WAVES_PER_EU (REDSET_BLOCK / 256)
#endif
// LDS-DMA input ring (A/B knob, 0 = off): every wave streams its inputs
// with global_load_lds_dwordx4 into a private ring of REDSET_GLDS stages in
// LDS (no VGPR destination, no barrier), waits for the oldest stage with a
// counted vmcnt and reads it back with ds_read_b128; stores as the plain
// sweep. Stages shrink to fit kGldsLdsBudget for wide NIN.
#ifndef REDSET_GLDS
#define REDSET_GLDS 0
#endif
// Wave priority (A/B knob, 0 = off): 1 raises s_setprio while a wave issues
// its loads, 2 while it computes and stores, 3 = 1 for gf_mac with >= 3
// outputs and for xor, 2 for gf_mac with <= 2 outputs.
#ifndef REDSET_SETPRIO
#define REDSET_SETPRIO 0
#endif
constexpr int sweep_prio(int nout) { return REDSET_SETPRIO == 3 ? (nout >= 3 ? 1 : 2) : REDSET_SETPRIO; }

#if REDSET_WAVES_PER_EU > 0
#define REDSET_KERNEL __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, REDSET_WAVES_PER_EU)))
#else
#define REDSET_KERNEL __global__ void __launch_bounds__(kBlock)
#endif

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

// LDS image per input: the low-nibble table (16 dwords, entry n at byte 4n)
// then the high-nibble table at kHiBase with entries kHiStride bytes apart.
// Stride 16 makes byte k of (w & 0xF0F0F0F0) the high table's offset as is,
// one op per input dword fewer than (w >> 2) & 0x3C3C3C3C, but measured 2.8%
// slower on the rebuild (profiles/r01_ab_sdwa_offsets.txt), so 4 stays (A/B
// knob; both strides keep the 16 entries in 16 distinct LDS banks).
// REDSET_HI_B64 = 1: high-nibble entries 16 B apart (offset = byte & 0xF0,
// one SDWA op and no shift) read with ds_read_b64, whose banks are (a/4) mod
// 64, so the 16 entries stay conflict-free (as ds_read_b32 they would pair
// up 2-way); the upper dword is unused.
#ifndef REDSET_HI_B64
#define REDSET_HI_B64 0
#endif
#if REDSET_HI_B64
#undef REDSET_HI_STRIDE
#define REDSET_HI_STRIDE 16
#endif
#ifndef REDSET_HI_STRIDE
#define REDSET_HI_STRIDE 4
#endif
constexpr int kHiStride = REDSET_HI_STRIDE;
constexpr int kHiBase = 16 * 4;
constexpr int kTableBytes = kHiBase + 16 * kHiStride;

__device__ __forceinline__ void build_tables(uint32_t* lds, const GfJob& J, int nin, int nout) {
  const int entries = nin * 32;  // (input, half, nibble)
  for (int e = threadIdx.x; e < entries; e += blockDim.x) {
    const int i = e >> 5;
    const int h = (e >> 4) & 1;
    const int n = e & 15;
    const uint32_t x = static_cast<uint32_t>(n) << (4 * h);
    uint32_t v = 0;
    for (int j = 0; j < nout; ++j) v |= gf_mul_dev(J.coef[j][i], x) << (8 * j);
    const int off = i * kTableBytes + (h ? kHiBase + n * kHiStride : n * 4);
    *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + off) = v;
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

// 4 * (nibble of byte B of x >> or << 2) in one VALU op: v_and_b32 with an
// SDWA byte select on x (x = w << 2: low nibble of byte B of w; x = w >> 2:
// its high nibble), 60 = 0x3C keeps the four nibble bits at offset 2
// which table offsets a kernel with `nout` outputs computes by SDWA:
// bit 0 = low-nibble offsets, bit 1 = high-nibble offsets
constexpr int sdwa_parts(int nout) {
  return REDSET_SDWA_OFFSETS == 1 ? 3 : REDSET_SDWA_OFFSETS == 2 ? (nout <= 2 ? 3 : REDSET_SDWA_WIDE_PARTS) : 0;
}

// byte B of x & mask (an SGPR) in one op, the same SDWA form
template <int B>
__device__ __forceinline__ uint32_t byte_and(uint32_t x, uint32_t mask) {
  uint32_t r;
  asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%3"
      : "=v"(r)
      : "s"(mask), "v"(x), "i"(B));
  return r;
}

template <int B>
__device__ __forceinline__ uint32_t nibble_offset(uint32_t x) {
  uint32_t r;
  asm("v_and_b32_sdwa %0, 60, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_%2"
      : "=v"(r)
      : "v"(x), "i"(B));
  return r;
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

// high-nibble table entry at byte offset `off` (REDSET_HI_B64: a 64-bit read)
__device__ __forceinline__ uint32_t lds_hi_at(const uint32_t* lds, uint32_t off) {
#if REDSET_HI_B64
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const volatile u2 lds_u2;
  // volatile: a plain read whose upper half is unused is narrowed to ds_read_b32
  return ((lds_u2*) (reinterpret_cast<const char*>(lds) + off))->x;
#else
  return lds_at(lds, off);
#endif
}

// gather byte j of a[0..3] into one dword
__device__ __forceinline__ uint32_t gather_byte(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int j) {
  const uint32_t sel_lo = 0x0c0c0000u | (static_cast<uint32_t>(4 + j) << 8) | static_cast<uint32_t>(j);
  const uint32_t sel_hi = 0x00000c0cu | (static_cast<uint32_t>(4 + j) << 24) | (static_cast<uint32_t>(j) << 16);
  return __builtin_amdgcn_perm(a1, a0, sel_lo) | __builtin_amdgcn_perm(a3, a2, sel_hi);
}

// Global-address-space views of the cell pointers: loads and stores through
// them are global_load/store (vmcnt only), not flat ones, which would also
// count on lgkmcnt and make every LDS table wait drain the HBM prefetch.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;

// NOUT and ACC are compile-time so that every loop iteration issues a fixed
// sequence of memory instructions (NIN prefetch loads, [NOUT accumulate
// loads], NOUT stores): the compiler can then wait for exactly the loads it
// needs with a counted vmcnt instead of vmcnt(0), which is what lets the next
// position's loads stay in flight behind this position's arithmetic and
// stores (vmcnt counts stores too on gfx9).
template <int NIN>
__device__ __forceinline__ void load_vec(v4u (&x)[NIN], g_cu4* const (&in)[NIN], size_t v) {
#pragma unroll
  for (int i = 0; i < NIN; ++i) {
#if REDSET_LOAD_POLICY == 1
    x[i] = __builtin_nontemporal_load(in[i] + v);
#else
    x[i] = in[i][v];
#endif
  }
}

// one 16-B store of an output stream
__device__ __forceinline__ void store_vec(g_u4* p, size_t v, v4u r) {
#if REDSET_STORE_POLICY == 1
  __builtin_nontemporal_store(r, p + v);
#else
  p[v] = r;
#endif
}

// acc (packed partial products of all outputs, 16 bytes) ^= coef[.][i] * x;
// SDWA: table offsets by SDWA byte selects (see REDSET_SDWA_OFFSETS)
// TB: byte offset of the tables in LDS (a constant, so it folds into the
// ds_read immediate like the input's own offset; the streamed kernels keep
// two jobs' tables, TB selects one)
template <int SDWA, int TB = 0>
__device__ __forceinline__ void gf_acc_input(const uint32_t* lds, const v4u& x, int i, uint32_t (&acc)[16]) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t ol[4], oh[4];
    if constexpr ((SDWA & 1) != 0) {
      // one SDWA op per table offset instead of 1.5
      const uint32_t wl = w[q] << 2;
      ol[0] = nibble_offset<0>(wl), ol[1] = nibble_offset<1>(wl), ol[2] = nibble_offset<2>(wl);
      ol[3] = nibble_offset<3>(wl);
    } else {
      // byte b of lo4 = 4 * (low nibble of byte b) = table offset
      const uint32_t lo4 = (w[q] << 2) & 0x3C3C3C3Cu;
      ol[0] = byte_of<0>(lo4), ol[1] = byte_of<8>(lo4), ol[2] = byte_of<16>(lo4), ol[3] = byte_of<24>(lo4);
    }
    if constexpr ((SDWA & 2) != 0) {
      if constexpr (kHiStride == 16) {
        oh[0] = byte_and<0>(w[q], 0xF0u), oh[1] = byte_and<1>(w[q], 0xF0u), oh[2] = byte_and<2>(w[q], 0xF0u);
        oh[3] = byte_and<3>(w[q], 0xF0u);
      } else {
        const uint32_t wh = w[q] >> 2;
        oh[0] = nibble_offset<0>(wh), oh[1] = nibble_offset<1>(wh), oh[2] = nibble_offset<2>(wh);
        oh[3] = nibble_offset<3>(wh);
      }
    } else {
      const uint32_t hi4 = kHiStride == 16 ? (w[q] & 0xF0F0F0F0u) : ((w[q] >> 2) & 0x3C3C3C3Cu);
      oh[0] = byte_of<0>(hi4), oh[1] = byte_of<8>(hi4), oh[2] = byte_of<16>(hi4), oh[3] = byte_of<24>(hi4);
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, TB + i * kTableBytes + ol[b]),
                            lds_hi_at(lds, TB + i * kTableBytes + kHiBase + oh[b]));
    }
  }
}

// transpose the packed accumulators back to per-output bytes and store
template <int NOUT, bool ACC>
__device__ __forceinline__ void gf_finish(const uint32_t (&acc)[16], g_u4* const (&out)[NOUT], size_t v, bool store) {
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    v4u r;
    r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
    r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
    r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
    r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
    if constexpr (ACC) {
      if (store) out[j][v] = r ^ out[j][v];
    } else {
      store_vec(out[j], v, r);
    }
  }
}

// out[j][v] (^)= sum_i coef[j][i] * x[i] for one 16-B position of every cell
template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_vec(const uint32_t* lds, const v4u (&x)[NIN], g_u4* const (&out)[NOUT],
                                           size_t v, bool store) {
#if REDSET_MEMONLY
  // timing-only build (A/B of the arithmetic's cost): same loads and stores,
  // XOR instead of GF products -- results are wrong by design
  v4u m = x[0];
#pragma unroll
  for (int i = 1; i < NIN; ++i) m ^= x[i];
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
    if constexpr (ACC) {
      if (store) out[j][v] = m ^ out[j][v];
    } else {
      store_vec(out[j], v, m + j);  // the real kernel's store policy
    }
  }
  return;
#endif
  uint32_t acc[16];
#pragma unroll
  for (int b = 0; b < 16; ++b) acc[b] = 0;
#pragma unroll
  for (int i = 0; i < NIN; ++i) gf_acc_input<sdwa_parts(NOUT)>(lds, x[i], i, acc);
  gf_finish<NOUT, ACC>(acc, out, v, store);
}

template <int NIN, bool ACC>
__device__ __forceinline__ void xor_vec(const v4u (&x)[NIN], g_u4* out, size_t v, bool store) {
  v4u r = x[0];
#pragma unroll
  for (int i = 1; i < NIN; ++i) r ^= x[i];
  if constexpr (ACC) {
    if (store) out[v] = r ^ out[v];
  } else {
    store_vec(out, v, r);
  }
}

// Incremental forms of gf_mac_vec / xor_vec for the loader ring's consumers
// (ring_sweep): begin(), then add<I0>(x) for inputs [I0, I0 + N) of one
// 16-B position, then finish(v) stores it. A consumer of a wide stripe adds
// its inputs in chunks so that only one chunk is live in VGPRs.
template <int NOUT, bool ACC>
struct GfAcc {
  const uint32_t* lds;
  g_u4* out[NOUT];
#if REDSET_MEMONLY
  v4u m;  // timing-only build: XOR instead of GF products (wrong by design)
  __device__ __forceinline__ void begin() { m = v4u{0, 0, 0, 0}; }
  template <int I0, int N, int TB = 0>
  __device__ __forceinline__ void add(const v4u (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) m ^= x[i];
  }
  __device__ __forceinline__ void finish(size_t v) {
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      if constexpr (ACC) out[j][v] = m ^ out[j][v];
      else store_vec(out[j], v, m + j);
    }
  }
#else
  uint32_t acc[16];
  __device__ __forceinline__ void begin() {
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0;
  }
  template <int I0, int N, int TB = 0>
  __device__ __forceinline__ void add(const v4u (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) gf_acc_input<sdwa_parts(NOUT), TB>(lds, x[i], I0 + i, acc);
  }
  __device__ __forceinline__ void finish(size_t v) {
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      v4u r;
      r.x = gather_byte(acc[0], acc[1], acc[2], acc[3], j);
      r.y = gather_byte(acc[4], acc[5], acc[6], acc[7], j);
      r.z = gather_byte(acc[8], acc[9], acc[10], acc[11], j);
      r.w = gather_byte(acc[12], acc[13], acc[14], acc[15], j);
      if constexpr (ACC) out[j][v] = r ^ out[j][v];
      else store_vec(out[j], v, r);
    }
  }
#endif
};

template <bool ACC>
struct XorAcc {
  g_u4* out;
  v4u r;
  __device__ __forceinline__ void begin() { r = v4u{0, 0, 0, 0}; }
  template <int I0, int N>
  __device__ __forceinline__ void add(const v4u (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) r ^= x[i];
  }
  __device__ __forceinline__ void finish(size_t v) {
    if constexpr (ACC) out[v] = r ^ out[v];
    else store_vec(out, v, r);
  }
};

// The vector sweep shared by gf_mac and xor_reduce. The job's blocks sweep
// its cells together, block-interleaved: at any moment they cover one
// contiguous window of every cell, which keeps HBM row locality across the
// ~100 concurrent cell streams (+8% over one contiguous range per block,
// tools/gfbench.hip "GS").
//
// Software pipeline, unrolled by two over ping-pong register sets: the next
// position's NIN loads are issued before this position's arithmetic and
// stores, and nothing copies registers between the sets, so the compiler
// waits for exactly the older loads (a counted vmcnt) and the prefetch stays
// in flight behind the stores (gfx9's vmcnt counts stores too). Every lane
// runs the same scalar trip count; positions past the end work on the last
// vector instead (clamped loads, and a store of the value that position
// already holds), so each iteration issues a fixed instruction sequence, the
// waits can count the stores, and the body is emitted only twice. Bodies get
// (position, in_range); only an accumulating body must skip out-of-range
// stores, since re-applying its XOR would not be idempotent.
//
// `prime(position)` runs once after the first loads: a non-accumulating body
// stores zeros to the position its first step will overwrite, so the loop is
// entered with the same loads-then-stores sequence in flight as on the back
// edge and the compiler's waits in the first half count the stores too.
template <int NIN, int PRIO, typename Body, typename Prime>
__device__ __forceinline__ void sweep(g_cu4* const (&in)[NIN], size_t nvec, size_t vstep, int part, Body body,
                                      Prime prime) {
#if !REDSET_PIPELINE
  // plain sweep: load, wait, combine, store
  (void) prime;
  for (size_t v = static_cast<size_t>(part) * kBlock + threadIdx.x; v < nvec; v += vstep) {
    v4u x[NIN];
    if constexpr (PRIO == 1) {
      // a wave issues its loads at raised priority
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(2);
      load_vec<NIN>(x, in, v);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      load_vec<NIN>(x, in, v);
    }
    if constexpr (PRIO == 2) {
      // the arithmetic and stores run at raised priority
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(2);
      body(x, v, true);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
    } else {
      body(x, v, true);
    }
  }
  return;
#endif
  const size_t last = nvec - 1;
  const size_t pairs = (nvec + 2 * vstep - 1) / (2 * vstep);
  size_t v = static_cast<size_t>(part) * kBlock + threadIdx.x;
  v4u xa[NIN], xb[NIN];
  load_vec<NIN>(xa, in, v < nvec ? v : last);
  prime(v < nvec ? v : last);
  for (size_t k = 0; k < pairs; ++k) {
    const size_t vb = v + vstep;
    load_vec<NIN>(xb, in, vb < nvec ? vb : last);
    // keep the prefetch ahead of the arithmetic that waits on xa
    __builtin_amdgcn_sched_barrier(0);
    body(xa, v < nvec ? v : last, v < nvec);
    const size_t va = vb + vstep;
    load_vec<NIN>(xa, in, va < nvec ? va : last);
    __builtin_amdgcn_sched_barrier(0);
    body(xb, vb < nvec ? vb : last, vb < nvec);
    v = va;
  }
}

#if REDSET_GLDS
constexpr int kWavesPerBlock = kBlock / 64;
constexpr int kGldsLdsBudget = 144 * 1024;
// stages of the ring for NIN inputs: REDSET_GLDS, fewer if the ring would
// not fit (1 = no overlap inside the wave)
template <int NIN>
constexpr int glds_stages() {
  int st = REDSET_GLDS;
  while (st > 1 && st * NIN * 1024 * kWavesPerBlock > kGldsLdsBudget) --st;
  return st;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until the stage issued `a` load groups and `b` store groups ago has
// landed: vmcnt counts loads, LDS-DMA and stores together, in issue order
template <int NIN, int NOUT, int A, int B>
__device__ __forceinline__ void wait_stage_ab() {
  wait_vm<A * NIN + B * NOUT>();
}
template <int NIN, int NOUT, int S>
__device__ __forceinline__ void wait_stage(int a, int b) {
  static_assert(S >= 1 && S <= 3, "ring depth");
  if constexpr (S == 1) {
    wait_vm<0>();
  } else if constexpr (S == 2) {
    if (a == 1) {
      if (b == 1) wait_stage_ab<NIN, NOUT, 1, 1>(); else wait_stage_ab<NIN, NOUT, 1, 0>();
    } else {
      if (b == 1) wait_stage_ab<NIN, NOUT, 0, 1>(); else wait_stage_ab<NIN, NOUT, 0, 0>();
    }
  } else {
    switch (a * 3 + b) {
      case 0: wait_stage_ab<NIN, NOUT, 0, 0>(); break;
      case 1: wait_stage_ab<NIN, NOUT, 0, 1>(); break;
      case 2: wait_stage_ab<NIN, NOUT, 0, 2>(); break;
      case 3: wait_stage_ab<NIN, NOUT, 1, 0>(); break;
      case 4: wait_stage_ab<NIN, NOUT, 1, 1>(); break;
      case 5: wait_stage_ab<NIN, NOUT, 1, 2>(); break;
      case 6: wait_stage_ab<NIN, NOUT, 2, 0>(); break;
      case 7: wait_stage_ab<NIN, NOUT, 2, 1>(); break;
      default: wait_stage_ab<NIN, NOUT, 2, 2>(); break;
    }
  }
}

typedef __attribute__((address_space(3))) v4u l_u4;

// The wave's positions: base + k * vstep + lane, k < iters. Stage k's NIN
// loads go to ring slot k % S; position clamped to the last vector (its
// store skipped) for lanes past the end.
template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_glds_sweep(const uint32_t* tables, l_u4* ring, g_cu4* const (&in)[NIN],
                                                  g_u4* const (&out)[NOUT], size_t nvec, size_t vstep, size_t base) {
  constexpr int S = glds_stages<NIN>();
  const int lane = threadIdx.x & 63;
  if (base >= nvec) return;
  const size_t last = nvec - 1;
  const int iters = static_cast<int>((nvec - base + vstep - 1) / vstep);
  // inline asm, not __builtin_amdgcn_global_load_lds: hipcc treats the
  // builtin as an LDS write on vmcnt and drains vmcnt(0) before the next
  // ds_read of ANY ring slot, which would serialise the stages; asm LDS-DMA
  // is invisible to its wait bookkeeping, so wait_stage counts it instead
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ring)));
  auto issue = [&](int k) {
    const size_t v = base + static_cast<size_t>(k) * vstep + lane;
    const size_t vc = v < nvec ? v : last;
    const uint32_t slot = ring0 + static_cast<uint32_t>((k % S) * NIN * 1024);
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      uint32_t keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
#if REDSET_LOAD_POLICY == 1
          " nt"
#endif
          "\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(in[i] + vc), "s"(slot + static_cast<uint32_t>(i * 1024))
          : "memory");
    }
  };
  for (int k = 0; k < S - 1 && k < iters; ++k) issue(k);
  for (int k = 0; k < iters; ++k) {
    if (k + S - 1 < iters) issue(k + S - 1);
    // load groups issued after stage k, store groups issued after it
    const int a = (S - 1) < (iters - 1 - k) ? (S - 1) : (iters - 1 - k);
    const int b = k < (S - 1) ? k : (S - 1);
    wait_stage<NIN, NOUT, S>(a, b);
    const l_u4* slot = ring + (k % S) * NIN * 64;
    v4u x[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) x[i] = slot[i * 64 + lane];
    const size_t v = base + static_cast<size_t>(k) * vstep + lane;
    gf_mac_vec<NIN, NOUT, ACC>(tables, x, out, v < nvec ? v : last, v < nvec);
  }
}
#endif

#if REDSET_RING
// Loader-wave LDS-DMA ring (shape per kernel below: D items in flight, R
// rows per item). Wave 0 of the block is the loader: it streams items -- R
// 1 KiB rows (64 lanes x 16 B) of every input -- with global_load_lds_dwordx4 into a
// ring of S slots in LDS and publishes an item (FULL word of its slot) once
// a counted vmcnt says it has landed. The other waves (15 at the default
// 1024 threads) consume items in turn:
// wait for FULL, ds_read_b128 their lane's 16 B of each input, release the
// slot (FREE word), combine and store. A consumer never waits on HBM loads or
// on a store acknowledgement behind them, the loader never on arithmetic.
// Deadlock freedom: before the loader waits for a free slot it drains and
// publishes every item it holds, so every issued item is eventually
// published and consumed.
//
// The ring is only staging: every spin is bounded (kRingSpinCap polls) and
// a capped spin never costs correctness. A consumer whose FULL wait caps
// loads its lane's 16 B of each input straight from HBM (and releases the
// slot); a loader whose FREE wait caps stops streaming without touching the
// busy slot and raises the block's BYPASS word, after which every item it
// has not published is loaded directly by its consumer. Each capped spin
// adds 1 to the launch's fault word (redset_hip_ring_faults()): a
// performance event, not an error. Capped spins did happen once, from a
// missing barrier between the jobs of an in-kernel job loop (round 2,
// profiles/r02s62_gpu_tests_ring_fault.log, fixed at the top of ring_sweep);
// a build with -DREDSET_RING_SPIN_CAP=4 drives both fallbacks on every
// launch and is checked bit for bit (tests/test_gpu_ring_fallback.py).
// LDS for the ring's slots (the GF tables take 2 KiB more): 144 KiB gives
// wide stripes a slot more (16 inputs: 9 instead of 8), +0.9% on RS(16+4);
// stripes of <= 8 inputs keep 16 slots (profiles/r03_ring_depth_sweep.txt)
#ifndef REDSET_RING_KIB
#define REDSET_RING_KIB 144
#endif
// 1: a loader that finds its next slot busy first drains and publishes
// what it holds (A/B knob; 0 = spin on the slot with its items pending)
#ifndef REDSET_RING_DRAIN
#define REDSET_RING_DRAIN 1
#endif
constexpr int kRingBudget = REDSET_RING_KIB * 1024;
// Ring shape per kernel: R = 64-vector rows of every input per item, D =
// items the loader keeps in flight (ring_depth below). gf_mac: 1 row (the
// consumers' GF math sets part of the pace; two-row items cost 3%). XOR: 2
// rows (+3-4% over 1 row; profiles/r02_ab_ring_rows.txt).
#ifndef REDSET_RING_GF_ROWS
#define REDSET_RING_GF_ROWS 1
#endif
#ifndef REDSET_RING_XOR_ROWS
#define REDSET_RING_XOR_ROWS 2
#endif
// D is picked so that about F 1 KiB rows are pending behind the item being
// published: D - 1 = round(F / (NIN * R)), at most REDSET_RING_MAX_DEPTH items.
// F = 16, except 20 for the one-row items of xor past 8 inputs (light
// consumers; with two-row items 16 stays best). Measured on one
// box for every width 1-16 against fixed D = 2, 3, 4, 6, 9 (profiles/
// r03_ring_depth_sweep.txt): the rule is best or within run-to-run noise
// (~2%) everywhere -- RS(8+3): 8 inputs, D = 3; XOR p = 8: 7 inputs x 2
// rows, D = 2 -- and gains on narrow stripes against round 2's fixed depths:
// GF 2 / 4 inputs +37% / +17%, XOR 3 inputs +27%. REDSET_RING_FIXED_DEPTH > 0
// overrides (A/B).
#ifndef REDSET_RING_ROWS_IN_FLIGHT
#define REDSET_RING_ROWS_IN_FLIGHT 16
#endif
#ifndef REDSET_RING_XOR_ROWS_IN_FLIGHT
#define REDSET_RING_XOR_ROWS_IN_FLIGHT 20
#endif
#ifndef REDSET_RING_MAX_DEPTH
#define REDSET_RING_MAX_DEPTH 9
#endif
#ifndef REDSET_RING_FIXED_DEPTH
#define REDSET_RING_FIXED_DEPTH 0
#endif
// XOR kernels with more inputs than this use the one-row GF shape (A/B knob)
#ifndef REDSET_RING_XOR_WIDE
#define REDSET_RING_XOR_WIDE 8
#endif
// s_sleep argument (x 64 clocks) between a consumer's polls of a FULL word:
// polls take issue slots from the co-resident consumers that are computing
// (~17% of the LDS instructions at 1, profiles/r02s60_ring_pmc_lds.txt);
// 8 measured +0.9% on the RS step, rebuild +1.5-2% (4 and 16 alike;
// profiles/r02_ab_ring_sleep.txt)
#ifndef REDSET_RING_SLEEP
#define REDSET_RING_SLEEP 8
#endif
// s_setprio of the loader wave (A/B knob, 0 = same priority as consumers)
#ifndef REDSET_RING_LOADER_PRIO
#define REDSET_RING_LOADER_PRIO 0
#endif
#ifndef REDSET_RING_MAX_SLOTS
#define REDSET_RING_MAX_SLOTS 16
#endif
template <int NIN>
constexpr int ring_slots() {
  return kRingBudget / (NIN * 1024) > REDSET_RING_MAX_SLOTS ? REDSET_RING_MAX_SLOTS : kRingBudget / (NIN * 1024);
}
// polls before a handshake gives up on the ring (A/B and test knob: a
// tiny cap exercises the direct-load fallbacks on every launch)
#ifndef REDSET_RING_SPIN_CAP
#define REDSET_RING_SPIN_CAP (1u << 24)
#endif
constexpr unsigned kRingSpinCap = REDSET_RING_SPIN_CAP;
// Waits that end by construction and have no fallback (the streamed kernels'
// table hand-over and a position's claim): their cap is only insurance
// against a hang from a bug, counted like a capped spin, and independent of
// the test knob above (a capped table wait would use another job's tables).
constexpr unsigned kRingHangCap = 1u << 26;
// Inputs a ring consumer holds in VGPRs at once; wider stripes are combined in
// two chunks (ring_sweep). A/B knob.
#ifndef REDSET_RING_CHUNK
#define REDSET_RING_CHUNK 8
#endif
constexpr int kRingChunk = REDSET_RING_CHUNK;
// items the loader keeps in flight for NIN inputs of R-row items (see
// REDSET_RING_ROWS_IN_FLIGHT), within the ring's slots and vmcnt's 6 bits
template <int NIN, int R, int F>
constexpr int ring_depth() {
  constexpr int rows = NIN * R;
  int d = REDSET_RING_FIXED_DEPTH > 0 ? REDSET_RING_FIXED_DEPTH : 1 + (F + rows / 2) / rows;
  if (REDSET_RING_FIXED_DEPTH == 0 && d > REDSET_RING_MAX_DEPTH) d = REDSET_RING_MAX_DEPTH;
  if (d > ring_slots<rows>()) d = ring_slots<rows>();
  while (d > 1 && (d - 1) * rows > 63) --d;
  return d < 2 ? 2 : d;
}
typedef __attribute__((address_space(3))) v4u lr_u4;
typedef __attribute__((address_space(3))) volatile unsigned lr_flag;  // LDS, never flat
__device__ __forceinline__ unsigned ring_flag_ld(unsigned* p) { return *(lr_flag*) p; }
__device__ __forceinline__ void ring_flag_st(unsigned* p, unsigned v) { *(lr_flag*) p = v; }
// A loader publishes an item: lane 0 writes its FULL word (0), or (A/B knob
// REDSET_RING_PUBLISH_ALL=1) every lane writes the same value, which spares the
// exec-mask juggling of a one-lane write
#ifndef REDSET_RING_PUBLISH_ALL
#define REDSET_RING_PUBLISH_ALL 0
#endif
__device__ __forceinline__ void ring_publish(unsigned* p, unsigned v, int lane) {
#if REDSET_RING_PUBLISH_ALL
  (void) lane;
  ring_flag_st(p, v);
#else
  if (lane == 0) ring_flag_st(p, v);
#endif
}
template <int N>
__device__ __forceinline__ void ring_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// A consumer's fallback load of one input vector, complete on return: the
// load and its wait are one asm block, so the compiler never sees a VMEM
// load pending into the registers the ring path fills with ds_read (it would
// otherwise put an s_waitcnt vmcnt(0) -- a wait for this consumer's stores --
// in front of every ring read). The wait drains the wave's stores too, which
// only the rare fallback pays.
__device__ __forceinline__ v4u ring_direct_load(g_cu4* p) {
  v4u r;
  asm volatile("global_load_dwordx4 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=&v"(r) : "v"(p) : "memory");
  return r;
}

// Item k of this block covers vectors (k * G + part) * 64 + lane; `body`
// (GfAcc / XorAcc: begin, add<I0>(inputs), finish(v)) combines and stores one
// in-range vector position.
// LDS the ring of a kernel with NIN inputs and R-row items occupies (v4u)
template <int NIN, int R>
constexpr int ring_vecs() {
  return ring_slots<NIN * R>() * NIN * R * 64;
}

// `ring` is LDS storage of ring_vecs<NIN, R>() vectors, declared by the
// caller (gf_mac puts its GF tables in front of it, see gf_mac_body).
template <int NIN, int R, int D, typename Body>
__device__ __forceinline__ void ring_sweep(v4u* ring, g_cu4* const (&in)[NIN], size_t nvec, size_t G, size_t part,
                                           unsigned* fault, Body& body) {
  constexpr int S = ring_slots<NIN * R>();
  static_assert(D >= 1 && D - 1 < S && (D - 1) * NIN * R <= 63, "ring depth");
  constexpr int C = kBlock / 64 - 1;
  static_assert(C >= 1, "a consumer wave");
  __shared__ unsigned full[S], freed[S], bypass;
  // every wave has left the ring's previous use (a kernel looping over jobs
  // calls this once per job: the loader finishes a job first and must not
  // reset flags that consumers of that job still poll)
  __syncthreads();
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  if (threadIdx.x == 0) bypass = 0;
  __syncthreads();
  // Nothing the compiler knows of may be in flight when the loops start: its
  // wait insertion merges the state at a loop's entry into the loop, so a
  // load or store still pending here (job descriptor, tables, a previous
  // job's stores) whose registers the loader loop reuses puts a vmcnt(0)
  // into that loop -- every item then waits for all earlier LDS-DMA loads
  // (the loader's pipelining gone, a launch 60% slower; it happened to an
  // instrumented build). This wait, which the compiler does see, clears it.
  __builtin_amdgcn_s_waitcnt(0);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  const size_t rows = (nvec + 63) / 64;
  const size_t items = (rows + R - 1) / R;
  const size_t K = items > part ? (items - part + G - 1) / G : 0;
  // vector of row r of item k in this block
  auto vec_of = [&](size_t k, int r) { return ((k * G + part) * R + r) * 64 + lane; };
  if (wave == 0) {
    if constexpr (REDSET_RING_LOADER_PRIO > 0) __builtin_amdgcn_s_setprio(REDSET_RING_LOADER_PRIO);
    const uint32_t ring0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lr_u4*) ring)));
    // items [pub, k) are issued and not yet published
    size_t pub = 0;
    auto publish = [&]() {
      ring_publish(&full[pub % S], static_cast<unsigned>(pub / S) + 1, lane);
      ++pub;
    };
    for (size_t k = 0; k < K; ++k) {
      const unsigned use = static_cast<unsigned>(k / S);
      if (ring_flag_ld(&freed[k % S]) < use) {
#if REDSET_RING_DRAIN
        ring_wait_vm<0>();
        while (pub < k) publish();
#endif
        unsigned spins = 0;
        while (ring_flag_ld(&freed[k % S]) < use && ++spins < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
        if (spins >= kRingSpinCap) {
          // a consumer still holds the slot: leave it alone, hand every item
          // not yet published to its consumer's direct loads, and stop
          ring_wait_vm<0>();
          while (pub < k) publish();
          if (lane == 0) {
            ring_flag_st(&bypass, 1u);
            if (fault) atomicAdd(fault, 1u);
          }
          return;
        }
      }
      const uint32_t slot = ring0 + static_cast<uint32_t>((k % S) * NIN * R * 1024);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const size_t v = vec_of(k, r);
        const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          uint32_t keep;
          asm volatile(
              "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
#if REDSET_LOAD_POLICY == 1
              " nt"
#endif
              "\n\ts_mov_b32 m0, %0"
              : "=&s"(keep)
              : "v"(in[i] + vc), "s"(slot + static_cast<uint32_t>((i * R + r) * 1024))
              : "memory");
        }
      }
      if (k + 1 - pub == static_cast<size_t>(D)) {
        ring_wait_vm<(D - 1) * NIN * R>();  // the oldest pending item has landed
        publish();
      }
    }
    ring_wait_vm<0>();
    while (pub < K) publish();
    return;
  }
  for (size_t k = wave - 1; k < K; k += C) {
    const unsigned want = static_cast<unsigned>(k / S) + 1;
    unsigned spins = 0;
    bool direct = false;
    while (ring_flag_ld(&full[k % S]) < want) {
      if (ring_flag_ld(&bypass) != 0u || ++spins >= kRingSpinCap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
    }
    if (direct) {
      // the item never arrived in time (or the loader stopped): take this
      // lane's bytes from HBM; the ring copy, if it ever lands, is unread.
      // Release the slot for item k + S only after item k - S's consumer
      // has (FREE = want - 1), or the loader could overwrite a slot that
      // consumer still reads; if that never happens the loader's own capped
      // wait raises BYPASS.
      if (spins >= kRingSpinCap && lane == 0 && fault) atomicAdd(fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[k % S]) + 1u < want && ++s2 < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
      if (lane == 0 && ring_flag_ld(&freed[k % S]) + 1u >= want) ring_flag_st(&freed[k % S], want);
    }
    const lr_u4* sl = (const lr_u4*) ring + (k % S) * NIN * R * 64;
    // inputs [I0, I0 + N) of row r into x, from the slot or from HBM
    auto fetch = [&](auto i0, auto& x, int r) {
      constexpr int I0 = decltype(i0)::value;
      constexpr int N = sizeof(x) / sizeof(x[0]);
      if (!direct) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = sl[((I0 + i) * R + r) * 64 + lane];
      } else {
        const size_t v = vec_of(k, r);
        const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = ring_direct_load(in[I0 + i] + vc);
      }
    };
    auto release = [&]() {
      if (!direct) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) ring_flag_st(&freed[k % S], want);
      }
    };
    if constexpr (NIN <= kRingChunk) {
      // the whole item in VGPRs: the slot is free before the arithmetic
      v4u x[R][NIN];
#pragma unroll
      for (int r = 0; r < R; ++r) fetch(std::integral_constant<int, 0>{}, x[r], r);
      release();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const size_t v = vec_of(k, r);
        if (v < nvec) {
          body.begin();
          body.template add<0>(x[r]);
          body.finish(v);
        }
      }
    } else {
      // wide stripe: two chunks, so only one is live in VGPRs (all NIN inputs
      // plus the accumulators would spill past the 128 VGPRs of a 1024-thread
      // block); the slot is held while the first chunk is combined
      static_assert(R == 1, "wide stripes use one-row items");
      body.begin();
      {
        v4u x[kRingChunk];
        fetch(std::integral_constant<int, 0>{}, x, 0);
        body.template add<0>(x);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep chunk 1's reads behind chunk 0's arithmetic
      {
        v4u x[NIN - kRingChunk];
        fetch(std::integral_constant<int, kRingChunk>{}, x, 0);
        release();
        body.template add<kRingChunk>(x);
      }
      const size_t v = vec_of(k, 0);
      if (v < nvec) body.finish(v);
    }
  }
}
#endif

// One static LDS array per input count, the GF tables first and the loader
// ring behind them: the tables' addresses (< 2 KiB) then fold into ds_read's
// 16-bit immediate offset, so a lookup's address is the table offset alone. As
// two arrays the compiler put the 128 KiB ring first, and every lookup paid a
// v_add of the tables' base (0x20000) -- 4 of ~20 VALU ops per input dword.
// (A function-scope static: gf_mac_body and gf_mac_stream share it, where two
// arrays would each get their own LDS.)
constexpr int kTableVecs = kMaxIn * kTableBytes / 16;
template <int NIN>
__device__ __forceinline__ v4u* gf_lds() {
#if REDSET_RING
  constexpr int kRingVecs = ring_vecs<NIN, REDSET_RING_GF_ROWS>();
#else
  constexpr int kRingVecs = 0;
#endif
  __shared__ v4u smem[kTableVecs + kRingVecs];
  return smem;
}

template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_body(const GfLaunch& L, const GfJob& J, int part) {
  v4u* const smem = gf_lds<NIN>();
  uint32_t* const lds = reinterpret_cast<uint32_t*>(smem);

  build_tables(lds, J, NIN, NOUT);
  __syncthreads();

  const size_t nvec = L.bytes_only ? 0 : L.nbytes / 16;
  const size_t vstep = static_cast<size_t>(L.blocks_per_job) * kBlock;
  if (nvec > 0) {
    g_cu4* in[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (J.in[i]);
    g_u4* out[NOUT];
#pragma unroll
    for (int j = 0; j < NOUT; ++j) out[j] = (g_u4*) (J.out[j]);
#if REDSET_RING
    GfAcc<NOUT, ACC> body;
    body.lds = lds;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) body.out[j] = out[j];
    constexpr int kDepth = ring_depth<NIN, REDSET_RING_GF_ROWS, REDSET_RING_ROWS_IN_FLIGHT>();
    ring_sweep<NIN, REDSET_RING_GF_ROWS, kDepth>(smem + kTableVecs, in, nvec, static_cast<size_t>(L.blocks_per_job),
                                                 static_cast<size_t>(part), L.fault, body);
#elif REDSET_GLDS
    __shared__ v4u ring_mem[glds_stages<NIN>() * NIN * 64 * kWavesPerBlock];
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    l_u4* ring = (l_u4*) (ring_mem) + wave * glds_stages<NIN>() * NIN * 64;
    gf_mac_glds_sweep<NIN, NOUT, ACC>(lds, ring, in, out, nvec, vstep,
                                      static_cast<size_t>(part) * kBlock + static_cast<size_t>(wave) * 64);
#else
    sweep<NIN, sweep_prio(NOUT)>(
        in, nvec, vstep, part,
        [&](const v4u (&x)[NIN], size_t v, bool st) { gf_mac_vec<NIN, NOUT, ACC>(lds, x, out, v, st); },
        [&](size_t v) {
          if constexpr (!ACC) {
#pragma unroll
            for (int j = 0; j < NOUT; ++j) out[j][v] = v4u{0, 0, 0, 0};
          }
        });
#endif
  }

  // byte path: the tail after the last whole 16-B vector, or everything when
  // some pointer is not 16-B aligned; spread over the job's blocks
  const size_t tail0 = nvec * 16;
  for (size_t k = tail0 + static_cast<size_t>(part) * kBlock + threadIdx.x; k < L.nbytes; k += vstep) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
      const uint32_t b = J.in[i][k];
      acc ^= lds_at(lds, i * kTableBytes + (b & 15u) * 4) ^ lds_at(lds, i * kTableBytes + kHiBase + (b >> 4) * kHiStride);
    }
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      uint8_t r = static_cast<uint8_t>(acc >> (8 * j));
      if constexpr (ACC) r ^= J.out[j][k];
      J.out[j][k] = r;
    }
  }
}

#if REDSET_RING
// kJobsStreamed (codec_kernels.h): one launch, every block streams its items
// of ALL the launch's jobs (stripes) through one continuous loader ring --
// job 0's items, then job 1's, ... -- so a block that finishes its share of
// a stripe goes straight on to the next stripe's: no launch gap and no
// per-stripe tail (the edges of a launch idle 3.5% of its CU time and
// launches sit 2.5 us apart, profiles/r03_block_clock.txt), and no ring
// drain between stripes. The GF tables of two jobs live in the table region
// (NIN <= 8: 2 x NIN x 128 B <= 2 KiB), job j's in buffer j & 1; the loader
// wave builds job j's tables when it reaches job j's first item, once every
// consumer is past job j - 2's items (prog[], the next item each consumer
// takes), and announces them in tab_job. Consumers pick the buffer by a
// branch over two copies of the arithmetic, so the tables' offsets still
// fold into the ds_read immediates. Deadlock freedom: a consumer waits only
// on FULL (capped: direct loads) and on tab_job; the loader's wait on prog
// needs only items of jobs <= j - 2, whose tables exist, so it always ends.
// Same staging rules as ring_sweep (capped FULL/FREE waits, BYPASS).
// Host side: only for whole 16-B vectors (!bytes_only, nbytes % 16 == 0)
// and NIN <= 8 (redset_hip.cpp).
template <int NIN, int NOUT>
__device__ __forceinline__ void build_tables_wave(uint32_t* lds, int tb, const __attribute__((address_space(4))) GfJob* J,
                                                  int lane) {
  // lanes 0-31: input i2, lanes 32-63: input i2 + 1; lane & 31 = (half, nibble);
  // the coefficients are wave-uniform (scalar loads, nothing on vmcnt)
  const int h = (lane >> 4) & 1;
  const int n = lane & 15;
  const uint32_t x = static_cast<uint32_t>(n) << (4 * h);
  // coefficient rows as dwords: byte loads would be vector loads, whose waits
  // (vmcnt) would also drain the loader's LDS-DMA queue
  typedef __attribute__((address_space(4))) const uint32_t c_u32;
  uint32_t cw[NOUT][(NIN + 3) / 4];
#pragma unroll
  for (int j = 0; j < NOUT; ++j)
#pragma unroll
    for (int q = 0; q < (NIN + 3) / 4; ++q) cw[j][q] = ((c_u32*) &J->coef[j][0])[q];
  auto coef = [&](int j, int i) { return (cw[j][i >> 2] >> (8 * (i & 3))) & 0xFFu; };
#pragma unroll
  for (int i2 = 0; i2 < NIN; i2 += 2) {
    const int i = i2 + (lane >> 5);
    if (i < NIN) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < NOUT; ++j) {
        const uint32_t c0 = coef(j, i2);
        const uint32_t c1 = (i2 + 1 < NIN) ? coef(j, i2 + 1) : 0u;
        v |= gf_mul_dev((lane >> 5) ? c1 : c0, x) << (8 * j);
      }
      const int off = tb + i * kTableBytes + (h ? kHiBase + n * kHiStride : n * 4);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + off) = v;
    }
  }
}

template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_stream(const GfLaunch& L) {
  static_assert(NIN <= 8 && 2 * NIN * kTableBytes <= kTableVecs * 16, "two jobs' tables in the table region");
  static_assert(REDSET_RING_GF_ROWS == 1, "one-row items");
  constexpr int S = ring_slots<NIN>();
  constexpr int D = ring_depth<NIN, 1, REDSET_RING_ROWS_IN_FLIGHT>();
  constexpr int C = kBlock / 64 - 1;
  constexpr int kTab = NIN * kTableBytes;  // one job's tables (bytes)
  static_assert(D >= 2 && D - 1 < S && (D - 1) * NIN <= 63, "ring depth");
  typedef __attribute__((address_space(4))) const GfJob c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  v4u* const smem = gf_lds<NIN>();
  uint32_t* const lds = reinterpret_cast<uint32_t*>(smem);
  v4u* const ring = smem + kTableVecs;
  __shared__ unsigned full[S], freed[S], bypass, tab_job, prog[C];

  const size_t nvec = L.nbytes / 16;
  const size_t G = gridDim.x;
  const size_t part = blockIdx.x;
  const size_t rows = (nvec + 63) / 64;
  const unsigned K = rows > part ? static_cast<unsigned>((rows - part + G - 1) / G) : 0u;
  const unsigned njobs = static_cast<unsigned>(L.njobs);
  const unsigned total = K * njobs;
  if (K == 0) return;  // uniform over the block: no work here

  // job 0's tables into buffer 0 (the whole block), flags
  for (int e = threadIdx.x; e < NIN * 32; e += blockDim.x) {
    const int i = e >> 5, h = (e >> 4) & 1, n = e & 15;
    const uint32_t x = static_cast<uint32_t>(n) << (4 * h);
    uint32_t v = 0;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) v |= gf_mul_dev(jobs[0].coef[j][i], x) << (8 * j);
    lds[(i * kTableBytes + (h ? kHiBase + n * kHiStride : n * 4)) / 4] = v;
  }
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  if (threadIdx.x < C) prog[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0) bypass = 0, tab_job = 0;
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);  // see ring_sweep
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  auto vec_of = [&](unsigned k) { return (static_cast<size_t>(k) * G + part) * 64 + lane; };

  if (wave == 0) {
    if constexpr (REDSET_RING_LOADER_PRIO > 0) __builtin_amdgcn_s_setprio(REDSET_RING_LOADER_PRIO);
    const uint32_t ring0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lr_u4*) ring)));
    unsigned pub = 0;  // items [pub, g) are issued and not yet published
    auto publish = [&]() {
      ring_publish(&full[pub % S], pub / S + 1, lane);
      ++pub;
    };
    // every consumer's next item is >= T (all items before T are done)
    auto past = [&](unsigned T) {
      const bool ok = lane >= C || ring_flag_ld(&prog[lane]) >= T;
      return __builtin_amdgcn_ballot_w64(!ok) == 0;
    };
    // job j's tables into buffer j & 1, once every consumer is past job
    // j - 2; if they are not yet, first publish every item issued (with
    // fewer items per job than in flight, some may be job j - 2's)
    auto next_tables = [&](unsigned j, unsigned g) {
      if (j >= 2 && !past((j - 1) * K)) {
        ring_wait_vm<0>();
        while (pub < g) publish();
        // always ends (see above); the cap only keeps a bug from hanging the
        // GPU -- a capped wait is counted and every test checks the count
        unsigned spins = 0;
        while (!past((j - 1) * K) && ++spins < kRingHangCap) __builtin_amdgcn_s_sleep(1);
        if (spins >= kRingHangCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
      }
      build_tables_wave<NIN, NOUT>(lds, (j & 1) * kTab, jobs + j, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) ring_flag_st(&tab_job, j);
    };
    const uint8_t* in[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) in[i] = jobs[0].in[i];
    unsigned job = 0, k = 0;
    for (unsigned g = 0; g < total; ++g, ++k) {
      if (k == K) {
        k = 0;
        ++job;
        next_tables(job, g);
#pragma unroll
        for (int i = 0; i < NIN; ++i) in[i] = jobs[job].in[i];
      }
      const unsigned use = g / S;
      if (ring_flag_ld(&freed[g % S]) < use) {
#if REDSET_RING_DRAIN
        ring_wait_vm<0>();
        while (pub < g) publish();
#endif
        unsigned spins = 0;
        while (ring_flag_ld(&freed[g % S]) < use && ++spins < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
        if (spins >= kRingSpinCap) {
          // as in ring_sweep: publish what is issued, hand the rest to the
          // consumers' direct loads -- but keep building the tables they need
          ring_wait_vm<0>();
          while (pub < g) publish();
          if (lane == 0) {
            ring_flag_st(&bypass, 1u);
            if (L.fault) atomicAdd(L.fault, 1u);
          }
          for (unsigned j = job + 1; j < njobs; ++j) next_tables(j, g);
          return;
        }
      }
      const uint32_t slot = ring0 + (g % S) * NIN * 1024;
      const size_t v = vec_of(k);
      const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
      for (int i = 0; i < NIN; ++i) {
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
#if REDSET_LOAD_POLICY == 1
            " nt"
#endif
            "\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"((g_cu4*) (in[i]) + vc), "s"(slot + static_cast<uint32_t>(i * 1024))
            : "memory");
      }
      if (g + 1 - pub == static_cast<unsigned>(D)) {
        ring_wait_vm<(D - 1) * NIN>();
        publish();
      }
    }
    ring_wait_vm<0>();
    while (pub < total) publish();
    return;
  }

  // consumers: items c, c + C, ... of the block's sequence
  const int c = wave - 1;
  GfAcc<NOUT, ACC> body;
  body.lds = lds;
  g_cu4* in[NIN];
  int cur = -1;
  unsigned job = static_cast<unsigned>(c) / K, k = static_cast<unsigned>(c) % K;
  for (unsigned g = c; g < total; g += C) {
    if (static_cast<int>(job) != cur) {
      cur = static_cast<int>(job);
      unsigned spins = 0;  // always ends; capped as the loader's wait above
      while (ring_flag_ld(&tab_job) < job && ++spins < kRingHangCap) __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
      if (spins >= kRingHangCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
#pragma unroll
      for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (jobs[job].in[i]);
#pragma unroll
      for (int j = 0; j < NOUT; ++j) body.out[j] = (g_u4*) (jobs[job].out[j]);
    }
    const unsigned want = g / S + 1;
    unsigned spins = 0;
    bool direct = false;
    while (ring_flag_ld(&full[g % S]) < want) {
      if (ring_flag_ld(&bypass) != 0u || ++spins >= kRingSpinCap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
    }
    const size_t v = vec_of(k);
    v4u x[NIN];
    if (!direct) {
      const lr_u4* sl = (const lr_u4*) ring + (g % S) * NIN * 64;
#pragma unroll
      for (int i = 0; i < NIN; ++i) x[i] = sl[i * 64 + lane];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) ring_flag_st(&freed[g % S], want);
    } else {
      // as in ring_sweep
      if (spins >= kRingSpinCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[g % S]) + 1u < want && ++s2 < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
      if (lane == 0 && ring_flag_ld(&freed[g % S]) + 1u >= want) ring_flag_st(&freed[g % S], want);
      const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
      for (int i = 0; i < NIN; ++i) x[i] = ring_direct_load(in[i] + vc);
    }
    if (v < nvec) {
      body.begin();
      if (job & 1) body.template add<0, NIN, kTab>(x);
      else body.template add<0, NIN, 0>(x);
      body.finish(v);
    }
    // this item's lookups are done (finish used their results): its job's
    // table buffer may be rebuilt once every consumer says so
    if (lane == 0) ring_flag_st(&prog[c], g + C);
    k += C;
    while (k >= K) k -= K, ++job;
  }
  if (lane == 0) ring_flag_st(&prog[c], 0xFFFFFFFFu);
}
#endif

#if REDSET_RING
// Slow, table-free product of one 16-B position (the claimed kernel's last
// resort, for items whose tables may not exist: see gf_mac_claimed): a dword
// at a time, bytes multiplied in parallel within it (shift-and-add with the
// 0x11D reduction per byte), loops kept rolled so that it adds few registers
// to the consumer loop it sits in
__device__ __forceinline__ uint32_t gf_mul_bytes(uint32_t c, uint32_t x) {
  uint32_t r = 0;
#pragma unroll 1
  for (int b = 0; b < 8; ++b) {
    if ((c >> b) & 1u) r ^= x;
    x = ((x & 0x7F7F7F7Fu) << 1) ^ (((x >> 7) & 0x01010101u) * 0x1Du);
  }
  return r;
}
template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_vec_slow(const __attribute__((address_space(4))) GfJob* J, g_cu4* const (&in)[NIN],
                                                size_t v) {
#pragma unroll 1
  for (int j = 0; j < NOUT; ++j) {
    uint32_t* o = reinterpret_cast<uint32_t*>(J->out[j]) + 4 * v;
#pragma unroll 1
    for (int w = 0; w < 4; ++w) {
      uint32_t r = 0;
#pragma unroll 1
      for (int i = 0; i < NIN; ++i)
        r ^= gf_mul_bytes(J->coef[j][i], reinterpret_cast<const uint32_t*>(J->in[i])[4 * v + w]);
      o[w] = ACC ? (o[w] ^ r) : r;
    }
  }
}

// items per claim, and batches the claimer keeps claimed ahead of the loader
#ifndef REDSET_CLAIM_BATCH
#define REDSET_CLAIM_BATCH 4
#endif
#ifndef REDSET_CLAIM_LOOK
#define REDSET_CLAIM_LOOK 2
#endif
// kJobsClaimed: gf_mac_stream's continuous ring over all the launch's jobs,
// with the items claimed at run time. The rows of every job are dealt to 8
// queues (row % 8; block b serves queue b % 8, i.e. one queue per XCD, as the
// static mapping deals rows to XCDs; one queue if the grid is not a multiple
// of 8); the blocks of a queue claim batches of B consecutive items with a
// returning atomic on the queue's counter, so they sweep the XCD's rows in
// order together and finish together: no block runs ahead into the next
// stripe (gf_mac_stream's drift: all 11 stripes in one launch lost 3.5%,
// profiles/r03_ab_stream.txt) and none idles at the end of a stripe.
// Queue item u: job u / RQ, row (u % RQ) * nq + q, RQ = ceil(rows / nq) rounded
// up to B (a batch never spans two jobs; rows past the end are skipped).
// Wave 1 is the claimer: it keeps up to kLook batches claimed ahead of the
// loader (bbase[], nclaimed; its atomic's wait stalls only itself -- in the
// loader a returning atomic would drain the LDS-DMA queue with vmcnt(0)).
// Ring position p holds item bbase[(p / B) % NB] + p % B. Waves 2-15 consume.
// bbase[] entries are not overwritten before every position of their batch
// was released (NB * B >= S + (kLook + 1) * B). Fallbacks (capped waits): a
// consumer loads an unpublished position straight from HBM; a capped loader
// stops (BYPASS), the claimer stops, the consumers finish the claimed
// batches and then claim batches themselves, computing without tables where
// the loader never built them (gf_mac_vec_slow). Capped waits are counted.
// The last block to finish zeroes the counters for the next launch.
template <int NIN, int NOUT, bool ACC>
__device__ __forceinline__ void gf_mac_claimed(const GfLaunch& L) {
  static_assert(NIN <= 8 && 2 * NIN * kTableBytes <= kTableVecs * 16, "two jobs' tables in the table region");
  static_assert(REDSET_RING_GF_ROWS == 1, "one-row items");
  constexpr int S = ring_slots<NIN>();
  constexpr int D = ring_depth<NIN, 1, REDSET_RING_ROWS_IN_FLIGHT>();
  constexpr int C = kBlock / 64 - 2;  // consumer waves
  constexpr int kTab = NIN * kTableBytes;
  constexpr unsigned B = REDSET_CLAIM_BATCH;
  constexpr unsigned kLook = REDSET_CLAIM_LOOK;
  constexpr unsigned NB = 32;
  static_assert(C >= 1 && NB * B >= S + (kLook + 1) * B, "batch ring");
  typedef __attribute__((address_space(4))) const GfJob c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  v4u* const smem = gf_lds<NIN>();
  uint32_t* const lds = reinterpret_cast<uint32_t*>(smem);
  v4u* const ring = smem + kTableVecs;
  __shared__ unsigned full[S], freed[S], prog[C], bbase[NB];
  __shared__ unsigned bypass, tab_job, seq_end, nclaimed, claim_end, lbatch, first;

  const size_t nvec = L.nbytes / 16;
  const unsigned rows = static_cast<unsigned>((nvec + 63) / 64);
  // queue of this block: blockIdx % 8 (the XCD the dispatcher deals it to);
  // one queue when the grid is not a multiple of 8 blocks, so that every
  // queue has blocks and all queues the same number of them
  const unsigned nq = (gridDim.x % kClaimQueues == 0) ? kClaimQueues : 1u;
  const unsigned q = blockIdx.x % nq;
  const unsigned RQ = ((rows + nq - 1) / nq + B - 1) / B * B;
  const unsigned njobs = static_cast<unsigned>(L.njobs);
  const unsigned total = RQ * njobs;  // items of one queue
  unsigned* const qctr = L.claim + q * kClaimStride;
  unsigned* const fin = L.claim + kClaimQueues * kClaimStride;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  auto vec_of = [&](unsigned u) { return (static_cast<size_t>((u % RQ) * nq + q)) * 64 + lane; };
  auto row_ok = [&](unsigned u) { return (u % RQ) * nq + q < rows; };

  if (threadIdx.x == 0) {
    const unsigned b0 = atomicAdd(qctr, B);
    bbase[0] = b0;
    first = b0;
  }
  __syncthreads();
  const unsigned b0 = first;
  if (b0 < total) {
    const unsigned job0 = b0 / RQ;
    for (int e = threadIdx.x; e < NIN * 32; e += blockDim.x) {
      const int i = e >> 5, h = (e >> 4) & 1, n = e & 15;
      const uint32_t x = static_cast<uint32_t>(n) << (4 * h);
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < NOUT; ++j) v |= gf_mul_dev(jobs[job0].coef[j][i], x) << (8 * j);
      lds[((job0 & 1) * kTab + i * kTableBytes + (h ? kHiBase + n * kHiStride : n * 4)) / 4] = v;
    }
  }
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  if (threadIdx.x < C) prog[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0) {
    bypass = 0;
    tab_job = b0 < total ? b0 / RQ : 0;
    seq_end = b0 < total ? 0xFFFFFFFFu : 0u;
    nclaimed = b0 < total ? 1u : 0u;
    claim_end = b0 < total ? 0xFFFFFFFFu : 0u;
    lbatch = 0;
  }
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);  // see ring_sweep

  if (wave == 0) {
    if (b0 < total) {
      const uint32_t ring0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lr_u4*) ring)));
      unsigned pub = 0;
      auto publish = [&]() {
        ring_publish(&full[pub % S], pub / S + 1, lane);
        ++pub;
      };
      auto past = [&](unsigned T) {
        const bool ok = lane >= C || ring_flag_ld(&prog[lane]) >= T;
        return __builtin_amdgcn_ballot_w64(!ok) == 0;
      };
      unsigned job = b0 / RQ;
      unsigned last_end[2] = {0u, 0u};  // position after the last job that used each table buffer
      const uint8_t* in[NIN];
#pragma unroll
      for (int i = 0; i < NIN; ++i) in[i] = jobs[job].in[i];
      unsigned p = 0;
      bool stop = false;
      for (unsigned n = 0; !stop; ++n) {
        // batch n's base from the claimer (claimed ahead; a wait is rare)
        if (lane == 0) ring_flag_st(&lbatch, n);
        if (ring_flag_ld(&nclaimed) <= n && ring_flag_ld(&claim_end) > n) {
          ring_wait_vm<0>();
          while (pub < p) publish();
          unsigned spins = 0;
          while (ring_flag_ld(&nclaimed) <= n && ring_flag_ld(&claim_end) > n && ring_flag_ld(&bypass) == 0u &&
                 ++spins < kRingSpinCap)
            __builtin_amdgcn_s_sleep(1);
          if (spins >= kRingSpinCap || (ring_flag_ld(&nclaimed) <= n && ring_flag_ld(&bypass) != 0u)) {
            if (lane == 0) {
              ring_flag_st(&bypass, 1u);
              if (L.fault) atomicAdd(L.fault, 1u);
            }
            stop = true;
            break;
          }
        }
        if (ring_flag_ld(&nclaimed) <= n) break;  // the queue is empty: the end
        const unsigned base = __builtin_amdgcn_readfirstlane(ring_flag_ld(&bbase[n % NB]));
        const unsigned bj = base / RQ;
        if (bj != job) {
          // a new job at position p: its tables go to buffer bj & 1, last used
          // by a job that ended at last_end[bj & 1]
          last_end[job & 1] = p;
          job = bj;
          const unsigned T = last_end[job & 1];
          if (!past(T)) {
            ring_wait_vm<0>();
            while (pub < p) publish();
            unsigned spins = 0;
            while (!past(T) && ++spins < kRingHangCap) __builtin_amdgcn_s_sleep(1);
            if (spins >= kRingHangCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
          }
          build_tables_wave<NIN, NOUT>(lds, (job & 1) * kTab, jobs + job, lane);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) ring_flag_st(&tab_job, job);
#pragma unroll
          for (int i = 0; i < NIN; ++i) in[i] = jobs[job].in[i];
        }
        // rows of this batch: (bq + i) * nq + q (RQ is a multiple of B, so a
        // batch stays in one job; one division per batch)
        const unsigned bq = base - bj * RQ;
        // (checking a batch's B slots at once, one LDS round trip instead of
        // B, measured -1% on the encode: r03s46)
        for (unsigned i = 0; i < B; ++i, ++p) {
          const unsigned use = p / S;
          if (ring_flag_ld(&freed[p % S]) < use) {
#if REDSET_RING_DRAIN
            ring_wait_vm<0>();
            while (pub < p) publish();
#endif
            unsigned spins = 0;
            while (ring_flag_ld(&freed[p % S]) < use && ++spins < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
            if (spins >= kRingSpinCap) {
              // stop: publish what is issued; the consumers take the rest of
              // the claimed batches directly, then claim on their own
              ring_wait_vm<0>();
              while (pub < p) publish();
              if (lane == 0) {
                ring_flag_st(&bypass, 1u);
                if (L.fault) atomicAdd(L.fault, 1u);
              }
              stop = true;
              break;
            }
          }
          // (p is uniform; the compiler cannot tell after the capped waits)
          const uint32_t slot = __builtin_amdgcn_readfirstlane(ring0 + (p % S) * NIN * 1024);
          const unsigned row = (bq + i) * nq + q;
          const size_t v = row < rows ? static_cast<size_t>(row) * 64 + lane : 0;
          const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
          for (int k = 0; k < NIN; ++k) {
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
#if REDSET_LOAD_POLICY == 1
                " nt"
#endif
                "\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"((g_cu4*) (in[k]) + vc), "s"(slot + static_cast<uint32_t>(k * 1024))
                : "memory");
          }
          if (p + 1 - pub == static_cast<unsigned>(D)) {
            ring_wait_vm<(D - 1) * NIN>();
            publish();
          }
        }
      }
      ring_wait_vm<0>();
      while (pub < p) publish();
      // the positions the consumers may expect: all issued, or (stopped) every
      // position of the batches claimed so far
      if (lane == 0) {
        const unsigned nc = ring_flag_ld(&nclaimed);
        ring_flag_st(&seq_end, stop && nc * B > p ? nc * B : p);
      }
    }
  } else if (wave == 1) {
    // claimer: keep up to kLook batches claimed ahead of the loader's batch
    if (b0 < total) {
      for (unsigned n = 1;; ++n) {
        unsigned spins = 0;
        while (n >= ring_flag_ld(&lbatch) + 1 + kLook && ring_flag_ld(&bypass) == 0u && ++spins < kRingSpinCap)
          __builtin_amdgcn_s_sleep(2);
        if (ring_flag_ld(&bypass) != 0u || spins >= kRingSpinCap) {
          if (spins >= kRingSpinCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
          if (lane == 0) ring_flag_st(&bypass, 1u);
          break;
        }
        unsigned bb = 0;
        if (lane == 0) bb = atomicAdd(qctr, B);
        bb = __builtin_amdgcn_readfirstlane(bb);
        if (bb >= total) {
          if (lane == 0) ring_flag_st(&claim_end, n);
          break;
        }
        if (lane == 0) {
          ring_flag_st(&bbase[n % NB], bb);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          ring_flag_st(&nclaimed, n + 1);
        }
      }
    }
  } else {
    // consumers: positions c, c + C, ... of the block's sequence
    const int c = wave - 2;
    GfAcc<NOUT, ACC> body;
    body.lds = lds;
    g_cu4* in[NIN];
    int cur = -1;
    unsigned cur_lo = 0;  // first queue item of job `cur`
    for (unsigned p = c;; p += C) {
      const unsigned want = p / S + 1;
      unsigned spins = 0;
      bool direct = false, done = false;
      while (ring_flag_ld(&full[p % S]) < want) {
        if (p >= ring_flag_ld(&seq_end)) {
          done = true;
          break;
        }
        if (ring_flag_ld(&bypass) != 0u || ++spins >= kRingSpinCap) {
          direct = true;
          break;
        }
        __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
      }
      if (done) break;
      unsigned u;
      if (!direct) {
        // claimed, and its bbase entry cannot be reused before this position is released
        u = ring_flag_ld(&bbase[(p / B) % NB]) + p % B;
      } else {
        if (spins >= kRingSpinCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
        // the position's item from its batch's base once the batch is claimed;
        // a batch is never claimed once the queue is empty (claim_end) or the
        // claimer has stopped (BYPASS): then this sequence ends here. Nothing
        // else keeps the claim back, so the wait ends (hang cap only)
        unsigned s3 = 0;
        while (ring_flag_ld(&nclaimed) <= p / B && ring_flag_ld(&claim_end) > p / B && ring_flag_ld(&bypass) == 0u &&
               ++s3 < kRingHangCap)
          __builtin_amdgcn_s_sleep(1);
        if (s3 >= kRingHangCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
        if (ring_flag_ld(&nclaimed) <= p / B) break;
        u = ring_flag_ld(&bbase[(p / B) % NB]) + p % B;
      }
      u = __builtin_amdgcn_readfirstlane(u);
      if (cur < 0 || u - cur_lo >= RQ) {  // another job than the last position's (rare): divide
        const unsigned jn = u / RQ;
        cur = static_cast<int>(jn);
        cur_lo = jn * RQ;
#pragma unroll
        for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (jobs[jn].in[i]);
#pragma unroll
        for (int j = 0; j < NOUT; ++j) body.out[j] = (g_u4*) (jobs[jn].out[j]);
      }
      const unsigned job = static_cast<unsigned>(cur);
      const unsigned row = (u - cur_lo) * nq + q;
      const size_t v = static_cast<size_t>(row) * 64 + lane;
      const bool ok = row < rows && v < nvec;
      v4u x[NIN];
      if (!direct) {
        const lr_u4* sl = (const lr_u4*) ring + (p % S) * NIN * 64;
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[i] = sl[i * 64 + lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) ring_flag_st(&freed[p % S], want);
      } else {
        unsigned s2 = 0;
        while (ring_flag_ld(&freed[p % S]) + 1u < want && ++s2 < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
        if (lane == 0 && ring_flag_ld(&freed[p % S]) + 1u >= want) ring_flag_st(&freed[p % S], want);
        const size_t vc = ok ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[i] = ring_direct_load(in[i] + vc);
      }
      // this job's tables: wait for them unless the loader has stopped
      bool tables = true;
      if (ring_flag_ld(&tab_job) < job) {
        unsigned s4 = 0;
        while (ring_flag_ld(&tab_job) < job && ring_flag_ld(&bypass) == 0u && ++s4 < kRingSpinCap)
          __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
        tables = ring_flag_ld(&tab_job) >= job;
      }
      if (ok) {
        if (tables) {
          body.begin();
          if (job & 1) body.template add<0, NIN, kTab>(x);
          else body.template add<0, NIN, 0>(x);
          body.finish(v);
        } else {
          gf_mac_vec_slow<NIN, NOUT, ACC>(jobs + job, in, v);
        }
      }
      if (lane == 0) ring_flag_st(&prog[c], p + C);
    }
    if (lane == 0) ring_flag_st(&prog[c], 0xFFFFFFFFu);
    // the loader stopped early: claim what is left, batch by batch, and
    // compute it without tables
    if (ring_flag_ld(&bypass) != 0u) {
      while (true) {
        unsigned bb = 0;
        if (lane == 0) bb = atomicAdd(qctr, B);
        bb = __builtin_amdgcn_readfirstlane(bb);
        if (bb >= total) break;
        const unsigned job = bb / RQ;
        g_cu4* jin[NIN];
#pragma unroll
        for (int i = 0; i < NIN; ++i) jin[i] = (g_cu4*) (jobs[job].in[i]);
        for (unsigned i = 0; i < B; ++i) {
          const unsigned u = bb + i;
          const size_t v = vec_of(u);
          if (row_ok(u) && v < nvec) gf_mac_vec_slow<NIN, NOUT, ACC>(jobs + job, jin, v);
        }
      }
    }
  }
  // every claim of this block is done: count it; the launch's last block
  // zeroes the queues for the next launch (stream order makes it visible)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned done = atomicAdd(fin, 1u);
    if (done == gridDim.x - 1) {
      __threadfence();
      for (int k = 0; k < kClaimQueues; ++k) atomicExch(L.claim + k * kClaimStride, 0u);
      atomicExch(fin, 0u);
    }
  }
}
#endif

#if REDSET_RING
// kJobsStreamed for XOR (see gf_mac_stream): the launch's jobs through one
// continuous ring, item g of a block = item g % K of job g / K; no tables, so
// no hand-over between jobs. Same items (R rows), depth and fallbacks as
// xor_body's ring_sweep.
// the XOR kernels' ring, one static array shared by xor_body and xor_stream
template <int NIN, int R>
__device__ __forceinline__ v4u* xor_lds() {
  __shared__ v4u ring[ring_vecs<NIN, R>()];
  return ring;
}

template <int NIN, bool ACC>
__device__ __forceinline__ void xor_stream(const XorLaunch& L) {
  constexpr int R = NIN > REDSET_RING_XOR_WIDE ? 1 : REDSET_RING_XOR_ROWS;
  constexpr int D =
      ring_depth<NIN, R, R == 1 ? REDSET_RING_XOR_ROWS_IN_FLIGHT : REDSET_RING_ROWS_IN_FLIGHT>();
  constexpr int S = ring_slots<NIN * R>();
  constexpr int C = kBlock / 64 - 1;
  static_assert(D >= 2 && D - 1 < S && (D - 1) * NIN * R <= 63, "ring depth");
  typedef __attribute__((address_space(4))) const XorJob c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  v4u* const ring = xor_lds<NIN, R>();
  __shared__ unsigned full[S], freed[S], bypass;

  const size_t nvec = L.nbytes / 16;
  const size_t G = gridDim.x;
  const size_t part = blockIdx.x;
  const size_t rows = (nvec + 63) / 64;
  const size_t items = (rows + R - 1) / R;
  const unsigned K = items > part ? static_cast<unsigned>((items - part + G - 1) / G) : 0u;
  const unsigned total = K * static_cast<unsigned>(L.njobs);
  if (K == 0) return;
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  if (threadIdx.x == 0) bypass = 0;
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);  // see ring_sweep
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
  const int lane = threadIdx.x & 63;
  auto vec_of = [&](unsigned k, int r) { return ((static_cast<size_t>(k) * G + part) * R + r) * 64 + lane; };

  if (wave == 0) {
    const uint32_t ring0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lr_u4*) ring)));
    unsigned pub = 0;
    auto publish = [&]() {
      ring_publish(&full[pub % S], pub / S + 1, lane);
      ++pub;
    };
    const uint8_t* in[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) in[i] = jobs[0].in[i];
    unsigned job = 0, k = 0;
    for (unsigned g = 0; g < total; ++g, ++k) {
      if (k == K) {
        k = 0;
        ++job;
#pragma unroll
        for (int i = 0; i < NIN; ++i) in[i] = jobs[job].in[i];
      }
      const unsigned use = g / S;
      if (ring_flag_ld(&freed[g % S]) < use) {
#if REDSET_RING_DRAIN
        ring_wait_vm<0>();
        while (pub < g) publish();
#endif
        unsigned spins = 0;
        while (ring_flag_ld(&freed[g % S]) < use && ++spins < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
        if (spins >= kRingSpinCap) {
          ring_wait_vm<0>();
          while (pub < g) publish();
          if (lane == 0) {
            ring_flag_st(&bypass, 1u);
            if (L.fault) atomicAdd(L.fault, 1u);
          }
          return;
        }
      }
      const uint32_t slot = ring0 + (g % S) * NIN * R * 1024;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const size_t v = vec_of(k, r);
        const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          uint32_t keep;
          asm volatile(
              "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
#if REDSET_LOAD_POLICY == 1
              " nt"
#endif
              "\n\ts_mov_b32 m0, %0"
              : "=&s"(keep)
              : "v"((g_cu4*) (in[i]) + vc), "s"(slot + static_cast<uint32_t>((i * R + r) * 1024))
              : "memory");
        }
      }
      if (g + 1 - pub == static_cast<unsigned>(D)) {
        ring_wait_vm<(D - 1) * NIN * R>();
        publish();
      }
    }
    ring_wait_vm<0>();
    while (pub < total) publish();
    return;
  }

  const int c = wave - 1;
  XorAcc<ACC> body;
  g_cu4* in[NIN];
  int cur = -1;
  unsigned job = static_cast<unsigned>(c) / K, k = static_cast<unsigned>(c) % K;
  for (unsigned g = c; g < total; g += C) {
    if (static_cast<int>(job) != cur) {
      cur = static_cast<int>(job);
#pragma unroll
      for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (jobs[job].in[i]);
      body.out = (g_u4*) (jobs[job].out);
    }
    const unsigned want = g / S + 1;
    unsigned spins = 0;
    bool direct = false;
    while (ring_flag_ld(&full[g % S]) < want) {
      if (ring_flag_ld(&bypass) != 0u || ++spins >= kRingSpinCap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(REDSET_RING_SLEEP);
    }
    if (direct) {
      // as in ring_sweep
      if (spins >= kRingSpinCap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[g % S]) + 1u < want && ++s2 < kRingSpinCap) __builtin_amdgcn_s_sleep(1);
      if (lane == 0 && ring_flag_ld(&freed[g % S]) + 1u >= want) ring_flag_st(&freed[g % S], want);
    }
    const lr_u4* sl = (const lr_u4*) ring + (g % S) * NIN * R * 64;
    v4u x[R][NIN];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!direct) {
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[r][i] = sl[(i * R + r) * 64 + lane];
      } else {
        const size_t v = vec_of(k, r);
        const size_t vc = v < nvec ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[r][i] = ring_direct_load(in[i] + vc);
      }
    }
    if (!direct) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) ring_flag_st(&freed[g % S], want);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t v = vec_of(k, r);
      if (v < nvec) {
        body.begin();
        body.template add<0>(x[r]);
        body.finish(v);
      }
    }
    k += C;
    while (k >= K) k -= K, ++job;
  }
}
#endif

template <int NIN, bool ACC>
__device__ __forceinline__ void xor_body(const XorLaunch& L, const XorJob& J, int part) {
  const size_t nvec = L.bytes_only ? 0 : L.nbytes / 16;
  const size_t vstep = static_cast<size_t>(L.blocks_per_job) * kBlock;
  if (nvec > 0) {
    g_cu4* in[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (J.in[i]);
    g_u4* out = (g_u4*) (J.out);
#if REDSET_RING
    // two-row items hold 2 * NIN input vectors per lane: past 8 inputs that
    // no longer fits 1024-thread blocks' 128 VGPRs, so wide XOR sets take
    // the GF kernels' one-row shape
    constexpr int kRows = NIN > REDSET_RING_XOR_WIDE ? 1 : REDSET_RING_XOR_ROWS;
    constexpr int kDepth = ring_depth<NIN, kRows, kRows == 1 ? REDSET_RING_XOR_ROWS_IN_FLIGHT : REDSET_RING_ROWS_IN_FLIGHT>();
    v4u* const ring = xor_lds<NIN, kRows>();
    XorAcc<ACC> body;
    body.out = out;
    ring_sweep<NIN, kRows, kDepth>(ring, in, nvec, static_cast<size_t>(L.blocks_per_job),
                                   static_cast<size_t>(part), L.fault, body);
#else
    sweep<NIN, sweep_prio(3)>(
        in, nvec, vstep, part, [&](const v4u (&x)[NIN], size_t v, bool st) { xor_vec<NIN, ACC>(x, out, v, st); },
        [&](size_t v) {
          if constexpr (!ACC) out[v] = v4u{0, 0, 0, 0};
        });
#endif
  }
  const size_t tail0 = nvec * 16;
  for (size_t k = tail0 + static_cast<size_t>(part) * kBlock + threadIdx.x; k < L.nbytes; k += vstep) {
    uint8_t r = ACC ? J.out[k] : 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) r ^= J.in[i][k];
    J.out[k] = r;
  }
}

// Optional (A/B only): give each XCD a contiguous run of the job's block
// windows instead of every 8th one (blocks are dealt round-robin over the
// 8 XCDs, so blocks b and b+8 share one).
__device__ __forceinline__ int job_block(int b, int per_job) {
#if defined(REDSET_XCD_REMAP) && REDSET_XCD_REMAP
  if ((per_job & 7) == 0) return (b & 7) * (per_job >> 3) + (b >> 3);
#endif
  return b;
}

// entry points: jobs from a device array (plans), or one job passed by
// value in the kernel arguments (stripe primitives, no device descriptor)
// Timing-only knob (never shipped): every block records its start and end
// (s_memrealtime, 100 MHz) and its hardware placement into the words behind
// the fault word (codec_kernels.hip sizes them; read by
// redset_hip_debug_block_clock), to see how evenly a launch's blocks finish.
#ifndef REDSET_BLOCK_CLOCK
#define REDSET_BLOCK_CLOCK 0
#endif
struct BlockClock {
#if REDSET_BLOCK_CLOCK
  // block start (thread 64) and every consumer wave's end (atomicMax by its
  // lane 0): no barrier, and nothing from the ring's loader wave (wave 0) --
  // a compiler-visible store in that wave makes hipcc put a vmcnt(0) wait
  // into its LDS-DMA issue loop (measured: the launch 60% slower)
  unsigned long long* c;
  __device__ __forceinline__ explicit BlockClock(unsigned* f)
      : c(reinterpret_cast<unsigned long long*>(f + 64) + 3 * blockIdx.x) {
    if (threadIdx.x == 64) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      const unsigned long long t = __builtin_amdgcn_s_memrealtime();
      const unsigned long long id = (static_cast<unsigned long long>(xcc) << 32) | hw;
      // one asm block, stores and their wait: no VMEM event the compiler's
      // wait insertion could carry into the loader's loop (a plain store here
      // does, see above)
      asm volatile(
          "global_store_dwordx2 %0, %1, off\n\t"
          "global_store_dwordx2 %0, %2, off offset:8\n\t"
          "global_store_dwordx2 %0, %3, off offset:16\n\t"
          "s_waitcnt vmcnt(0)"
          :
          : "v"(c), "v"(t), "v"(0ull), "v"(id)
          : "memory");
    }
  }
  __device__ __forceinline__ ~BlockClock() {
    if ((threadIdx.x & 63) == 0 && threadIdx.x >= 64) atomicMax(c + 1, __builtin_amdgcn_s_memrealtime());
  }
#else
  __device__ __forceinline__ explicit BlockClock(unsigned*) {}
#endif
};

template <int NIN, int NOUT, bool ACC>
REDSET_KERNEL gf_mac_kernel(GfLaunch L) {
  BlockClock clock(L.fault);
#if REDSET_RING
  if constexpr (NIN <= 8 && REDSET_RING_GF_ROWS == 1) {
    if (L.sequential == kJobsStreamed && !L.bytes_only && L.nbytes % 16 == 0) {
      gf_mac_stream<NIN, NOUT, ACC>(L);
      return;
    }
    if (L.sequential == kJobsClaimed && L.claim && !L.bytes_only && L.nbytes % 16 == 0) {
      gf_mac_claimed<NIN, NOUT, ACC>(L);
      return;
    }
  }
#endif
  if (L.sequential == kJobsInKernel || L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) {
    // every block sweeps every job in turn: one stripe's cells in flight at
    // a time, with no launch boundary between stripes
    for (int j = 0; j < L.njobs; ++j) {
      if (j > 0) __syncthreads();  // all waves are done with the last job's tables
      gf_mac_body<NIN, NOUT, ACC>(L, L.jobs[L.job0 + j], blockIdx.x);
    }
    return;
  }
  const int job = blockIdx.x / L.blocks_per_job;
  gf_mac_body<NIN, NOUT, ACC>(L, L.jobs[L.job0 + job], job_block(blockIdx.x - job * L.blocks_per_job, L.blocks_per_job));
}

template <int NIN, int NOUT, bool ACC>
REDSET_KERNEL gf_mac_kernel_arg(GfLaunch L, GfJob J) {
  gf_mac_body<NIN, NOUT, ACC>(L, J, blockIdx.x);
}

template <int NIN, bool ACC>
REDSET_KERNEL xor_kernel(XorLaunch L) {
  BlockClock clock(L.fault);
#if REDSET_RING
  if constexpr (NIN <= REDSET_RING_CHUNK) {
    if (L.sequential == kJobsStreamed && !L.bytes_only && L.nbytes % 16 == 0) {
      xor_stream<NIN, ACC>(L);
      return;
    }
  }
#endif
  if (L.sequential == kJobsInKernel || L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) {
    for (int j = 0; j < L.njobs; ++j) xor_body<NIN, ACC>(L, L.jobs[L.job0 + j], blockIdx.x);
    return;
  }
  const int job = blockIdx.x / L.blocks_per_job;
  xor_body<NIN, ACC>(L, L.jobs[L.job0 + job], job_block(blockIdx.x - job * L.blocks_per_job, L.blocks_per_job));
}

template <int NIN, bool ACC>
REDSET_KERNEL xor_kernel_arg(XorLaunch L, XorJob J) {
  xor_body<NIN, ACC>(L, J, blockIdx.x);
}

template <int N>
constexpr KernelSet make_kernel_set() {
  return KernelSet{
      {{&gf_mac_kernel<N, 1, false>, &gf_mac_kernel<N, 1, true>},
       {&gf_mac_kernel<N, 2, false>, &gf_mac_kernel<N, 2, true>},
       {&gf_mac_kernel<N, 3, false>, &gf_mac_kernel<N, 3, true>},
       {&gf_mac_kernel<N, 4, false>, &gf_mac_kernel<N, 4, true>}},
      {{&gf_mac_kernel_arg<N, 1, false>, &gf_mac_kernel_arg<N, 1, true>},
       {&gf_mac_kernel_arg<N, 2, false>, &gf_mac_kernel_arg<N, 2, true>},
       {&gf_mac_kernel_arg<N, 3, false>, &gf_mac_kernel_arg<N, 3, true>},
       {&gf_mac_kernel_arg<N, 4, false>, &gf_mac_kernel_arg<N, 4, true>}},
      {&xor_kernel<N, false>, &xor_kernel<N, true>},
      {&xor_kernel_arg<N, false>, &xor_kernel_arg<N, true>},
  };
}

}  // namespace

}  // namespace redset_hip

// Defines `const KernelSet* FN(int nin)` for the listed input counts
// (consecutive, starting at FIRST), nullptr for any other count.
#define REDSET_DEFINE_KERNEL_SETS(FN, FIRST, ...)                                  \
  namespace redset_hip {                                                           \
  const KernelSet* FN(int nin) {                                                   \
    static const KernelSet sets[] = {__VA_ARGS__};                                 \
    const int n = static_cast<int>(sizeof(sets) / sizeof(sets[0]));                \
    return (nin >= FIRST && nin < FIRST + n) ? &sets[nin - FIRST] : nullptr;       \
  }                                                                                \
  }
