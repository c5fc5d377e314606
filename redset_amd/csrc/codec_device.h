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
//   Inputs stream in through a loader-wave LDS-DMA ring (ring_sweep); the 16
//   packed accumulators are transposed back to per-output bytes with v_perm.
//
// xor_reduce: out = XOR of inputs (reference reduce_xor, src/redset_xor.c:35-42;
//   CUDA xor_gpu, src/redset_xor_gpu.cu:20-26), one pass, 16-B vectors.
//
// Kernel templates only; every codec_sets_*.hip instantiates them for a
// range of input counts (split so the instantiations compile in parallel)
// and exposes them through a KernelSet table (codec_kernels.h).
//
// This is the shipping kernel source: every constant below is the measured
// choice (DESIGN.md section 4 gives each one's A/B). The alternatives that
// lost -- the per-wave sweep and its software pipeline, a per-wave LDS-DMA
// ring, wave priorities, 64-bit high-nibble reads, all-lane publishes, other
// cache policies, XCD-contiguous windows, the XOR-for-GF memory skeleton and
// the per-block clock -- live on the branch r3-ab-apparatus with the tools
// that built them. The one build option left is REDSET_HIP_TEST_KNOBS
// (test twin library only, see kRingSpinCap).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "codec_kernels.h"

// One 1024-thread block per CU (1 loader + 15 consumer waves, codec_kernels.h)
// compiled for its own 4 waves per SIMD: up to 128 VGPRs per lane.
#define REDSET_KERNEL \
  __global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, kBlock / 256)))

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
// then the high-nibble table at kHiBase (entry n at kHiBase + 4n). Both keep
// their 16 entries in 16 distinct LDS banks.
constexpr int kHiStride = 4;
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

// 4 * (nibble of byte B of x >> or << 2) in one VALU op: v_and_b32 with an
// SDWA byte select on x (x = w << 2: low nibble of byte B of w; x = w >> 2:
// its high nibble), 60 = 0x3C keeps the four nibble bits at offset 2. One op
// per table offset instead of a shift-and-mask plus an extract (+0.7% on the
// encode with the tables at the bottom of LDS, profiles/r03_ab_tables_first.txt)
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

// gather byte j of a[0..3] into one dword
__device__ __forceinline__ uint32_t gather_byte(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, int j) {
  const uint32_t sel_lo = 0x0c0c0000u | (static_cast<uint32_t>(4 + j) << 8) | static_cast<uint32_t>(j);
  const uint32_t sel_hi = 0x00000c0cu | (static_cast<uint32_t>(4 + j) << 24) | (static_cast<uint32_t>(j) << 16);
  return __builtin_amdgcn_perm(a1, a0, sel_lo) | __builtin_amdgcn_perm(a3, a2, sel_hi);
}

// Global-address-space views of the cell pointers: loads and stores through
// them are global_load/store (vmcnt only), not flat ones, which would also
// count on lgkmcnt and make every LDS wait drain the HBM loads.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u g_cu4;
typedef __attribute__((address_space(1))) v4u g_u4;

// One 16-B store of an output stream. Every cell byte is read or written
// exactly once, so stores (and the ring's LDS-DMA loads) are non-temporal:
// +3% on the RS step and +7% on XOR against the default policy, while either
// direction alone gains nothing (profiles/r01_ab_cache_policy.txt).
__device__ __forceinline__ void store_vec(g_u4* p, size_t v, v4u r) { __builtin_nontemporal_store(r, p + v); }

// acc (packed partial products of all outputs, 16 bytes) ^= coef[.][i] * x.
// TB: byte offset of the tables in LDS (a constant, so it folds into the
// ds_read immediate like the input's own offset; the streamed kernels keep
// two jobs' tables, TB selects one)
template <int TB = 0>
__device__ __forceinline__ void gf_acc_input(const uint32_t* lds, const v4u& x, int i, uint32_t (&acc)[16]) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t ol[4], oh[4];
    const uint32_t wl = w[q] << 2;
    ol[0] = nibble_offset<0>(wl), ol[1] = nibble_offset<1>(wl), ol[2] = nibble_offset<2>(wl);
    ol[3] = nibble_offset<3>(wl);
    const uint32_t wh = w[q] >> 2;
    oh[0] = nibble_offset<0>(wh), oh[1] = nibble_offset<1>(wh), oh[2] = nibble_offset<2>(wh);
    oh[3] = nibble_offset<3>(wh);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      acc[4 * q + b] = xor3(acc[4 * q + b], lds_at(lds, TB + i * kTableBytes + ol[b]),
                            lds_at(lds, TB + i * kTableBytes + kHiBase + oh[b]));
    }
  }
}

// Incremental combine for the loader ring's consumers (ring_sweep):
// begin(), then add<I0>(x) for inputs [I0, I0 + N) of one 16-B position,
// then finish(v) stores it. A consumer of a wide stripe adds its inputs in
// chunks so that only one chunk is live in VGPRs.
template <int NOUT, bool ACC>
struct GfAcc {
  const uint32_t* lds;
  g_u4* out[NOUT];
  uint32_t acc[16];
  __device__ __forceinline__ void begin() {
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = 0;
  }
  template <int I0, int N, int TB = 0>
  __device__ __forceinline__ void add(const v4u (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) gf_acc_input<TB>(lds, x[i], I0 + i, acc);
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
// adds 1 to the launch's first fault word (redset_hip_ring_faults()): a
// performance event, not an error. (Waits with no fallback count in the
// second word instead, see kRingHangCap.) Capped spins did happen once, from a
// missing barrier between the jobs of an in-kernel job loop (round 2,
// profiles/r02s62_gpu_tests_ring_fault.log, fixed at the top of ring_sweep);
// the test twin library runs the suite with a 4-poll cap, which drives both
// fallbacks on every launch, and is checked bit for bit
// (tests/test_gpu_test_build.py).
//
// LDS for the ring's slots (the GF tables take 2 KiB more): 144 KiB gives
// wide stripes a slot more (16 inputs: 9 instead of 8), +0.9% on RS(16+4);
// stripes of <= 8 inputs keep 16 slots (profiles/r03_ring_depth_sweep.txt)
constexpr int kRingBudget = 144 * 1024;
constexpr int kRingMaxSlots = 16;
// Ring shape per kernel: R = 64-vector rows of every input per item. gf_mac:
// 1 row (the consumers' GF math sets part of the pace; two-row items cost
// 3%). XOR: 2 rows (+3-4% over 1 row; profiles/r02_ab_ring_rows.txt) up to
// kRingXorWide inputs, 1 row past that (two-row items would spill).
constexpr int kRingGfRows = 1;
constexpr int kRingXorRows = 2;
constexpr int kRingXorWide = 8;
// D, the items the loader keeps in flight, is picked so that about F 1 KiB
// rows are pending behind the item being published: D - 1 = round(F / (NIN *
// R)), at most kRingMaxDepth items. F = 16, except 20 for the one-row items
// of xor past 8 inputs (light consumers; with two-row items 16 stays best).
// Measured on one box for every width 1-16 against fixed D = 2, 3, 4, 6, 9
// (profiles/r03_ring_depth_sweep.txt): the rule is best or within run-to-run
// noise (~2%) everywhere -- RS(8+3): 8 inputs, D = 3; XOR p = 8: 7 inputs x
// 2 rows, D = 2 -- and gains on narrow stripes against round 2's fixed
// depths: GF 2 / 4 inputs +37% / +17%, XOR 3 inputs +27%.
constexpr int kRingRowsInFlight = 16;
constexpr int kRingXorRowsInFlight = 20;
constexpr int kRingMaxDepth = 9;
// s_sleep argument (x 64 clocks) between a consumer's polls of a FULL word:
// polls take issue slots from the co-resident consumers that are computing
// (~17% of the LDS instructions at 1, profiles/r02s60_ring_pmc_lds.txt);
// 8 measured +0.9% on the RS step, rebuild +1.5-2% (4 and 16 alike;
// profiles/r02_ab_ring_sleep.txt)
constexpr int kRingSleep = 8;
template <int NIN>
constexpr int ring_slots() {
  return kRingBudget / (NIN * 1024) > kRingMaxSlots ? kRingMaxSlots : kRingBudget / (NIN * 1024);
}
// Polls before a handshake gives up on the ring. The test twin library
// (REDSET_HIP_TEST_KNOBS) takes the cap from the launch (GfLaunch::spin_cap,
// REDSET_HIP_TEST_SPIN_CAP): a tiny cap exercises the direct-load fallbacks
// on every launch.
constexpr unsigned kRingSpinCap = 1u << 24;
#if REDSET_HIP_TEST_KNOBS
#define RING_SPIN_CAP(L) ((L).spin_cap)
#else
#define RING_SPIN_CAP(L) kRingSpinCap
#endif
// Waits that end by construction and have no fallback (the streamed kernels'
// table hand-over, the claimed kernel's claim records and its loader's wait
// for the claimer): their cap is only insurance against a hang from a bug.
// A capped one is NOT a performance event -- the wait proceeds with another
// job's tables or drops positions, so the launch's outputs are wrong -- and
// it counts in the launch's SECOND fault word (L.fault[1], the hang word;
// redset_hip_hang_faults). Every product entry point that runs kernels reads
// that word after its last sync and fails the call when it moved. The test
// twin takes this cap from the launch too (GfLaunch::hang_cap,
// REDSET_HIP_TEST_HANG_CAP), independent of the spin cap, so the suite can
// make it fire and check that the call fails.
constexpr unsigned kRingHangCap = 1u << 26;
#if REDSET_HIP_TEST_KNOBS
#define RING_HANG_CAP(L) ((L).hang_cap)
#else
#define RING_HANG_CAP(L) kRingHangCap
#endif
#define RING_HANG_FAULT(L) atomicAdd((L).fault + 1, 1u)
// Test builds: the loader sleeps before it publishes a job's tables
// (REDSET_HIP_TEST_TABLE_DELAY rounds of s_sleep 127), so consumers reach the
// next job first and wait on the table hand-over.
#if REDSET_HIP_TEST_KNOBS
#define RING_TABLE_DELAY(L) \
  for (unsigned d_ = 0; d_ < (L).table_delay; ++d_) __builtin_amdgcn_s_sleep(127)
#else
#define RING_TABLE_DELAY(L) (void) 0
#endif
// Inputs a ring consumer holds in VGPRs at once; wider stripes are combined in
// two chunks (ring_sweep).
constexpr int kRingChunk = 8;
// items the loader keeps in flight for NIN inputs of R-row items (see
// kRingRowsInFlight), within the ring's slots and vmcnt's 6 bits
template <int NIN, int R, int F>
constexpr int ring_depth() {
  constexpr int rows = NIN * R;
  int d = 1 + (F + rows / 2) / rows;
  if (d > kRingMaxDepth) d = kRingMaxDepth;
  if (d > ring_slots<rows>()) d = ring_slots<rows>();
  while (d > 1 && (d - 1) * rows > 63) --d;
  return d < 2 ? 2 : d;
}
typedef __attribute__((address_space(3))) v4u lr_u4;
typedef __attribute__((address_space(3))) volatile unsigned lr_flag;  // LDS, never flat
__device__ __forceinline__ unsigned ring_flag_ld(unsigned* p) { return *(lr_flag*) p; }
__device__ __forceinline__ void ring_flag_st(unsigned* p, unsigned v) { *(lr_flag*) p = v; }
// A loader publishes an item: lane 0 writes its FULL word
__device__ __forceinline__ void ring_publish(unsigned* p, unsigned v, int lane) {
  if (lane == 0) ring_flag_st(p, v);
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
// The loader's LDS-DMA of one input row into the slot at LDS address `lds`
// (M0), issued from inline asm: hipcc treats the builtin form as an LDS
// write on vmcnt and drains vmcnt(0) before the next ds_read of any slot,
// which would serialise the ring; the ring's waits count it instead.
__device__ __forceinline__ void ring_dma(g_cu4* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
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
                                           unsigned* fault, unsigned cap, Body& body) {
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
        ring_wait_vm<0>();
        while (pub < k) publish();
        unsigned spins = 0;
        while (ring_flag_ld(&freed[k % S]) < use && ++spins < cap) __builtin_amdgcn_s_sleep(1);
        if (spins >= cap) {
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
        for (int i = 0; i < NIN; ++i) ring_dma(in[i] + vc, slot + static_cast<uint32_t>((i * R + r) * 1024));
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
      if (ring_flag_ld(&bypass) != 0u || ++spins >= cap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(kRingSleep);
    }
    if (direct) {
      // the item never arrived in time (or the loader stopped): take this
      // lane's bytes from HBM; the ring copy, if it ever lands, is unread.
      // Release the slot for item k + S only after item k - S's consumer
      // has (FREE = want - 1), or the loader could overwrite a slot that
      // consumer still reads; if that never happens the loader's own capped
      // wait raises BYPASS.
      if (spins >= cap && lane == 0 && fault) atomicAdd(fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[k % S]) + 1u < want && ++s2 < cap) __builtin_amdgcn_s_sleep(1);
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
  constexpr int kRingVecs = ring_vecs<NIN, kRingGfRows>();
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
    GfAcc<NOUT, ACC> body;
    body.lds = lds;
#pragma unroll
    for (int j = 0; j < NOUT; ++j) body.out[j] = (g_u4*) (J.out[j]);
    constexpr int kDepth = ring_depth<NIN, kRingGfRows, kRingRowsInFlight>();
    ring_sweep<NIN, kRingGfRows, kDepth>(smem + kTableVecs, in, nvec, static_cast<size_t>(L.blocks_per_job),
                                         static_cast<size_t>(part), L.fault, RING_SPIN_CAP(L), body);
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
  static_assert(kRingGfRows == 1, "one-row items");
  constexpr int S = ring_slots<NIN>();
  constexpr int D = ring_depth<NIN, 1, kRingRowsInFlight>();
  constexpr int C = kBlock / 64 - 1;
  constexpr int kTab = NIN * kTableBytes;  // one job's tables (bytes)
  static_assert(D >= 2 && D - 1 < S && (D - 1) * NIN <= 63, "ring depth");
  typedef __attribute__((address_space(4))) const GfJob c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  const unsigned cap = RING_SPIN_CAP(L);
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
        // GPU -- a capped wait goes to the hang word and fails the call
        unsigned spins = 0;
        while (!past((j - 1) * K) && ++spins < RING_HANG_CAP(L)) __builtin_amdgcn_s_sleep(1);
        if (spins >= RING_HANG_CAP(L) && lane == 0 && L.fault) RING_HANG_FAULT(L);
      }
      build_tables_wave<NIN, NOUT>(lds, (j & 1) * kTab, jobs + j, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      RING_TABLE_DELAY(L);
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
        ring_wait_vm<0>();
        while (pub < g) publish();
        unsigned spins = 0;
        while (ring_flag_ld(&freed[g % S]) < use && ++spins < cap) __builtin_amdgcn_s_sleep(1);
        if (spins >= cap) {
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
      for (int i = 0; i < NIN; ++i) ring_dma((g_cu4*) (in[i]) + vc, slot + static_cast<uint32_t>(i * 1024));
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
      while (ring_flag_ld(&tab_job) < job && ++spins < RING_HANG_CAP(L)) __builtin_amdgcn_s_sleep(kRingSleep);
      if (spins >= RING_HANG_CAP(L) && lane == 0 && L.fault) RING_HANG_FAULT(L);
#pragma unroll
      for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (jobs[job].in[i]);
#pragma unroll
      for (int j = 0; j < NOUT; ++j) body.out[j] = (g_u4*) (jobs[job].out[j]);
    }
    const unsigned want = g / S + 1;
    unsigned spins = 0;
    bool direct = false;
    while (ring_flag_ld(&full[g % S]) < want) {
      if (ring_flag_ld(&bypass) != 0u || ++spins >= cap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(kRingSleep);
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
      if (spins >= cap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[g % S]) + 1u < want && ++s2 < cap) __builtin_amdgcn_s_sleep(1);
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

// Slow, table-free product of one 16-B position (the claimed kernel's last
// resort, for items whose tables may not exist: see claimed_sweep): a dword
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

// Items per claim (batches of 2 / 8 / 16 rows lose 3-5%), and batches the
// claimer keeps claimed ahead of the loader (a longer look-ahead changes
// nothing; profiles/r03_ab_stream.txt)
constexpr unsigned kClaimBatch = 4;
constexpr unsigned kClaimLook = 2;
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
// A batch the claimer took from its queue is always recorded (bbase[],
// nclaimed) before it raises CLAIMER_DONE, and nobody decides where the
// block's claimed sequence ends -- the loader's seq_end after a stop, a
// consumer's "not claimed" -- before CLAIMER_DONE: otherwise a batch claimed
// in the window between the claimer's BYPASS check and its record would be
// gone from the queue and computed by no one. The counters are
// zeroed by the launcher on the stream before every launch.
// The combine of a claimed launch (claimed_sweep): GF, with per-job tables
// in two LDS buffers (gf_lds: tables first, the ring behind them), or XOR.
template <int NIN_, int NOUT, bool ACC>
struct GfClaim {
  static constexpr int NIN = NIN_;
  static_assert(NIN <= 8 && 2 * NIN * kTableBytes <= kTableVecs * 16, "two jobs' tables in the table region");
  static_assert(kRingGfRows == 1, "one-row items");
  static constexpr bool kTables = true;
  static constexpr int kSlots = ring_slots<NIN>();
  static constexpr int kRingOff = kTableVecs;
  static constexpr int kTab = NIN * kTableBytes;  // one job's tables (bytes)
  using Launch = GfLaunch;
  using Job = GfJob;
  using Body = GfAcc<NOUT, ACC>;
  typedef __attribute__((address_space(4))) const GfJob c_job;
  static __device__ __forceinline__ v4u* lds() { return gf_lds<NIN>(); }
  static __device__ __forceinline__ void init(Body& b, const uint32_t* lds) { b.lds = lds; }
  static __device__ __forceinline__ void set_out(Body& b, const c_job* J) {
#pragma unroll
    for (int j = 0; j < NOUT; ++j) b.out[j] = (g_u4*) (J->out[j]);
  }
  // job j's tables into buffer j & 1: the whole block (first job), or the loader wave
  static __device__ __forceinline__ void first_tables(uint32_t* lds, const c_job* J, unsigned j) {
    for (int e = threadIdx.x; e < NIN * 32; e += blockDim.x) {
      const int i = e >> 5, h = (e >> 4) & 1, n = e & 15;
      const uint32_t x = static_cast<uint32_t>(n) << (4 * h);
      uint32_t v = 0;
#pragma unroll
      for (int o = 0; o < NOUT; ++o) v |= gf_mul_dev(J->coef[o][i], x) << (8 * o);
      lds[((j & 1) * kTab + i * kTableBytes + (h ? kHiBase + n * kHiStride : n * 4)) / 4] = v;
    }
  }
  static __device__ __forceinline__ void next_tables(uint32_t* lds, const c_job* J, unsigned j, int lane) {
    build_tables_wave<NIN, NOUT>(lds, (j & 1) * kTab, J, lane);
  }
  static __device__ __forceinline__ void combine(Body& b, const v4u (&x)[NIN], unsigned job, size_t v) {
    b.begin();
    if (job & 1) b.template add<0, NIN, kTab>(x);
    else b.template add<0, NIN, 0>(x);
    b.finish(v);
  }
  static __device__ __forceinline__ void slow(const c_job* J, g_cu4* const (&in)[NIN], size_t v) {
    gf_mac_vec_slow<NIN, NOUT, ACC>(J, in, v);
  }
};

template <typename Pol>
__device__ __forceinline__ void claimed_sweep(const typename Pol::Launch& L) {
  constexpr int NIN = Pol::NIN;
  constexpr int S = Pol::kSlots;
  constexpr int D = ring_depth<NIN, 1, kRingRowsInFlight>();
  constexpr int C = kBlock / 64 - 2;  // consumer waves
  constexpr unsigned B = kClaimBatch;
  constexpr unsigned kLook = kClaimLook;
  constexpr unsigned NB = 32;
  static_assert(C >= 1 && NB * B >= S + (kLook + 1) * B, "batch ring");
  static_assert(D - 1 < S && (D - 1) * NIN <= 63, "ring depth");
  typedef __attribute__((address_space(4))) const typename Pol::Job c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  const unsigned cap = RING_SPIN_CAP(L);
  v4u* const smem = Pol::lds();
  uint32_t* const lds = reinterpret_cast<uint32_t*>(smem);
  v4u* const ring = smem + Pol::kRingOff;
  __shared__ unsigned full[S], freed[S], prog[C], bbase[NB];
  __shared__ unsigned bypass, tab_job, seq_end, nclaimed, claim_end, lbatch, first, claimer_done;

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
  if (b0 < total) Pol::first_tables(lds, jobs + b0 / RQ, b0 / RQ);
  if (threadIdx.x < S) full[threadIdx.x] = 0, freed[threadIdx.x] = 0;
  if (threadIdx.x < C) prog[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0) {
    bypass = 0;
    tab_job = b0 < total ? b0 / RQ : 0;
    seq_end = b0 < total ? 0xFFFFFFFFu : 0u;
    nclaimed = b0 < total ? 1u : 0u;
    claim_end = b0 < total ? 0xFFFFFFFFu : 0u;
    claimer_done = b0 < total ? 0u : 1u;
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
                 ++spins < cap)
            __builtin_amdgcn_s_sleep(1);
          if (spins >= cap || (ring_flag_ld(&nclaimed) <= n && ring_flag_ld(&bypass) != 0u)) {
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
          if (Pol::kTables && !past(T)) {
            ring_wait_vm<0>();
            while (pub < p) publish();
            unsigned spins = 0;
            while (!past(T) && ++spins < RING_HANG_CAP(L)) __builtin_amdgcn_s_sleep(1);
            if (spins >= RING_HANG_CAP(L) && lane == 0 && L.fault) RING_HANG_FAULT(L);
          }
          if constexpr (Pol::kTables) {
            Pol::next_tables(lds, jobs + job, job, lane);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            RING_TABLE_DELAY(L);
            if (lane == 0) ring_flag_st(&tab_job, job);
          }
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
            ring_wait_vm<0>();
            while (pub < p) publish();
            unsigned spins = 0;
            while (ring_flag_ld(&freed[p % S]) < use && ++spins < cap) __builtin_amdgcn_s_sleep(1);
            if (spins >= cap) {
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
          for (int k = 0; k < NIN; ++k) ring_dma((g_cu4*) (in[k]) + vc, slot + static_cast<uint32_t>(k * 1024));
          if (p + 1 - pub == static_cast<unsigned>(D)) {
            ring_wait_vm<(D - 1) * NIN>();
            publish();
          }
        }
      }
      ring_wait_vm<0>();
      while (pub < p) publish();
      // the positions the consumers may expect: all issued, or (stopped) every
      // position of the batches claimed, once the claimer has recorded its
      // last one (it stops promptly after BYPASS; hang cap only)
      if (stop) {
        unsigned spins = 0;
        while (ring_flag_ld(&claimer_done) == 0u && ++spins < RING_HANG_CAP(L)) __builtin_amdgcn_s_sleep(1);
        if (spins >= RING_HANG_CAP(L) && lane == 0 && L.fault) RING_HANG_FAULT(L);
      }
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
        while (n >= ring_flag_ld(&lbatch) + 1 + kLook && ring_flag_ld(&bypass) == 0u && ++spins < cap)
          __builtin_amdgcn_s_sleep(2);
        if (ring_flag_ld(&bypass) != 0u || spins >= cap) {
          if (spins >= cap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
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
#if REDSET_HIP_TEST_KNOBS
        // test builds: widen the window between claiming and recording
        for (unsigned d = 0; d < L.claim_delay; ++d) __builtin_amdgcn_s_sleep(127);
#endif
        if (lane == 0) {
          ring_flag_st(&bbase[n % NB], bb);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          ring_flag_st(&nclaimed, n + 1);
        }
      }
      // every batch this wave took from the queue is recorded
      if (lane == 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        ring_flag_st(&claimer_done, 1u);
      }
    }
  } else {
    // consumers: positions c, c + C, ... of the block's sequence
    const int c = wave - 2;
    typename Pol::Body body;
    Pol::init(body, lds);
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
        if (ring_flag_ld(&bypass) != 0u || ++spins >= cap) {
          direct = true;
          break;
        }
        __builtin_amdgcn_s_sleep(kRingSleep);
      }
      if (done) break;
      unsigned u;
      if (!direct) {
        // claimed, and its bbase entry cannot be reused before this position is released
        u = ring_flag_ld(&bbase[(p / B) % NB]) + p % B;
      } else {
        if (spins >= cap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
        // the position's item from its batch's base once the batch is claimed;
        // a batch is never claimed once the queue is empty (claim_end) or the
        // claimer is done (after BYPASS): then this sequence ends here.
        // Nothing else keeps the claim back, so the wait ends (hang cap only)
        unsigned s3 = 0;
        while (ring_flag_ld(&nclaimed) <= p / B && ring_flag_ld(&claim_end) > p / B &&
               ring_flag_ld(&claimer_done) == 0u && ++s3 < RING_HANG_CAP(L))
          __builtin_amdgcn_s_sleep(1);
        if (s3 >= RING_HANG_CAP(L) && lane == 0 && L.fault) RING_HANG_FAULT(L);
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
        Pol::set_out(body, jobs + jn);
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
        while (ring_flag_ld(&freed[p % S]) + 1u < want && ++s2 < cap) __builtin_amdgcn_s_sleep(1);
        if (lane == 0 && ring_flag_ld(&freed[p % S]) + 1u >= want) ring_flag_st(&freed[p % S], want);
        const size_t vc = ok ? v : nvec - 1;
#pragma unroll
        for (int i = 0; i < NIN; ++i) x[i] = ring_direct_load(in[i] + vc);
      }
      // this job's tables: wait for them unless the loader has stopped
      bool tables = true;
      if (Pol::kTables && ring_flag_ld(&tab_job) < job) {
        unsigned s4 = 0;
        while (ring_flag_ld(&tab_job) < job && ring_flag_ld(&bypass) == 0u && ++s4 < cap)
          __builtin_amdgcn_s_sleep(kRingSleep);
        tables = ring_flag_ld(&tab_job) >= job;
      }
      if (ok) {
        if (tables) Pol::combine(body, x, job, v);
        else Pol::slow(jobs + job, in, v);
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
          if (row_ok(u) && v < nvec) Pol::slow(jobs + job, jin, v);
        }
      }
    }
  }
}

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


// XOR claimed launches (claimed_sweep): no tables; one-row positions in the
// XOR kernels' own ring array (xor_lds, shared with xor_body: two-row items
// of <= 8 inputs there, so twice the slots here). A twin-only order: it
// measured 8% slower than a launch per stripe (redset_hip.cpp
// xor_claim_default)
template <int NIN_, bool ACC>
struct XorClaim {
  static constexpr int NIN = NIN_;
  static_assert(NIN <= kRingChunk, "claimed XOR of <= 8 inputs");
  static constexpr int kRows = NIN > kRingXorWide ? 1 : kRingXorRows;  // xor_body's items
  static constexpr bool kTables = false;
  static constexpr int kSlots = ring_vecs<NIN, kRows>() / (NIN * 64);
  static constexpr int kRingOff = 0;
  using Launch = XorLaunch;
  using Job = XorJob;
  using Body = XorAcc<ACC>;
  typedef __attribute__((address_space(4))) const XorJob c_job;
  static __device__ __forceinline__ v4u* lds() { return xor_lds<NIN, kRows>(); }
  static __device__ __forceinline__ void init(Body&, const uint32_t*) {}
  static __device__ __forceinline__ void set_out(Body& b, const c_job* J) { b.out = (g_u4*) (J->out); }
  static __device__ __forceinline__ void first_tables(uint32_t*, const c_job*, unsigned) {}
  static __device__ __forceinline__ void next_tables(uint32_t*, const c_job*, unsigned, int) {}
  static __device__ __forceinline__ void combine(Body& b, const v4u (&x)[NIN], unsigned, size_t v) {
    b.begin();
    b.template add<0>(x);
    b.finish(v);
  }
  static __device__ __forceinline__ void slow(const c_job* J, g_cu4* const (&in)[NIN], size_t v) {
    v4u r = ring_direct_load(in[0] + v);
#pragma unroll
    for (int i = 1; i < NIN; ++i) r ^= ring_direct_load(in[i] + v);
    g_u4* o = (g_u4*) (J->out);
    if constexpr (ACC) o[v] = r ^ o[v];
    else store_vec(o, v, r);
  }
};

template <int NIN, bool ACC>
__device__ __forceinline__ void xor_stream(const XorLaunch& L) {
  constexpr int R = NIN > kRingXorWide ? 1 : kRingXorRows;
  constexpr int D = ring_depth<NIN, R, R == 1 ? kRingXorRowsInFlight : kRingRowsInFlight>();
  constexpr int S = ring_slots<NIN * R>();
  constexpr int C = kBlock / 64 - 1;
  static_assert(D >= 2 && D - 1 < S && (D - 1) * NIN * R <= 63, "ring depth");
  typedef __attribute__((address_space(4))) const XorJob c_job;
  const c_job* const jobs = (const c_job*) (L.jobs + L.job0);
  const unsigned cap = RING_SPIN_CAP(L);
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
        ring_wait_vm<0>();
        while (pub < g) publish();
        unsigned spins = 0;
        while (ring_flag_ld(&freed[g % S]) < use && ++spins < cap) __builtin_amdgcn_s_sleep(1);
        if (spins >= cap) {
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
        for (int i = 0; i < NIN; ++i)
          ring_dma((g_cu4*) (in[i]) + vc, slot + static_cast<uint32_t>((i * R + r) * 1024));
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
      if (ring_flag_ld(&bypass) != 0u || ++spins >= cap) {
        direct = true;
        break;
      }
      __builtin_amdgcn_s_sleep(kRingSleep);
    }
    if (direct) {
      // as in ring_sweep
      if (spins >= cap && lane == 0 && L.fault) atomicAdd(L.fault, 1u);
      unsigned s2 = 0;
      while (ring_flag_ld(&freed[g % S]) + 1u < want && ++s2 < cap) __builtin_amdgcn_s_sleep(1);
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

template <int NIN, bool ACC>
__device__ __forceinline__ void xor_body(const XorLaunch& L, const XorJob& J, int part) {
  const size_t nvec = L.bytes_only ? 0 : L.nbytes / 16;
  const size_t vstep = static_cast<size_t>(L.blocks_per_job) * kBlock;
  if (nvec > 0) {
    g_cu4* in[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) in[i] = (g_cu4*) (J.in[i]);
    // two-row items hold 2 * NIN input vectors per lane: past 8 inputs that
    // no longer fits 1024-thread blocks' 128 VGPRs, so wide XOR sets take
    // the GF kernels' one-row shape
    constexpr int kRows = NIN > kRingXorWide ? 1 : kRingXorRows;
    constexpr int kDepth = ring_depth<NIN, kRows, kRows == 1 ? kRingXorRowsInFlight : kRingRowsInFlight>();
    v4u* const ring = xor_lds<NIN, kRows>();
    XorAcc<ACC> body;
    body.out = (g_u4*) (J.out);
    ring_sweep<NIN, kRows, kDepth>(ring, in, nvec, static_cast<size_t>(L.blocks_per_job), static_cast<size_t>(part),
                                   L.fault, RING_SPIN_CAP(L), body);
  }
  const size_t tail0 = nvec * 16;
  for (size_t k = tail0 + static_cast<size_t>(part) * kBlock + threadIdx.x; k < L.nbytes; k += vstep) {
    uint8_t r = ACC ? J.out[k] : 0;
#pragma unroll
    for (int i = 0; i < NIN; ++i) r ^= J.in[i][k];
    J.out[k] = r;
  }
}

// entry points: jobs from a device array (plans), or one job passed by
// value in the kernel arguments (stripe primitives, no device descriptor)
template <int NIN, int NOUT, bool ACC>
REDSET_KERNEL gf_mac_kernel(GfLaunch L) {
  if constexpr (NIN <= 8) {
    if (L.sequential == kJobsStreamed && !L.bytes_only && L.nbytes % 16 == 0) {
      gf_mac_stream<NIN, NOUT, ACC>(L);
      return;
    }
    if (L.sequential == kJobsClaimed && L.claim && !L.bytes_only && L.nbytes % 16 == 0) {
      claimed_sweep<GfClaim<NIN, NOUT, ACC>>(L);
      return;
    }
  }
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
  gf_mac_body<NIN, NOUT, ACC>(L, L.jobs[L.job0 + job], blockIdx.x - job * L.blocks_per_job);
}

template <int NIN, int NOUT, bool ACC>
REDSET_KERNEL gf_mac_kernel_arg(GfLaunch L, GfJob J) {
  gf_mac_body<NIN, NOUT, ACC>(L, J, blockIdx.x);
}

template <int NIN, bool ACC>
REDSET_KERNEL xor_kernel(XorLaunch L) {
  if constexpr (NIN <= kRingChunk) {
    if (L.sequential == kJobsStreamed && !L.bytes_only && L.nbytes % 16 == 0) {
      xor_stream<NIN, ACC>(L);
      return;
    }
    if (L.sequential == kJobsClaimed && L.claim && !L.bytes_only && L.nbytes % 16 == 0) {
      claimed_sweep<XorClaim<NIN, ACC>>(L);
      return;
    }
  }
  if (L.sequential == kJobsInKernel || L.sequential == kJobsStreamed || L.sequential == kJobsClaimed) {
    for (int j = 0; j < L.njobs; ++j) xor_body<NIN, ACC>(L, L.jobs[L.job0 + j], blockIdx.x);
    return;
  }
  const int job = blockIdx.x / L.blocks_per_job;
  xor_body<NIN, ACC>(L, L.jobs[L.job0 + job], blockIdx.x - job * L.blocks_per_job);
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
