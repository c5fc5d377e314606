// redset_hip.cpp -- C ABI (include/redset_hip.h): GF state, whole-set plans
// for RS / XOR encode and rebuild, and stripe primitives.
//
// A plan turns the reference's per-rank, per-slice loops (encode:
// src/redset_reedsolomon.c:309-391, decode: :631-768, XOR: src/redset_xor.c:
// 243-288, src/redset_xor_serial.c:202-273) into a few kernel launches over
// whole cells: one job per stripe, each reading its input cells once and
// writing its output cells once. Planning happens once on the host; execute
// only enqueues kernels, so it can be captured into a hipGraph.
#include "redset_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <tuple>
#include <vector>

#include "codec_kernels.h"
#include "gf256.h"
#include "stripe_map.h"

using redset_hip::CellRef;
using redset_hip::fail;
using redset_hip::GfJob;
using redset_hip::GfLaunch;
using redset_hip::kMaxIn;
using redset_hip::kMaxOut;
using redset_hip::StripeMap;
using redset_hip::XorJob;
using redset_hip::XorLaunch;

// widest stripe primitive call: p + e <= 256 bounds any redset stripe
constexpr int kMaxCombine = 256;

struct redset_hip_plan {
  redset_hip_plan_info info{};
  GfJob* d_gf = nullptr;  // device job arrays
  XorJob* d_xor = nullptr;
  unsigned* d_claim = nullptr;  // kJobsClaimed launches' queue counters
  std::vector<GfLaunch> gf_launches;
  std::vector<XorLaunch> xor_launches;
};

namespace {

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return REDSET_SUCCESS;
  return fail("%s: %s", what, hipGetErrorString(e));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Test builds only (REDSET_HIP_TEST_KNOBS, codec_kernels.h): an environment
// override of a planning choice; the product library always takes `dflt`.
// Read at every plan build.
int test_knob(const char* name, int dflt) {
#if REDSET_HIP_TEST_KNOBS
  const char* s = std::getenv(name);
  if (s && s[0] >= '0' && s[0] <= '9') return std::atoi(s);
#else
  (void) name;
#endif
  return dflt;
}

// Resident blocks per CU the codec aims for: one block of the ring's 1024
// threads (1 loader + 15 consumer waves, codec_kernels.h), alone on the CU
// (it takes 146 KiB of LDS).
int target_blocks_per_cu(int occupancy) { return std::max(1, std::min(1, occupancy)); }

// Resident XOR blocks per CU: one, as for gf_mac (the ring's block fills the
// CU's LDS; with the per-wave sweep before it, one 256-thread block per CU
// also beat two, profiles/r01_ab_xor_blocks.txt).
int xor_blocks_cap() { return 1; }

// Job order of a plan's launches (codec_kernels.h). Stripes in sequence, one
// launch each over the whole grid (kJobsInLaunches), keep one stripe's ~11
// cell streams in flight instead of every stripe's ~120: +6.5% on the 64 MiB
// RS(8+3) step; two or three stripes per launch cost 3% / 6%, and one launch
// looping over the stripes (kJobsInKernel) 5% (profiles/r01_sequential_jobs.txt).
// Each launch pays a ramp-up and a drain, so sequence only pays for big cells:
// side by side wins at 16 MiB cells (5.30 vs 5.14 TB/s), sequence at 24 MiB
// (5.43 vs 5.16) and 32 MiB (5.46 vs 5.11); grouping 2-6 stripes per launch
// never beats both (profiles/r01_sequential_jobs.txt, cell-size sweeps). Sets
// with smaller cells keep their stripes side by side in one launch (0).
// Round 3, with the loader ring: GF stripes of <= 8 inputs over whole 16-B
// vectors (RS(8+3) encode and rebuild) run all in ONE launch whose blocks
// claim their items at run time (kJobsClaimed, codec_device.h
// gf_mac_claimed): one continuous loader ring per block over all the
// stripes, the blocks of each XCD sweeping its rows together, so no launch
// gaps, one tail per set instead of per stripe, and no drift between blocks:
// +3.5% on the RS(8+3) step against one launch per stripe, +1.5% against
// streamed pairs. Streamed (kJobsStreamed, static items) pays off only in
// pairs (+1.5..2.5%): with more stripes per launch the blocks drift apart
// and sweep different stripes at once (all 11: -3.5%); it stays the order of
// XOR A/B runs (profiles/r03_ab_stream.txt).
// Test builds: REDSET_HIP_SEQUENTIAL=0..4 forces an order (XOR launches take
// 1 for 4); REDSET_HIP_STREAM_JOBS sets the stripes per streamed or claimed
// launch (0 = all), REDSET_HIP_STRIPES_PER_LAUNCH those side by side per
// launch in sequence mode.
constexpr size_t kSequentialMinCell = 24u << 20;

// can_stream: the kernel has a streamed path for these jobs (GF: <= 8
// inputs, XOR: <= 8 inputs, both over whole 16-B vectors); can_claim: a
// claimed one (the same jobs: GF and XOR of <= 8 inputs over whole 16-B
// vectors; XOR claiming is off by default, xor_claim_default);
// claim_default / stream_default: which is the default for big cells.
int sequential_jobs(int njobs, size_t nbytes, bool can_stream, bool can_claim, bool claim_default,
                     bool stream_default) {
  if (njobs < 2) return 0;
  int order = nbytes >= kSequentialMinCell
                  ? (can_claim && claim_default ? redset_hip::kJobsClaimed
                     : can_stream && stream_default ? redset_hip::kJobsStreamed
                                                    : redset_hip::kJobsInLaunches)
                  : 0;
  const int forced = test_knob("REDSET_HIP_SEQUENTIAL", -1);
  if (forced >= 0 && forced <= 4) order = forced;
  if ((order == redset_hip::kJobsStreamed && !can_stream) || (order == redset_hip::kJobsClaimed && !can_claim))
    order = redset_hip::kJobsInLaunches;
  return order;
}

// Stripes per launch: in sequence mode side by side within the launch
// (default 1); streamed, two stripes one after another through the ring;
// claimed, the whole set in one launch (0 = all).
int stripes_per_launch(int order) {
  if (order == redset_hip::kJobsStreamed || order == redset_hip::kJobsClaimed)
    return test_knob("REDSET_HIP_STREAM_JOBS", order == redset_hip::kJobsClaimed ? 0 : 2);
  return std::max(1, test_knob("REDSET_HIP_STRIPES_PER_LAUNCH", 1));
}

// XOR plans keep a launch per stripe: streamed pairs (xor_stream) measured
// within the XOR leg's run-to-run spread, 6.26 against 6.30 TB/s over three
// alternating pairs (profiles/r03_ab_stream.txt). Test builds:
// REDSET_HIP_XOR_STREAM=1 streams them in pairs.
bool xor_stream_default() { return test_knob("REDSET_HIP_XOR_STREAM", 0) == 1; }

// XOR plans with claimed items (claimed_sweep, one launch per set): a measured
// negative, kept as a twin-only order (REDSET_HIP_XOR_CLAIM=1 or
// REDSET_HIP_SEQUENTIAL=4) the suite checks bit for bit: the XOR leg 5.60
// against 5.98-6.09 TB/s. Its one-row items and claim bookkeeping cost +27%
// SALU, +44% VALU and +54% LDS instructions per byte at equal HBM traffic,
// and with consumers this light the loader's per-item instruction stream sets
// the pace (profiles/r04s5_ab_xor_claim.txt, r04s6_xor_claim_pmc_sq.txt)
bool xor_claim_default() { return test_knob("REDSET_HIP_XOR_CLAIM", 0) == 1; }

int launches_of(int order, int njobs, int group) {
  if (order == redset_hip::kJobsStreamed || order == redset_hip::kJobsClaimed)
    return group > 0 ? (njobs + group - 1) / group : 1;
  return order == redset_hip::kJobsInLaunches ? (njobs + group - 1) / group : 1;
}

// jobs that share one launch's grid
int jobs_sharing_grid(int order, int njobs, int group) {
  return order == redset_hip::kJobsInLaunches                                            ? std::min(group, njobs)
         : (order == redset_hip::kJobsInKernel || order == redset_hip::kJobsStreamed ||
            order == redset_hip::kJobsClaimed)
             ? 1
                                                                                       : njobs;
}

// Blocks per job so the whole launch fits in one resident wave of blocks.
int blocks_per_job(int njobs, size_t nbytes, int occupancy, int blocks_total = 0) {
  const long target = blocks_total > 0
                          ? blocks_total
                          : static_cast<long>(redset_hip::device_cu_count()) * target_blocks_per_cu(occupancy);
  long bpj = std::max<long>(1, target / std::max(1, njobs));
  // at least one 16-B vector per thread per block
  const long vec_blocks = static_cast<long>((nbytes / 16 + redset_hip::kBlock - 1) / redset_hip::kBlock);
  bpj = std::min(bpj, std::max<long>(1, vec_blocks));
  return static_cast<int>(bpj);
}

// Device address of a cell in the set layout of include/redset_hip.h.
struct SetLayout {
  unsigned char* const* lofi;
  unsigned char* const* parity;
  size_t stride;
  uint8_t* at(const CellRef& c) const {
    return (c.kind == redset_hip::kData ? lofi[c.rank] : parity[c.rank]) + static_cast<size_t>(c.index) * stride;
  }
};

// Split stripe maps into launches of <= kMaxIn inputs x <= kMaxOut outputs.
// Output groups are independent; input groups of one output group run in
// order, the first overwriting and the rest accumulating. Jobs with equal
// shapes share a launch. XOR maps go to the XOR kernel.
int build_plan(redset_hip_plan* plan, const std::vector<StripeMap>& maps, const SetLayout& L, size_t nbytes) {
  struct GfPending {
    std::vector<GfJob> jobs;
    int nin, nout, accumulate, bytes_only;
  };
  struct XorPending {
    std::vector<XorJob> jobs;
    int nin, accumulate, bytes_only;
  };
  // (input group, nin, nout, unaligned, accumulate) / (input group, nin, unaligned, accumulate)
  std::map<std::tuple<int, int, int, int, int>, GfPending> gf;
  std::map<std::tuple<int, int, int, int>, XorPending> xr;
  unsigned long long rd = 0, wr = 0;
  for (const StripeMap& m : maps) {
    const int nin = static_cast<int>(m.in.size());
    const int nt = static_cast<int>(m.out.size());
    if (nt == 0) continue;
    if (nin == 0) return fail("stripe with outputs but no inputs");
    for (int og = 0; og * kMaxOut < nt; ++og) {
      const int o0 = og * kMaxOut, no = std::min(kMaxOut, nt - o0);
      if (m.xor_only && no != 1) return fail("XOR stripe with %d outputs", no);
      for (int ig = 0; ig * kMaxIn < nin; ++ig) {
        const int i0 = ig * kMaxIn, ni = std::min(kMaxIn, nin - i0);
        bool al = true;
        const int acc = ig > 0 || m.accumulate;
        rd += static_cast<unsigned long long>(ni + (acc ? no : 0)) * nbytes;
        wr += static_cast<unsigned long long>(no) * nbytes;
        if (m.xor_only) {
          XorJob J;
          std::memset(&J, 0, sizeof(J));
          for (int i = 0; i < ni; ++i) {
            J.in[i] = L.at(m.in[i0 + i]);
            al = al && aligned16(J.in[i]);
          }
          J.out = L.at(m.out[o0]);
          al = al && aligned16(J.out);
          XorPending& P = xr[std::make_tuple(ig, ni, al ? 0 : 1, acc)];
          P.nin = ni;
          P.accumulate = acc;
          P.bytes_only = al ? 0 : 1;
          P.jobs.push_back(J);
          continue;
        }
        GfJob J;
        std::memset(&J, 0, sizeof(J));
        for (int i = 0; i < ni; ++i) {
          J.in[i] = L.at(m.in[i0 + i]);
          al = al && aligned16(J.in[i]);
        }
        for (int j = 0; j < no; ++j) {
          J.out[j] = L.at(m.out[o0 + j]);
          al = al && aligned16(J.out[j]);
          for (int i = 0; i < ni; ++i) J.coef[j][i] = m.coef[static_cast<size_t>(o0 + j) * nin + i0 + i];
        }
        GfPending& P = gf[std::make_tuple(ig, ni, no, al ? 0 : 1, acc)];
        P.nin = ni;
        P.nout = no;
        P.accumulate = acc;
        P.bytes_only = al ? 0 : 1;
        P.jobs.push_back(J);
      }
    }
  }
  plan->info.bytes_read = rd;
  plan->info.bytes_written = wr;
  std::vector<GfJob> gall;
  std::vector<XorJob> xall;
  for (auto& kv : gf) {
    GfPending& P = kv.second;
    GfLaunch G;
    std::memset(&G, 0, sizeof(G));
    G.jobs = reinterpret_cast<const GfJob*>(gall.size());  // offset, patched below
    G.njobs = static_cast<int>(P.jobs.size());
    G.nin = P.nin;
    G.nout = P.nout;
    G.accumulate = P.accumulate;
    G.bytes_only = P.bytes_only;
    G.nbytes = nbytes;
    const bool whole = P.nin <= 8 && !P.bytes_only && nbytes % 16 == 0;
    // claimed items for 3-4 outputs (the RS(8+3) encode: 6.45-6.47 TB/s against
    // 6.22-6.27 streamed in pairs on two boxes); pairs for 1-2 (the rebuild:
    // 6.35-6.41 against 5.99-6.33 claimed; its lighter consumers leave the
    // loader, whose per-item cost the claimed order raises, setting the pace)
    G.sequential = sequential_jobs(G.njobs, nbytes, whole, whole, P.nout >= 3, true);
    G.group = stripes_per_launch(G.sequential);
    G.blocks_per_job = blocks_per_job(jobs_sharing_grid(G.sequential, G.njobs, G.group), nbytes,
                                      redset_hip::gf_blocks_per_cu(P.nin));
    gall.insert(gall.end(), P.jobs.begin(), P.jobs.end());
    plan->gf_launches.push_back(G);
  }
  for (auto& kv : xr) {
    XorPending& P = kv.second;
    XorLaunch X;
    std::memset(&X, 0, sizeof(X));
    X.jobs = reinterpret_cast<const XorJob*>(xall.size());
    X.njobs = static_cast<int>(P.jobs.size());
    X.nin = P.nin;
    X.accumulate = P.accumulate;
    X.bytes_only = P.bytes_only;
    X.nbytes = nbytes;
    const bool whole = P.nin <= 8 && !P.bytes_only && nbytes % 16 == 0;
    X.sequential = sequential_jobs(X.njobs, nbytes, whole, whole, xor_claim_default(), xor_stream_default());
    X.group = stripes_per_launch(X.sequential);
    X.blocks_per_job = blocks_per_job(jobs_sharing_grid(X.sequential, X.njobs, X.group), nbytes, xor_blocks_cap());
    xall.insert(xall.end(), P.jobs.begin(), P.jobs.end());
    plan->xor_launches.push_back(X);
  }
  plan->info.jobs = static_cast<int>(gall.size() + xall.size());
  plan->info.launches = 0;
  for (const GfLaunch& G : plan->gf_launches) plan->info.launches += launches_of(G.sequential, G.njobs, G.group);
  for (const XorLaunch& X : plan->xor_launches) plan->info.launches += launches_of(X.sequential, X.njobs, X.group);
  if (!gall.empty()) {
    if (int rc = hip_check(hipMalloc(&plan->d_gf, gall.size() * sizeof(GfJob)), "hipMalloc(plan jobs)")) return rc;
    if (int rc = hip_check(hipMemcpy(plan->d_gf, gall.data(), gall.size() * sizeof(GfJob), hipMemcpyHostToDevice),
                           "hipMemcpy(plan jobs)"))
      return rc;
    for (GfLaunch& G : plan->gf_launches) G.jobs = plan->d_gf + reinterpret_cast<uintptr_t>(G.jobs);
  }
  // claimed launches (the kernel takes them over whole 16-B vectors and <= 8
  // inputs only, as the streamed ones): their queue counters, zeroed
  size_t nclaim = 0;
  for (GfLaunch& G : plan->gf_launches)
    if (G.sequential == redset_hip::kJobsClaimed) ++nclaim;
  for (XorLaunch& X : plan->xor_launches)
    if (X.sequential == redset_hip::kJobsClaimed) ++nclaim;
  if (nclaim > 0) {
    const size_t bytes = nclaim * redset_hip::kClaimWords * sizeof(unsigned);
    if (int rc = hip_check(hipMalloc(&plan->d_claim, bytes), "hipMalloc(claim queues)")) return rc;
    if (int rc = hip_check(hipMemset(plan->d_claim, 0, bytes), "hipMemset(claim queues)")) return rc;
    size_t k = 0;
    for (GfLaunch& G : plan->gf_launches)
      if (G.sequential == redset_hip::kJobsClaimed) G.claim = plan->d_claim + (k++) * redset_hip::kClaimWords;
    for (XorLaunch& X : plan->xor_launches)
      if (X.sequential == redset_hip::kJobsClaimed) X.claim = plan->d_claim + (k++) * redset_hip::kClaimWords;
  }
  if (!xall.empty()) {
    if (int rc = hip_check(hipMalloc(&plan->d_xor, xall.size() * sizeof(XorJob)), "hipMalloc(plan jobs)")) return rc;
    if (int rc = hip_check(hipMemcpy(plan->d_xor, xall.data(), xall.size() * sizeof(XorJob), hipMemcpyHostToDevice),
                           "hipMemcpy(plan jobs)"))
      return rc;
    for (XorLaunch& X : plan->xor_launches) X.jobs = plan->d_xor + reinterpret_cast<uintptr_t>(X.jobs);
  }
  return REDSET_SUCCESS;
}

int check_set_args(const void* const* a, const void* const* b, int ranks, size_t chunk_size, size_t stride,
                   redset_hip_plan** out) {
  if (!out) return fail("null plan out-pointer");
  *out = nullptr;
  if (!a || !b) return fail("null member pointer array");
  for (int r = 0; r < ranks; ++r)
    if (!a[r] || !b[r]) return fail("null device pointer for member %d", r);
  if (stride < chunk_size) return fail("cell_stride (%zu) < chunk_size (%zu)", stride, chunk_size);
  return REDSET_SUCCESS;
}

int finish_plan(int kind, int ranks, int encoding, int missing, size_t chunk, const std::vector<StripeMap>& maps,
                const SetLayout& L, redset_hip_plan** out) {
  redset_hip_plan* plan = new (std::nothrow) redset_hip_plan;
  if (!plan) return fail("out of host memory");
  plan->info.kind = kind;
  plan->info.ranks = ranks;
  plan->info.encoding = encoding;
  plan->info.missing = missing;
  plan->info.chunk_size = chunk;
  if (int rc = build_plan(plan, maps, L, chunk)) {
    redset_hip_plan_destroy(plan);
    return rc;
  }
  *out = plan;
  return REDSET_SUCCESS;
}

}  // namespace

namespace redset_hip {

int run_stripe(const StripeMap& m, const uint8_t* const* in, uint8_t* const* out, size_t nbytes, void* stream,
               int blocks_total, bool accumulate) {
  const int nin = static_cast<int>(m.in.size()), nt = static_cast<int>(m.out.size());
  for (int og = 0; og * kMaxOut < nt; ++og) {
    const int o0 = og * kMaxOut, no = std::min(kMaxOut, nt - o0);
    for (int ig = 0; ig * kMaxIn < nin; ++ig) {
      const int i0 = ig * kMaxIn, ni = std::min(kMaxIn, nin - i0);
      bool al = true;
      int e;
      if (m.xor_only) {
        XorJob J;
        std::memset(&J, 0, sizeof(J));
        for (int i = 0; i < ni; ++i) {
          J.in[i] = in[i0 + i];
          al = al && aligned16(J.in[i]);
        }
        J.out = out[o0];
        al = al && aligned16(J.out);
        XorLaunch X;
        std::memset(&X, 0, sizeof(X));
        X.njobs = 1;
        X.nin = ni;
        X.accumulate = accumulate || ig > 0;
        X.bytes_only = al ? 0 : 1;
        X.nbytes = nbytes;
        X.blocks_per_job = blocks_per_job(1, nbytes, xor_blocks_cap(), blocks_total);
        e = launch_xor_single(X, J, stream);
      } else {
        GfJob J;
        std::memset(&J, 0, sizeof(J));
        for (int i = 0; i < ni; ++i) {
          J.in[i] = in[i0 + i];
          al = al && aligned16(J.in[i]);
        }
        for (int j = 0; j < no; ++j) {
          J.out[j] = out[o0 + j];
          al = al && aligned16(J.out[j]);
          for (int i = 0; i < ni; ++i) J.coef[j][i] = m.coef[static_cast<size_t>(o0 + j) * nin + i0 + i];
        }
        GfLaunch G;
        std::memset(&G, 0, sizeof(G));
        G.njobs = 1;
        G.nin = ni;
        G.nout = no;
        G.accumulate = accumulate || ig > 0;
        G.bytes_only = al ? 0 : 1;
        G.nbytes = nbytes;
        G.blocks_per_job = blocks_per_job(1, nbytes, gf_blocks_per_cu(ni), blocks_total);
        e = launch_gf_single(G, J, stream);
      }
      if (e) return hip_check(static_cast<hipError_t>(e), "stripe kernel launch");
    }
  }
  return REDSET_SUCCESS;
}

}  // namespace redset_hip

extern "C" {

int redset_hip_test_build(void) { return redset_hip::test_knobs(); }

int redset_hip_ring_faults(unsigned* count, int clear) {
  if (!count) return fail("ring_faults: null argument");
  return hip_check(static_cast<hipError_t>(redset_hip::read_ring_faults(count, clear)), "ring_faults");
}
int redset_hip_hang_faults(void* stream, unsigned* count, int clear) {
  if (!count) return fail("hang_faults: null argument");
  return hip_check(static_cast<hipError_t>(redset_hip::read_hang_faults(stream, count, clear)), "hang_faults");
}
const char* redset_hip_last_error(void) { return redset_hip::last_error(); }
int redset_hip_record_error(const char* msg) { return fail("%s", msg ? msg : "unknown error"); }

int redset_hip_rs_shape(const redset_hip_rs* rs, int* ranks, int* encoding) {
  if (!rs) return fail("rs_shape: null codec");
  if (ranks) *ranks = rs->ranks;
  if (encoding) *encoding = rs->encoding;
  return REDSET_SUCCESS;
}
const char* redset_hip_version(void) { return "redset-hip 0.3 (gfx950)"; }
int redset_hip_abi_version(void) { return REDSET_HIP_ABI_VERSION; }

int redset_hip_rs_create(int ranks, int encoding, redset_hip_rs** out) {
  if (!out) return fail("null out-pointer");
  *out = nullptr;
  // same rules as redset_construct_rs, src/redset_reedsolomon.c:158-185
  if (encoding < 1 || encoding >= ranks) return fail("invalid encoding %d for %d ranks", encoding, ranks);
  if (ranks + encoding > 256) return fail("ranks + encoding = %d exceeds GF(2^8)", ranks + encoding);
  redset_hip_rs* rs = new (std::nothrow) redset_hip_rs;
  if (!rs) return fail("out of host memory");
  rs->ranks = ranks;
  rs->encoding = encoding;
  rs->mat = redset_hip::encoding_matrix(ranks, encoding);
  *out = rs;
  return REDSET_SUCCESS;
}

void redset_hip_rs_destroy(redset_hip_rs* rs) { delete rs; }

int redset_hip_rs_matrix(const redset_hip_rs* rs, unsigned char* mat_out) {
  if (!rs || !mat_out) return fail("null argument");
  std::memcpy(mat_out, rs->mat.data(), rs->mat.size());
  return REDSET_SUCCESS;
}

int redset_hip_rs_get_encoding_id(int ranks, int encoding, int rank, int chunk_id) {
  return redset_hip::encoding_id(ranks, encoding, rank, chunk_id);
}

int redset_hip_rs_get_data_id(int ranks, int encoding, int rank, int chunk_id) {
  return redset_hip::data_id(ranks, encoding, rank, chunk_id);
}

int redset_hip_rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int chunk_id,
                                unsigned char* coef_out) {
  if (!rs || !coef_out || !rebuild_ranks) return fail("null argument");
  if (chunk_id < 0 || chunk_id >= rs->ranks) return fail("chunk id %d out of range", chunk_id);
  std::vector<uint8_t> D;
  if (int rc = redset_hip::rs_decode_matrix(rs, missing, rebuild_ranks, chunk_id, D)) return rc;
  std::memcpy(coef_out, D.data(), D.size());
  return REDSET_SUCCESS;
}

size_t redset_hip_cell_stride(size_t chunk_size) {
  constexpr size_t kAlign = 256, kPad = size_t(16) << 20;
  size_t stride = (chunk_size + kAlign - 1) / kAlign * kAlign;
  if (stride == 0) stride = kAlign;
  if (stride % kPad == 0) stride += kPad;
  return stride;
}

int redset_hip_rs_plan_encode(const redset_hip_rs* rs, unsigned char* const* lofi, unsigned char* const* parity,
                              size_t chunk_size, size_t stride, redset_hip_plan** out) {
  if (!rs) return fail("null rs state");
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(parity),
                              rs->ranks, chunk_size, stride, out))
    return rc;
  std::vector<StripeMap> maps(rs->ranks);
  for (int c = 0; c < rs->ranks; ++c) redset_hip::rs_encode_map(rs, c, maps[c]);
  return finish_plan(REDSET_HIP_PLAN_RS_ENCODE, rs->ranks, rs->encoding, 0, chunk_size, maps,
                     SetLayout{lofi, parity, stride}, out);
}

int redset_hip_rs_plan_rebuild(const redset_hip_rs* rs, int missing, const int* rebuild_ranks,
                               unsigned char* const* lofi, unsigned char* const* parity, size_t chunk_size,
                               size_t stride, redset_hip_plan** out) {
  if (!rs) return fail("null rs state");
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(parity),
                              rs->ranks, chunk_size, stride, out))
    return rc;
  if (missing < 0 || missing > rs->encoding)
    return fail("cannot rebuild %d members with %d parity chunks", missing, rs->encoding);
  if (missing > 0 && !rebuild_ranks) return fail("null rebuild_ranks");
  std::vector<StripeMap> maps;
  for (int c = 0; c < rs->ranks && missing > 0; ++c) {
    StripeMap m;
    if (int rc = redset_hip::rs_rebuild_map(rs, missing, rebuild_ranks, c, m)) return rc;
    maps.push_back(std::move(m));
  }
  return finish_plan(REDSET_HIP_PLAN_RS_REBUILD, rs->ranks, rs->encoding, missing, chunk_size, maps,
                     SetLayout{lofi, parity, stride}, out);
}

int redset_hip_xor_plan_encode(int ranks, unsigned char* const* lofi, unsigned char* const* xorc, size_t chunk_size,
                               size_t stride, redset_hip_plan** out) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(xorc),
                              ranks, chunk_size, stride, out))
    return rc;
  std::vector<StripeMap> maps(ranks);
  for (int c = 0; c < ranks; ++c) redset_hip::xor_encode_map(ranks, c, maps[c]);
  return finish_plan(REDSET_HIP_PLAN_XOR_ENCODE, ranks, 1, 0, chunk_size, maps, SetLayout{lofi, xorc, stride}, out);
}

int redset_hip_xor_plan_rebuild(int ranks, int root, unsigned char* const* lofi, unsigned char* const* xorc,
                                size_t chunk_size, size_t stride, redset_hip_plan** out) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  if (root < 0 || root >= ranks) return fail("root %d out of range", root);
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(xorc),
                              ranks, chunk_size, stride, out))
    return rc;
  std::vector<StripeMap> maps(ranks);
  for (int c = 0; c < ranks; ++c) redset_hip::xor_rebuild_map(ranks, root, c, maps[c]);
  return finish_plan(REDSET_HIP_PLAN_XOR_REBUILD, ranks, 1, 1, chunk_size, maps, SetLayout{lofi, xorc, stride}, out);
}

int redset_hip_plan_combine(const redset_hip_combine_job* jobs, int njobs, size_t nbytes, redset_hip_plan** out) {
  if (!out) return fail("plan_combine: null out-pointer");
  *out = nullptr;
  if (njobs < 0 || (njobs > 0 && !jobs)) return fail("plan_combine: bad job list");
  // every job's cells as entries of one pointer table, so the set planner
  // (build_plan) takes them as cells of a layout with stride 0: cell
  // (rank = table index, index 0)
  std::vector<unsigned char*> table;
  std::vector<StripeMap> maps(static_cast<size_t>(njobs));
  for (int k = 0; k < njobs; ++k) {
    const redset_hip_combine_job& J = jobs[k];
    if (J.nin < 1 || J.nin > kMaxCombine || J.nout < 1 || J.nout > kMaxCombine || !J.in || !J.out || !J.coef)
      return fail("plan_combine: job %d: nin=%d, nout=%d (1..%d) or null array", k, J.nin, J.nout, kMaxCombine);
    StripeMap& m = maps[static_cast<size_t>(k)];
    bool ones = J.nout == 1;
    for (int i = 0; i < J.nin; ++i) {
      if (!J.in[i]) return fail("plan_combine: job %d: null input %d", k, i);
      m.in.push_back(redset_hip::CellRef{static_cast<int>(table.size()), redset_hip::kData, 0});
      table.push_back(const_cast<unsigned char*>(J.in[i]));
    }
    for (int j = 0; j < J.nout; ++j) {
      if (!J.out[j]) return fail("plan_combine: job %d: null output %d", k, j);
      m.out.push_back(redset_hip::CellRef{static_cast<int>(table.size()), redset_hip::kData, 0});
      table.push_back(J.out[j]);
    }
    m.coef.assign(J.coef, J.coef + static_cast<size_t>(J.nin) * J.nout);
    for (uint8_t c : m.coef) ones = ones && c == 1;
    m.xor_only = ones;  // one output, every coefficient 1: the XOR kernel
    m.accumulate = J.accumulate != 0;
  }
  return finish_plan(0, 0, 0, 0, nbytes, maps, SetLayout{table.data(), table.data(), 0}, out);
}

int redset_hip_plan_execute(const redset_hip_plan* plan, void* stream) {
  if (!plan) return fail("null plan");
  for (const GfLaunch& G : plan->gf_launches)
    if (int e = redset_hip::launch_gf(G, stream)) return hip_check(static_cast<hipError_t>(e), "gf_mac launch");
  for (const XorLaunch& X : plan->xor_launches)
    if (int e = redset_hip::launch_xor(X, stream)) return hip_check(static_cast<hipError_t>(e), "xor launch");
  return REDSET_SUCCESS;
}

int redset_hip_plan_get_info(const redset_hip_plan* plan, redset_hip_plan_info* info) {
  if (!plan || !info) return fail("null argument");
  *info = plan->info;
  return REDSET_SUCCESS;
}

void redset_hip_plan_destroy(redset_hip_plan* plan) {
  if (!plan) return;
  if (plan->d_gf) (void) hipFree(plan->d_gf);
  if (plan->d_xor) (void) hipFree(plan->d_xor);
  if (plan->d_claim) (void) hipFree(plan->d_claim);
  delete plan;
}

int redset_hip_gf_combine(const unsigned char* const* in, int nin, unsigned char* const* out, int nout,
                          const unsigned char* coeffs, size_t nbytes, int accumulate, void* stream) {
  if (nin < 1 || nin > kMaxCombine || nout < 1 || nout > kMaxCombine)
    return fail("gf_combine: nin=%d, nout=%d (1..%d)", nin, nout, kMaxCombine);
  if (!in || !out || !coeffs) return fail("gf_combine: null argument");
  if (nin > kMaxIn || nout > kMaxOut) {
    // wider than one kernel pass: 16-input accumulate passes x 4-output groups
    redset_hip::StripeMap m;
    m.in.resize(nin);
    m.out.resize(nout);
    m.coef.assign(coeffs, coeffs + static_cast<size_t>(nin) * nout);
    for (int i = 0; i < nin; ++i)
      if (!in[i]) return fail("gf_combine: null input %d", i);
    for (int j = 0; j < nout; ++j)
      if (!out[j]) return fail("gf_combine: null output %d", j);
    return redset_hip::run_stripe(m, in, out, nbytes, stream, 0, accumulate != 0);
  }
  GfJob J;
  std::memset(&J, 0, sizeof(J));
  bool al = true;
  for (int i = 0; i < nin; ++i) {
    if (!in[i]) return fail("gf_combine: null input %d", i);
    J.in[i] = in[i];
    al = al && aligned16(in[i]);
  }
  for (int j = 0; j < nout; ++j) {
    if (!out[j]) return fail("gf_combine: null output %d", j);
    J.out[j] = out[j];
    al = al && aligned16(out[j]);
    for (int i = 0; i < nin; ++i) J.coef[j][i] = coeffs[j * nin + i];
  }
  GfLaunch G;
  std::memset(&G, 0, sizeof(G));
  G.njobs = 1;
  G.nin = nin;
  G.nout = nout;
  G.accumulate = accumulate ? 1 : 0;
  G.bytes_only = al ? 0 : 1;
  G.nbytes = nbytes;
  G.blocks_per_job = blocks_per_job(1, nbytes, redset_hip::gf_blocks_per_cu(nin));
  return hip_check(static_cast<hipError_t>(redset_hip::launch_gf_single(G, J, stream)), "gf_combine launch");
}

int redset_hip_xor_combine(const unsigned char* const* in, int nin, unsigned char* out, size_t nbytes, int accumulate,
                           void* stream) {
  if (nin < 1 || nin > kMaxCombine) return fail("xor_combine: nin=%d (1..%d)", nin, kMaxCombine);
  if (!in || !out) return fail("xor_combine: null argument");
  if (nin > kMaxIn) {
    redset_hip::StripeMap m;
    m.in.resize(nin);
    m.out.resize(1);
    m.coef.assign(static_cast<size_t>(nin), 1);
    m.xor_only = true;
    for (int i = 0; i < nin; ++i)
      if (!in[i]) return fail("xor_combine: null input %d", i);
    return redset_hip::run_stripe(m, in, &out, nbytes, stream, 0, accumulate != 0);
  }
  XorJob J;
  std::memset(&J, 0, sizeof(J));
  bool al = aligned16(out);
  for (int i = 0; i < nin; ++i) {
    if (!in[i]) return fail("xor_combine: null input %d", i);
    J.in[i] = in[i];
    al = al && aligned16(in[i]);
  }
  J.out = out;
  XorLaunch X;
  std::memset(&X, 0, sizeof(X));
  X.njobs = 1;
  X.nin = nin;
  X.accumulate = accumulate ? 1 : 0;
  X.bytes_only = al ? 0 : 1;
  X.nbytes = nbytes;
  X.blocks_per_job = blocks_per_job(1, nbytes, xor_blocks_cap());
  return hip_check(static_cast<hipError_t>(redset_hip::launch_xor_single(X, J, stream)), "xor_combine launch");
}

}  // extern "C"
