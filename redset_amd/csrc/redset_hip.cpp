// redset_hip.cpp -- C ABI (include/redset_hip.h): GF state, whole-set plans
// for RS / XOR encode and rebuild, and stripe primitives.
//
// A plan turns the reference's per-rank, per-slice loops (encode:
// src/redset_reedsolomon.c:309-391, decode: :631-768, XOR: src/redset_xor.c:
// 243-288, src/redset_xor_serial.c:202-273) into a few kernel launches over
// whole cells: one GfJob per stripe, each reading its input cells once and
// writing its output cells once. Planning happens once on the host; execute
// only enqueues kernels, so it can be captured into a hipGraph.
#include "redset_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <tuple>
#include <vector>

#include "codec_kernels.h"
#include "gf256.h"

using redset_hip::GfJob;
using redset_hip::GfLaunch;
using redset_hip::kMaxIn;
using redset_hip::kMaxOut;
using redset_hip::XorJob;
using redset_hip::XorLaunch;

struct redset_hip_rs {
  int ranks;
  int encoding;
  std::vector<uint8_t> mat;  // (p+e) x p
};

struct redset_hip_plan {
  redset_hip_plan_info info{};
  GfJob* d_gf = nullptr;  // device job arrays
  XorJob* d_xor = nullptr;
  std::vector<GfLaunch> gf_launches;
  std::vector<XorLaunch> xor_launches;
};

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return REDSET_FAILURE;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return REDSET_SUCCESS;
  return fail("%s: %s", what, hipGetErrorString(e));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// One output cell of a stripe and its coefficient over each input of the stripe.
struct Target {
  uint8_t* cell;
  std::vector<uint8_t> coef;  // one per stripe input
};

// A stripe's linear map: targets = coef * inputs.
struct Stripe {
  std::vector<const uint8_t*> inputs;
  std::vector<Target> targets;
};

// Resident 256-thread blocks per CU the codec aims for. HBM streams best at
// low occupancy here: 2 blocks (8 waves) per CU beat 4 and 8 by 3-5% on
// gf_mac, as fewer blocks beat more on a plain copy (tools/gfbench.hip,
// tools/membench.hip); REDSET_HIP_BLOCKS_PER_CU overrides it.
int target_blocks_per_cu(int occupancy) {
  static int env = -1;
  if (env < 0) {
    const char* s = std::getenv("REDSET_HIP_BLOCKS_PER_CU");
    env = (s && std::atoi(s) > 0) ? std::atoi(s) : 0;
  }
  const int want = env > 0 ? env : 2;
  return std::max(1, std::min(want, occupancy));
}

// Blocks per job so the whole launch fits in one resident wave of blocks.
int blocks_per_job(int njobs, size_t nbytes, int occupancy) {
  const long target = static_cast<long>(redset_hip::device_cu_count()) * target_blocks_per_cu(occupancy);
  long bpj = std::max<long>(1, target / std::max(1, njobs));
  // at least one 16-B vector per thread per block
  const long vec_blocks = static_cast<long>((nbytes / 16 + redset_hip::kBlock - 1) / redset_hip::kBlock);
  bpj = std::min(bpj, std::max<long>(1, vec_blocks));
  return static_cast<int>(bpj);
}

// Split stripes into launches of <= kMaxIn inputs x <= kMaxOut outputs.
// Output groups are independent; input groups of one output group run in
// order, the first overwriting and the rest accumulating. Stripes with equal
// input counts share a launch.
int build_gf_plan(redset_hip_plan* plan, const std::vector<Stripe>& stripes, size_t nbytes) {
  struct Pending {
    std::vector<GfJob> jobs;
    int nin, nout, accumulate, bytes_only;
  };
  std::map<std::tuple<int, int, int, int>, Pending> groups;  // (ig, nin, nout, og) ordering key
  unsigned long long rd = 0, wr = 0;
  for (const Stripe& s : stripes) {
    const int nin = static_cast<int>(s.inputs.size());
    const int nt = static_cast<int>(s.targets.size());
    if (nt == 0) continue;
    if (nin == 0) return fail("stripe with outputs but no inputs");
    for (int og = 0; og * kMaxOut < nt; ++og) {
      const int o0 = og * kMaxOut, no = std::min(kMaxOut, nt - o0);
      for (int ig = 0; ig * kMaxIn < nin; ++ig) {
        const int i0 = ig * kMaxIn, ni = std::min(kMaxIn, nin - i0);
        GfJob J;
        std::memset(&J, 0, sizeof(J));
        bool al = true;
        for (int i = 0; i < ni; ++i) {
          J.in[i] = s.inputs[i0 + i];
          al = al && aligned16(J.in[i]);
        }
        for (int j = 0; j < no; ++j) {
          J.out[j] = s.targets[o0 + j].cell;
          al = al && aligned16(J.out[j]);
          for (int i = 0; i < ni; ++i) J.coef[j][i] = s.targets[o0 + j].coef[i0 + i];
        }
        Pending& P = groups[std::make_tuple(ig, ni, no, al ? 0 : 1)];
        P.nin = ni;
        P.nout = no;
        P.accumulate = ig > 0;
        P.bytes_only = al ? 0 : 1;
        P.jobs.push_back(J);
        rd += static_cast<unsigned long long>(ni + (ig > 0 ? no : 0)) * nbytes;
        wr += static_cast<unsigned long long>(no) * nbytes;
      }
    }
  }
  size_t total = 0;
  for (auto& kv : groups) total += kv.second.jobs.size();
  plan->info.jobs = static_cast<int>(total);
  plan->info.bytes_read = rd;
  plan->info.bytes_written = wr;
  if (total == 0) return REDSET_SUCCESS;
  std::vector<GfJob> all;
  all.reserve(total);
  for (auto& kv : groups) {
    Pending& P = kv.second;
    GfLaunch L;
    std::memset(&L, 0, sizeof(L));
    L.jobs = reinterpret_cast<const GfJob*>(all.size());  // offset, patched below
    L.njobs = static_cast<int>(P.jobs.size());
    L.nin = P.nin;
    L.nout = P.nout;
    L.accumulate = P.accumulate;
    L.bytes_only = P.bytes_only;
    L.nbytes = nbytes;
    L.blocks_per_job = blocks_per_job(L.njobs, nbytes, redset_hip::gf_blocks_per_cu(P.nin));
    all.insert(all.end(), P.jobs.begin(), P.jobs.end());
    plan->gf_launches.push_back(L);
  }
  if (int rc = hip_check(hipMalloc(&plan->d_gf, all.size() * sizeof(GfJob)), "hipMalloc(plan jobs)")) return rc;
  if (int rc = hip_check(hipMemcpy(plan->d_gf, all.data(), all.size() * sizeof(GfJob), hipMemcpyHostToDevice),
                         "hipMemcpy(plan jobs)"))
    return rc;
  for (GfLaunch& L : plan->gf_launches) L.jobs = plan->d_gf + reinterpret_cast<uintptr_t>(L.jobs);
  plan->info.launches = static_cast<int>(plan->gf_launches.size());
  return REDSET_SUCCESS;
}

// XOR stripes: output = XOR of inputs; > kMaxIn inputs accumulate in passes.
struct XorStripe {
  std::vector<const uint8_t*> inputs;
  uint8_t* out;
};

int build_xor_plan(redset_hip_plan* plan, const std::vector<XorStripe>& stripes, size_t nbytes) {
  struct Pending {
    std::vector<XorJob> jobs;
    int nin, accumulate, bytes_only;
  };
  std::map<std::tuple<int, int, int>, Pending> groups;
  unsigned long long rd = 0, wr = 0;
  for (const XorStripe& s : stripes) {
    const int nin = static_cast<int>(s.inputs.size());
    if (nin == 0) return fail("XOR stripe with no inputs");
    for (int ig = 0; ig * kMaxIn < nin; ++ig) {
      const int i0 = ig * kMaxIn, ni = std::min(kMaxIn, nin - i0);
      XorJob J;
      std::memset(&J, 0, sizeof(J));
      bool al = aligned16(s.out);
      for (int i = 0; i < ni; ++i) {
        J.in[i] = s.inputs[i0 + i];
        al = al && aligned16(J.in[i]);
      }
      J.out = s.out;
      Pending& P = groups[std::make_tuple(ig, ni, al ? 0 : 1)];
      P.nin = ni;
      P.accumulate = ig > 0;
      P.bytes_only = al ? 0 : 1;
      P.jobs.push_back(J);
      rd += static_cast<unsigned long long>(ni + (ig > 0 ? 1 : 0)) * nbytes;
      wr += nbytes;
    }
  }
  size_t total = 0;
  for (auto& kv : groups) total += kv.second.jobs.size();
  plan->info.jobs = static_cast<int>(total);
  plan->info.bytes_read = rd;
  plan->info.bytes_written = wr;
  if (total == 0) return REDSET_SUCCESS;
  std::vector<XorJob> all;
  for (auto& kv : groups) {
    Pending& P = kv.second;
    XorLaunch L;
    std::memset(&L, 0, sizeof(L));
    L.jobs = reinterpret_cast<const XorJob*>(all.size());
    L.njobs = static_cast<int>(P.jobs.size());
    L.nin = P.nin;
    L.accumulate = P.accumulate;
    L.bytes_only = P.bytes_only;
    L.nbytes = nbytes;
    L.blocks_per_job = blocks_per_job(L.njobs, nbytes, 8);
    all.insert(all.end(), P.jobs.begin(), P.jobs.end());
    plan->xor_launches.push_back(L);
  }
  if (int rc = hip_check(hipMalloc(&plan->d_xor, all.size() * sizeof(XorJob)), "hipMalloc(plan jobs)")) return rc;
  if (int rc = hip_check(hipMemcpy(plan->d_xor, all.data(), all.size() * sizeof(XorJob), hipMemcpyHostToDevice),
                         "hipMemcpy(plan jobs)"))
    return rc;
  for (XorLaunch& L : plan->xor_launches) L.jobs = plan->d_xor + reinterpret_cast<uintptr_t>(L.jobs);
  plan->info.launches = static_cast<int>(plan->xor_launches.size());
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

// cell of member `rank` in stripe `chunk`: a data segment in lofi or a
// parity slot in the redundancy region
uint8_t* rs_cell(const redset_hip_rs* rs, unsigned char* const* lofi, unsigned char* const* parity, int rank,
                 int chunk, size_t stride) {
  const int p = rs->ranks, e = rs->encoding;
  const int enc = redset_hip::encoding_id(p, e, rank, chunk);
  if (enc < p) return lofi[rank] + static_cast<size_t>(redset_hip::data_id(p, e, rank, chunk)) * stride;
  return parity[rank] + static_cast<size_t>(enc - p) * stride;
}

// decode map of one stripe as (missing x p): column s = member s's cell
int decode_map(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int chunk, std::vector<uint8_t>& D) {
  const int p = rs->ranks, e = rs->encoding;
  const redset_hip::Field& F = redset_hip::field();
  std::vector<int> unknowns(missing);
  std::vector<char> erased(p, 0);
  for (int i = 0; i < missing; ++i) {
    if (rebuild_ranks[i] < 0 || rebuild_ranks[i] >= p) return fail("rebuild rank %d out of range", rebuild_ranks[i]);
    if (i > 0 && rebuild_ranks[i] <= rebuild_ranks[i - 1]) return fail("rebuild_ranks must be ascending");
    erased[rebuild_ranks[i]] = 1;
    unknowns[i] = redset_hip::encoding_id(p, e, rebuild_ranks[i], chunk);
  }
  std::vector<uint8_t> m;
  std::vector<int> rows;
  redset_hip::identify_rows(rs->mat, p, e, missing, unknowns.data(), m, rows);
  for (int i = 0; i < missing; ++i)
    if (rows[i] < 0) return fail("no parity row available for unknown %d", i);
  const std::vector<uint8_t> T = redset_hip::solve_transform(m, missing);
  // accumulator k (redset_rs_reduce_decode, src/redset_reedsolomon_common.c:
  // 855-899) = sum over surviving members s of a_k(s) * cell_s
  D.assign(static_cast<size_t>(missing) * p, 0);
  for (int s = 0; s < p; ++s) {
    if (erased[s]) continue;
    const int enc = redset_hip::encoding_id(p, e, s, chunk);
    for (int k = 0; k < missing; ++k) {
      const int row = rows[k] + p;
      uint8_t a;
      if (enc < p) a = rs->mat[static_cast<size_t>(row) * p + s];
      else a = (enc == row) ? 1 : 0;
      if (!a) continue;
      for (int i = 0; i < missing; ++i)
        D[static_cast<size_t>(i) * p + s] ^= F.mul(T[static_cast<size_t>(i) * missing + k], a);
    }
  }
  return REDSET_SUCCESS;
}

}  // namespace

extern "C" {

const char* redset_hip_last_error(void) { return g_err.c_str(); }
const char* redset_hip_version(void) { return "redset-hip 0.1 (gfx950)"; }

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

int redset_hip_rs_plan_encode(const redset_hip_rs* rs, unsigned char* const* lofi, unsigned char* const* parity,
                              size_t chunk_size, size_t stride, redset_hip_plan** out) {
  if (!rs) return fail("null rs state");
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(parity),
                              rs->ranks, chunk_size, stride, out))
    return rc;
  const int p = rs->ranks, e = rs->encoding;
  std::vector<Stripe> stripes(p);
  for (int c = 0; c < p; ++c) {
    Stripe& S = stripes[c];
    std::vector<int> data_ranks;
    for (int s = 0; s < p; ++s) {
      if (redset_hip::encoding_id(p, e, s, c) < p) {
        data_ranks.push_back(s);
        S.inputs.push_back(rs_cell(rs, lofi, parity, s, c, stride));
      }
    }
    for (int r = 0; r < p; ++r) {
      const int row = redset_hip::encoding_id(p, e, r, c);
      if (row < p) continue;
      Target t;
      t.cell = parity[r] + static_cast<size_t>(row - p) * stride;
      for (int s : data_ranks) t.coef.push_back(rs->mat[static_cast<size_t>(row) * p + s]);
      S.targets.push_back(std::move(t));
    }
  }
  redset_hip_plan* plan = new (std::nothrow) redset_hip_plan;
  if (!plan) return fail("out of host memory");
  plan->info.kind = REDSET_HIP_PLAN_RS_ENCODE;
  plan->info.ranks = p;
  plan->info.encoding = e;
  plan->info.chunk_size = chunk_size;
  if (int rc = build_gf_plan(plan, stripes, chunk_size)) {
    redset_hip_plan_destroy(plan);
    return rc;
  }
  *out = plan;
  return REDSET_SUCCESS;
}

int redset_hip_rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int chunk_id,
                                unsigned char* coef_out) {
  if (!rs || !coef_out || (missing > 0 && !rebuild_ranks)) return fail("null argument");
  if (missing < 1 || missing > rs->encoding) return fail("cannot rebuild %d members with %d parity", missing, rs->encoding);
  if (chunk_id < 0 || chunk_id >= rs->ranks) return fail("chunk id %d out of range", chunk_id);
  std::vector<uint8_t> D;
  if (int rc = decode_map(rs, missing, rebuild_ranks, chunk_id, D)) return rc;
  std::memcpy(coef_out, D.data(), D.size());
  return REDSET_SUCCESS;
}

int redset_hip_rs_plan_rebuild(const redset_hip_rs* rs, int missing, const int* rebuild_ranks,
                               unsigned char* const* lofi, unsigned char* const* parity, size_t chunk_size,
                               size_t stride, redset_hip_plan** out) {
  if (!rs) return fail("null rs state");
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(parity),
                              rs->ranks, chunk_size, stride, out))
    return rc;
  const int p = rs->ranks;
  if (missing < 0 || missing > rs->encoding)
    return fail("cannot rebuild %d members with %d parity chunks", missing, rs->encoding);
  if (missing > 0 && !rebuild_ranks) return fail("null rebuild_ranks");
  std::vector<Stripe> stripes;
  for (int c = 0; c < p && missing > 0; ++c) {
    std::vector<uint8_t> D;
    if (int rc = decode_map(rs, missing, rebuild_ranks, c, D)) return rc;
    Stripe S;
    std::vector<int> cols;
    for (int s = 0; s < p; ++s) {
      bool used = false;
      for (int i = 0; i < missing; ++i) used = used || D[static_cast<size_t>(i) * p + s] != 0;
      if (!used) continue;
      cols.push_back(s);
      S.inputs.push_back(rs_cell(rs, lofi, parity, s, c, stride));
    }
    for (int i = 0; i < missing; ++i) {
      Target t;
      t.cell = rs_cell(rs, lofi, parity, rebuild_ranks[i], c, stride);
      for (int s : cols) t.coef.push_back(D[static_cast<size_t>(i) * p + s]);
      S.targets.push_back(std::move(t));
    }
    stripes.push_back(std::move(S));
  }
  redset_hip_plan* plan = new (std::nothrow) redset_hip_plan;
  if (!plan) return fail("out of host memory");
  plan->info.kind = REDSET_HIP_PLAN_RS_REBUILD;
  plan->info.ranks = p;
  plan->info.encoding = rs->encoding;
  plan->info.missing = missing;
  plan->info.chunk_size = chunk_size;
  if (int rc = build_gf_plan(plan, stripes, chunk_size)) {
    redset_hip_plan_destroy(plan);
    return rc;
  }
  *out = plan;
  return REDSET_SUCCESS;
}

int redset_hip_xor_plan_encode(int ranks, unsigned char* const* lofi, unsigned char* const* xorc, size_t chunk_size,
                               size_t stride, redset_hip_plan** out) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(xorc),
                              ranks, chunk_size, stride, out))
    return rc;
  std::vector<XorStripe> stripes(ranks);
  for (int c = 0; c < ranks; ++c) {
    for (int s = 0; s < ranks; ++s) {
      if (s == c) continue;
      stripes[c].inputs.push_back(lofi[s] + static_cast<size_t>(redset_hip::xor_segment(s, c)) * stride);
    }
    stripes[c].out = xorc[c];
  }
  redset_hip_plan* plan = new (std::nothrow) redset_hip_plan;
  if (!plan) return fail("out of host memory");
  plan->info.kind = REDSET_HIP_PLAN_XOR_ENCODE;
  plan->info.ranks = ranks;
  plan->info.encoding = 1;
  plan->info.chunk_size = chunk_size;
  if (int rc = build_xor_plan(plan, stripes, chunk_size)) {
    redset_hip_plan_destroy(plan);
    return rc;
  }
  *out = plan;
  return REDSET_SUCCESS;
}

int redset_hip_xor_plan_rebuild(int ranks, int root, unsigned char* const* lofi, unsigned char* const* xorc,
                                size_t chunk_size, size_t stride, redset_hip_plan** out) {
  if (ranks < 2) return fail("XOR needs at least 2 ranks, got %d", ranks);
  if (root < 0 || root >= ranks) return fail("root %d out of range", root);
  if (int rc = check_set_args(reinterpret_cast<const void* const*>(lofi), reinterpret_cast<const void* const*>(xorc),
                              ranks, chunk_size, stride, out))
    return rc;
  auto cell = [&](int s, int c) -> uint8_t* {
    return s == c ? xorc[s] : lofi[s] + static_cast<size_t>(redset_hip::xor_segment(s, c)) * stride;
  };
  std::vector<XorStripe> stripes(ranks);
  for (int c = 0; c < ranks; ++c) {
    for (int s = 0; s < ranks; ++s)
      if (s != root) stripes[c].inputs.push_back(cell(s, c));
    stripes[c].out = cell(root, c);
  }
  redset_hip_plan* plan = new (std::nothrow) redset_hip_plan;
  if (!plan) return fail("out of host memory");
  plan->info.kind = REDSET_HIP_PLAN_XOR_REBUILD;
  plan->info.ranks = ranks;
  plan->info.encoding = 1;
  plan->info.missing = 1;
  plan->info.chunk_size = chunk_size;
  if (int rc = build_xor_plan(plan, stripes, chunk_size)) {
    redset_hip_plan_destroy(plan);
    return rc;
  }
  *out = plan;
  return REDSET_SUCCESS;
}

int redset_hip_plan_execute(const redset_hip_plan* plan, void* stream) {
  if (!plan) return fail("null plan");
  for (const GfLaunch& L : plan->gf_launches)
    if (int e = redset_hip::launch_gf(L, stream))
      return hip_check(static_cast<hipError_t>(e), "gf_mac launch");
  for (const XorLaunch& L : plan->xor_launches)
    if (int e = redset_hip::launch_xor(L, stream))
      return hip_check(static_cast<hipError_t>(e), "xor launch");
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
  delete plan;
}

int redset_hip_gf_combine(const unsigned char* const* in, int nin, unsigned char* const* out, int nout,
                          const unsigned char* coeffs, size_t nbytes, int accumulate, void* stream) {
  if (nin < 1 || nin > kMaxIn || nout < 1 || nout > kMaxOut)
    return fail("gf_combine: nin=%d (1..%d), nout=%d (1..%d)", nin, kMaxIn, nout, kMaxOut);
  if (!in || !out || !coeffs) return fail("gf_combine: null argument");
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
  GfLaunch L;
  std::memset(&L, 0, sizeof(L));
  L.njobs = 1;
  L.nin = nin;
  L.nout = nout;
  L.accumulate = accumulate ? 1 : 0;
  L.bytes_only = al ? 0 : 1;
  L.nbytes = nbytes;
  L.blocks_per_job = blocks_per_job(1, nbytes, redset_hip::gf_blocks_per_cu(nin));
  return hip_check(static_cast<hipError_t>(redset_hip::launch_gf_single(L, J, stream)), "gf_combine launch");
}

int redset_hip_xor_combine(const unsigned char* const* in, int nin, unsigned char* out, size_t nbytes, int accumulate,
                           void* stream) {
  if (nin < 1 || nin > kMaxIn) return fail("xor_combine: nin=%d (1..%d)", nin, kMaxIn);
  if (!in || !out) return fail("xor_combine: null argument");
  XorJob J;
  std::memset(&J, 0, sizeof(J));
  bool al = aligned16(out);
  for (int i = 0; i < nin; ++i) {
    if (!in[i]) return fail("xor_combine: null input %d", i);
    J.in[i] = in[i];
    al = al && aligned16(in[i]);
  }
  J.out = out;
  XorLaunch L;
  std::memset(&L, 0, sizeof(L));
  L.njobs = 1;
  L.nin = nin;
  L.accumulate = accumulate ? 1 : 0;
  L.bytes_only = al ? 0 : 1;
  L.nbytes = nbytes;
  L.blocks_per_job = blocks_per_job(1, nbytes, 8);
  return hip_check(static_cast<hipError_t>(redset_hip::launch_xor_single(L, J, stream)), "xor_combine launch");
}

}  // extern "C"
