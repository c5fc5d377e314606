// stripe_map.cpp -- see stripe_map.h.
#include "stripe_map.h"

#include <cstdarg>
#include <cstdio>
#include <string>

#include "gf256.h"

namespace redset_hip {

thread_local std::string g_last_error;

int fail(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return 1;  // REDSET_FAILURE
}

const char* last_error() { return g_last_error.c_str(); }

CellRef rs_cell(const redset_hip_rs* rs, int rank, int chunk) {
  const int p = rs->ranks, e = rs->encoding;
  const int enc = encoding_id(p, e, rank, chunk);
  if (enc < p) return CellRef{rank, kData, data_id(p, e, rank, chunk)};
  return CellRef{rank, kParity, enc - p};
}

int rs_encode_map(const redset_hip_rs* rs, int c, StripeMap& m) {
  const int p = rs->ranks, e = rs->encoding;
  m = StripeMap();
  std::vector<int> data_ranks;
  for (int s = 0; s < p; ++s) {
    if (encoding_id(p, e, s, c) < p) {
      data_ranks.push_back(s);
      m.in.push_back(rs_cell(rs, s, c));
    }
  }
  for (int r = 0; r < p; ++r) {
    const int row = encoding_id(p, e, r, c);
    if (row < p) continue;
    m.out.push_back(CellRef{r, kParity, row - p});
    for (int s : data_ranks) m.coef.push_back(rs->mat[static_cast<size_t>(row) * p + s]);
  }
  return 0;
}

int rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int chunk,
                     std::vector<uint8_t>& D) {
  const int p = rs->ranks, e = rs->encoding;
  const Field& F = field();
  if (missing < 1 || missing > e) return fail("cannot rebuild %d members with %d parity chunks", missing, e);
  std::vector<int> unknowns(missing);
  std::vector<char> erased(p, 0);
  for (int i = 0; i < missing; ++i) {
    if (rebuild_ranks[i] < 0 || rebuild_ranks[i] >= p) return fail("rebuild rank %d out of range", rebuild_ranks[i]);
    if (i > 0 && rebuild_ranks[i] <= rebuild_ranks[i - 1]) return fail("rebuild_ranks must be ascending");
    erased[rebuild_ranks[i]] = 1;
    unknowns[i] = encoding_id(p, e, rebuild_ranks[i], chunk);
  }
  std::vector<uint8_t> sys;
  std::vector<int> rows;
  identify_rows(rs->mat, p, e, missing, unknowns.data(), sys, rows);
  for (int i = 0; i < missing; ++i)
    if (rows[i] < 0) return fail("no parity row available for unknown %d", i);
  const std::vector<uint8_t> T = solve_transform(sys, missing);
  // accumulator k (redset_rs_reduce_decode, src/redset_reedsolomon_common.c:
  // 855-899) = sum over surviving members s of a_k(s) * cell_s; the solved
  // buffer i = sum_k T[i][k] * accumulator k
  D.assign(static_cast<size_t>(missing) * p, 0);
  for (int s = 0; s < p; ++s) {
    if (erased[s]) continue;
    const int enc = encoding_id(p, e, s, chunk);
    for (int k = 0; k < missing; ++k) {
      const int row = rows[k] + p;
      const uint8_t a = enc < p ? rs->mat[static_cast<size_t>(row) * p + s] : static_cast<uint8_t>(enc == row);
      if (!a) continue;
      for (int i = 0; i < missing; ++i)
        D[static_cast<size_t>(i) * p + s] ^= F.mul(T[static_cast<size_t>(i) * missing + k], a);
    }
  }
  return 0;
}

int rs_rebuild_map(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int c, StripeMap& m) {
  const int p = rs->ranks;
  m = StripeMap();
  std::vector<uint8_t> D;
  if (int rc = rs_decode_matrix(rs, missing, rebuild_ranks, c, D)) return rc;
  std::vector<int> cols;
  for (int s = 0; s < p; ++s) {
    bool used = false;
    for (int i = 0; i < missing; ++i) used = used || D[static_cast<size_t>(i) * p + s] != 0;
    if (!used) continue;
    cols.push_back(s);
    m.in.push_back(rs_cell(rs, s, c));
  }
  for (int i = 0; i < missing; ++i) {
    m.out.push_back(rs_cell(rs, rebuild_ranks[i], c));
    for (int s : cols) m.coef.push_back(D[static_cast<size_t>(i) * p + s]);
  }
  return 0;
}

namespace {
CellRef xor_cell(int s, int c) { return s == c ? CellRef{s, kParity, 0} : CellRef{s, kData, xor_segment(s, c)}; }
}  // namespace

int xor_encode_map(int ranks, int c, StripeMap& m) {
  m = StripeMap();
  m.xor_only = true;
  for (int s = 0; s < ranks; ++s)
    if (s != c) m.in.push_back(xor_cell(s, c));
  m.out.push_back(CellRef{c, kParity, 0});
  m.coef.assign(m.in.size(), 1);
  return 0;
}

int xor_rebuild_map(int ranks, int root, int c, StripeMap& m) {
  if (root < 0 || root >= ranks) return fail("root %d out of range", root);
  m = StripeMap();
  m.xor_only = true;
  for (int s = 0; s < ranks; ++s)
    if (s != root) m.in.push_back(xor_cell(s, c));
  m.out.push_back(xor_cell(root, c));
  m.coef.assign(m.in.size(), 1);
  return 0;
}

}  // namespace redset_hip
