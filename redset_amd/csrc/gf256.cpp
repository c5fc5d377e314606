// gf256.cpp -- see gf256.h.
#include "gf256.h"

#include <algorithm>

namespace redset_hip {

namespace {
// carry-less product reduced by 0x11D (reference gf_mult, :41-75)
uint8_t slow_mul(unsigned a, unsigned b) {
  unsigned r = 0;
  while (b) {
    if (b & 1u) r ^= a;
    a <<= 1;
    if (a & 0x100u) a ^= 0x11Du;
    b >>= 1;
  }
  return static_cast<uint8_t>(r);
}
}  // namespace

Field::Field() {
  unsigned v = 1;
  for (int i = 0; i < 255; ++i) {
    exp_[i] = static_cast<uint8_t>(v);
    exp_[i + 255] = static_cast<uint8_t>(v);
    log_[v] = static_cast<uint8_t>(i);
    v = slow_mul(v, 2);
  }
  exp_[510] = exp_[0];
  exp_[511] = exp_[1];
  log_[0] = 0;
  inv_[0] = 0;  // reference leaves imult[0] = 0 (:135)
  for (int a = 1; a < 256; ++a) inv_[a] = exp_[(255 - log_[a]) % 255];
}

const Field& field() {
  static const Field f;
  return f;
}

std::vector<uint8_t> encoding_matrix(int n, int k) {
  const Field& F = field();
  const int rows = n + k;
  std::vector<uint8_t> m(static_cast<size_t>(rows) * n);
  auto at = [&](int r, int c) -> uint8_t& { return m[static_cast<size_t>(r) * n + c]; };
  // Vandermonde: entry (r, c) = r^c
  for (int r = 0; r < rows; ++r) {
    uint8_t pw = 1;
    for (int c = 0; c < n; ++c) {
      at(r, c) = (c == 0) ? 1 : pw;
      pw = (c == 0) ? static_cast<uint8_t>(r) : F.mul(pw, static_cast<uint8_t>(r));
    }
  }
  // column elimination so the top block becomes I (with the reference's
  // pivot search and column swap rule)
  for (int r = 0; r < n; ++r) {
    int piv = r;
    for (int c = r; c < n; ++c) {
      if (at(r, c)) { piv = c; break; }
    }
    if (piv != r) {
      for (int rr = 0; rr < rows; ++rr) std::swap(at(rr, r), at(rr, piv));
    }
    const uint8_t s = F.inv(at(r, r));
    for (int rr = r; rr < rows; ++rr) at(rr, r) = F.mul(at(rr, r), s);
    for (int c = 0; c < n; ++c) {
      if (c == r || at(r, c) == 0) continue;
      const uint8_t f = at(r, c);
      for (int rr = r; rr < rows; ++rr) at(rr, c) ^= F.mul(f, at(rr, r));
    }
  }
  return m;
}

int encoding_id(int ranks, int encoding, int rank, int chunk_id) {
  const int d = ranks - encoding;
  const int id = (d - rank + ranks + chunk_id) % ranks;
  return id < d ? rank : ranks + (id - d);
}

int data_id(int ranks, int encoding, int rank, int chunk_id) {
  int id = chunk_id > rank ? chunk_id - encoding : chunk_id;
  const int lead = rank + encoding - ranks;
  return lead > 0 ? id - lead : id;
}

void identify_rows(const std::vector<uint8_t>& mat, int n, int k, int missing, const int* unknowns,
                   std::vector<uint8_t>& m, std::vector<int>& rows) {
  auto defined = [&](int row, int u) {
    return u < n ? mat[static_cast<size_t>(row + n) * n + u] != 0 : u == row + n;
  };
  std::vector<int> unknown_count(k, 0);
  std::vector<char> used(k, 0);
  for (int r = 0; r < k; ++r)
    for (int i = 0; i < missing; ++i) unknown_count[r] += defined(r, unknowns[i]) ? 1 : 0;
  m.assign(static_cast<size_t>(missing) * missing, 0);
  rows.assign(missing, -1);
  for (int i = 0; i < missing; ++i) {
    int best = -1, best_count = missing + 1;
    for (int r = 0; r < k; ++r) {
      if (used[r] || !defined(r, unknowns[i])) continue;
      if (unknown_count[r] < best_count) { best_count = unknown_count[r]; best = r; }
    }
    rows[i] = best;
    if (best < 0) continue;
    used[best] = 1;
    for (int j = 0; j < missing; ++j) {
      const int u = unknowns[j];
      m[static_cast<size_t>(i) * missing + j] =
          u < n ? mat[static_cast<size_t>(best + n) * n + u] : static_cast<uint8_t>(u == best + n);
    }
  }
}

std::vector<uint8_t> solve_transform(std::vector<uint8_t> m, int M) {
  const Field& F = field();
  std::vector<uint8_t> T(static_cast<size_t>(M) * M, 0);
  for (int i = 0; i < M; ++i) T[static_cast<size_t>(i) * M + i] = 1;
  auto A = [&](int r, int c) -> uint8_t& { return m[static_cast<size_t>(r) * M + c]; };
  auto scale = [&](int r, uint8_t v) {
    for (int c = 0; c < M; ++c) {
      A(r, c) = F.mul(A(r, c), v);
      T[static_cast<size_t>(r) * M + c] = F.mul(T[static_cast<size_t>(r) * M + c], v);
    }
  };
  auto madd = [&](uint8_t v, int a, int b) {  // row b ^= v * row a
    if (v == 0) return;
    for (int c = 0; c < M; ++c) {
      A(b, c) ^= F.mul(v, A(a, c));
      T[static_cast<size_t>(b) * M + c] ^= F.mul(v, T[static_cast<size_t>(a) * M + c]);
    }
  };
  for (int r = 0; r < M; ++r) {
    int piv = r;
    for (int c = r; c < M; ++c) {
      if (A(r, c)) { piv = c; break; }
    }
    if (piv != r)  // column swap of the coefficients only (reference :592)
      for (int rr = 0; rr < M; ++rr) std::swap(A(rr, r), A(rr, piv));
    if (A(r, r)) scale(r, F.inv(A(r, r)));
    for (int r2 = r + 1; r2 < M; ++r2) madd(A(r2, r), r, r2);
  }
  for (int r = M - 1; r > 0; --r)
    for (int r2 = r - 1; r2 >= 0; --r2) madd(A(r2, r), r, r2);
  return T;
}

}  // namespace redset_hip
