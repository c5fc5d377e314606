// gf256.h -- host-side GF(2^8) arithmetic, encoding matrix and stripe layout
// for the redset HIP codec (product code; the oracle under oracle/ is a
// separate restatement used only by tests).
//
// The field is GF(2^8) with x^8 + x^4 + x^3 + x^2 + 1 (0x11D) and generator
// 2, exactly as src/redset_reedsolomon_common.c:79-150 builds it, and the
// encoding matrix is the column-normalised Vandermonde matrix of
// src/redset_reedsolomon_common.c:634-725, so parity coefficients match the
// reference byte for byte.
#pragma once

#include <cstdint>
#include <vector>

namespace redset_hip {

struct Field {
  uint8_t exp_[512];   // exp_[i] = 2^i, doubled so log sums need no modulo
  uint8_t log_[256];
  uint8_t inv_[256];
  Field();
  uint8_t mul(uint8_t a, uint8_t b) const {
    if (a == 0 || b == 0) return 0;
    return exp_[log_[a] + log_[b]];
  }
  uint8_t inv(uint8_t a) const { return inv_[a]; }
};

const Field& field();

// (p+e) x p row-major encoding matrix (top p x p = identity).
// Reference: build_vandermonde + normalize_vandermonde,
// src/redset_reedsolomon_common.c:634-725.
std::vector<uint8_t> encoding_matrix(int ranks, int encoding);

// Reference: redset_rs_get_encoding_id, src/redset_reedsolomon_common.c:822-833
int encoding_id(int ranks, int encoding, int rank, int chunk_id);
// Reference: redset_rs_get_data_id, src/redset_reedsolomon_common.c:836-853
int data_id(int ranks, int encoding, int rank, int chunk_id);
// XOR segment of member `rank` in stripe `chunk` (rank != chunk).
// Reference: src/redset_xor.c:255-258, src/redset_xor_serial.c:216-227
inline int xor_segment(int rank, int chunk) { return chunk < rank ? chunk : chunk - 1; }

// Row selection for a decode.
// Reference: redset_rs_gaussian_solve_identify_rows,
// src/redset_reedsolomon_common.c:425-564.
void identify_rows(const std::vector<uint8_t>& mat, int ranks, int encoding, int missing,
                   const int* unknowns, std::vector<uint8_t>& m, std::vector<int>& rows);

// Runs the reference's in-place elimination (src/redset_reedsolomon_common.c:
// 570-630) on a symbolic right-hand side: returns T (missing x missing) such
// that the reference's solved buffer i equals sum_k T[i][k] * rhs_k. Because
// every step of that elimination is GF-linear in the buffers, applying T with
// one kernel pass reproduces the reference's bytes exactly, including the
// effect of its column swaps (which permute coefficients, never buffers).
std::vector<uint8_t> solve_transform(std::vector<uint8_t> m, int missing);

}  // namespace redset_hip
