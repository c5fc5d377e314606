// stripe_map.h -- which cells a stripe reads and writes, and with which
// GF(2^8) coefficients, independent of where the cells live (device set
// layout, pinned staging buffers, files). Shared by the device plans
// (redset_hip.cpp) and the host streaming pipeline (stream_pipeline.cpp).
#pragma once

#include <cstdint>
#include <vector>

struct redset_hip_rs {
  int ranks;
  int encoding;
  std::vector<uint8_t> mat;  // (p+e) x p
};

namespace redset_hip {

enum CellKind { kData = 0, kParity = 1 };

// A cell of the set: member `rank`'s logical-file segment `index` (kData) or
// redundancy slot `index` (kParity).
struct CellRef {
  int rank;
  int kind;
  int index;
};

// outputs = coef (nout x nin, row-major) * inputs, byte by byte
struct StripeMap {
  std::vector<CellRef> in;
  std::vector<CellRef> out;
  std::vector<uint8_t> coef;
  bool xor_only = false;  // XOR scheme: every coefficient is 1
  bool accumulate = false;  // XOR into the outputs (redset_hip_plan_combine jobs)
};

// cell of member `rank` in RS stripe `chunk` (src/redset_reedsolomon_common.c:822-853)
CellRef rs_cell(const redset_hip_rs* rs, int rank, int chunk);

// RS encode of stripe c: d data cells -> e parity cells (row p+i at member
// (c - i) mod p's slot i). src/redset_reedsolomon.c:329-376.
int rs_encode_map(const redset_hip_rs* rs, int c, StripeMap& m);

// RS rebuild of stripe c: the lost members' cells from the surviving cells
// with a nonzero decode coefficient. Reproduces redset_rs_reduce_decode +
// redset_rs_gaussian_solve (common.c:855-899, :570-630) as one linear map.
int rs_rebuild_map(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int c, StripeMap& m);

// decode map of stripe c as (missing x p); column s = member s's cell
int rs_decode_matrix(const redset_hip_rs* rs, int missing, const int* rebuild_ranks, int c, std::vector<uint8_t>& D);

// XOR stripe c: member c's parity = XOR of the other members' cells
// (src/redset_xor.c:251-266); rebuild of `root` from all others.
int xor_encode_map(int ranks, int c, StripeMap& m);
int xor_rebuild_map(int ranks, int root, int c, StripeMap& m);

// error reporting shared by all C-ABI entry points
int fail(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

// Enqueue one stripe's map on `stream` over cells at the given device
// pointers (in[i] for m.in[i], out[j] for m.out[j]), split into passes of
// <= 16 inputs x <= 4 outputs. blocks_total: grid size budget (0 = fill GPU).
// accumulate: XOR into the outputs instead of overwriting them.
int run_stripe(const StripeMap& m, const uint8_t* const* in, uint8_t* const* out, size_t nbytes, void* stream,
               int blocks_total, bool accumulate = false);

}  // namespace redset_hip
