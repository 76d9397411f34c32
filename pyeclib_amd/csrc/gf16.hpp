// GF(2^16) arithmetic, generator and decode matrices for the rs_vand code.
//
// Field: GF(2^16) with primitive polynomial 0x1100B and generator x, symbols
// are little-endian 16-bit words of each fragment payload.  This is the field
// of liberasurecode's builtin `liberasurecode_rs_vand` backend
// (liberasurecode 1.8.0, src/builtin/rs_vand/rs_galois.c; pinned by
// /root/reference Dockerfile:14 and selected through pyeclib's
// PyECLib_EC_Types.liberasurecode_rs_vand = 6, src/pyeclib/enums.py:15).
//
// Generator: the unique systematic matrix G = V * inverse(V_top) of the
// (k+m) x k Vandermonde matrix V[i][j] = i^j (row 0 = [1,0..0]), with each
// parity column then scaled so that the first parity row is all ones
// (liberasurecode_rs_vand.c: create_non_systematic_vand_matrix +
// make_systematic_matrix).
#pragma once

#include <cstdint>
#include <vector>

namespace ecamd {

constexpr int kGfBits = 16;
constexpr uint32_t kGfPoly = 0x1100B;
constexpr int kMaxFragments = 32;  // liberasurecode EC_MAX_FRAGMENTS

class Gf16 {
 public:
  static const Gf16& get();
  uint16_t mul(uint16_t a, uint16_t b) const {
    if (a == 0 || b == 0) return 0;
    return exp_[log_[a] + log_[b]];
  }
  uint16_t inv(uint16_t a) const { return exp_[65535 - log_[a]]; }
  uint16_t div(uint16_t a, uint16_t b) const {
    if (a == 0) return 0;
    return exp_[log_[a] + 65535 - log_[b]];
  }

 private:
  Gf16();
  std::vector<uint32_t> log_;  // 65536
  std::vector<uint16_t> exp_;  // 2 * 65535 (sums need no reduction)
};

// Row-major square / rectangular GF(2^16) matrices.
using GfMatrix = std::vector<uint16_t>;

// (k+m) x k systematic generator; rows 0..k-1 are the identity.
GfMatrix make_generator(int k, int m);

// Inverse of an n x n matrix; returns false when singular.
bool invert(const GfMatrix& a, GfMatrix& out, int n);

// Nibble lookup tables for the GPU region kernel.
//
// For an R x C coefficient matrix M (R <= 4 rows per table set), entry
// (c, q, v) (u64) packs the four 16-bit products M[r][c] * (v << 4q) for
// r = 0..3 (zero for r >= R) at bits 16r..16r+15.  Because multiplication by
// a constant is GF(2)-linear,
//   M[r][c] * x = XOR_q entry(c, q, nibble_q(x)).r
// Layout [c][q >> 1][v][q & 1]: entry (c, q, v) at byte
// 512c + 256(q >> 1) + 16v + 8(q & 1), so the lookup address of a nibble is
// that nibble times 16 -- a byte of the input masked with 0xF0 -- plus a
// compile-time offset (ec_kernels_impl.hpp).  One table set is C * 512 B.
void build_nibble_tables(const uint16_t* rows, int nrows, int ncols, uint64_t* out);

// Eight-row tables (4 < R <= 8: one encode pass for m = 5..8 instead of two
// passes that each re-read the object).  Entry (c, q, v) is 16 bytes: the
// eight 16-bit products M[r][c] * (v << 4q), r = 0..7 (zero for r >= R), at
// bytes 2r..2r+1.  Layout [c][q][v]: entry at byte 1024c + 256q + 16v, so the
// lookup address is again the nibble times 16 plus a compile-time offset,
// read with one ds_read_b128 per nibble.  One table set is C * 1024 B.
constexpr int kRowsWide = 8;
void build_nibble_tables_x8(const uint16_t* rows, int nrows, int ncols, uint16_t* out);

}  // namespace ecamd
