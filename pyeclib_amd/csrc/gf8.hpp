// GF(2^8) arithmetic and the ISA-L generator matrices behind liberasurecode's
// isa_l_rs_vand (backend id 4) and isa_l_rs_cauchy (id 7) codes
// (PyECLib_EC_Types, src/pyeclib/enums.py:13,16; ISA-L v2.32.0 pinned at
// Dockerfile:15).  ISA-L is an external dependency absent from this
// container, so the construction is restated from its published algorithm
// (erasure_code/ec_base.c): field polynomial 0x11D with generator 2,
//   gf_gen_rs_matrix:      rows k.. : a[i][j] = 2^((i-k) * j)
//   gf_gen_cauchy1_matrix: rows k.. : a[i][j] = 1 / (i ^ j)
// above a k x k identity.  Symbols are single bytes.
#pragma once

#include <cstdint>
#include <vector>

#include "gf16.hpp"  // GfMatrix

namespace ecamd {

constexpr uint32_t kGf8Poly = 0x11D;

class Gf8 {
 public:
  static const Gf8& get();
  uint16_t mul(uint16_t a, uint16_t b) const {
    if (a == 0 || b == 0) return 0;
    return exp_[log_[a] + log_[b]];
  }
  uint16_t inv(uint16_t a) const { return exp_[255 - log_[a]]; }

 private:
  Gf8();
  uint16_t log_[256];
  uint16_t exp_[512];
};

// (k+m) x k systematic generators (values < 256).
GfMatrix make_isal_rs_matrix(int k, int m);      // gf_gen_rs_matrix
GfMatrix make_isal_cauchy_matrix(int k, int m);  // gf_gen_cauchy1_matrix

// Inverse over GF(2^8); false when singular (ISA-L gf_invert_matrix).
bool invert8(const GfMatrix& a, GfMatrix& out, int n);

// Nibble tables for the GF(2^8) kernel: for an R x C matrix (R <= 4 rows per
// set), entry [c][q][v] (u32, q = 0..1) packs the products M[r][c] * (v << 4q)
// for r = 0..3 at bits 8r..8r+7.  One set is C * 128 B.
void build_nibble_tables8(const uint16_t* rows, int nrows, int ncols, uint32_t* out);

}  // namespace ecamd
