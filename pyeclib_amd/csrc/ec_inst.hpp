// Per-k kernel instantiations.  Each ec_inst_*.hip file instantiates one
// (field, operation) family for a range of k, so the kernels compile in
// parallel; ec_dispatch.cpp switches on k.  Per-k entry points:
//   launch_enc16_K  GF(2^16) encode (liberasurecode_rs_vand)
//   launch_dec16_K  GF(2^16) decode / reconstruct
//   launch_enc8_K   GF(2^8) encode (ISA-L layout: isa_l_rs_vand / _cauchy)
//   launch_dec8_K   GF(2^8) decode / reconstruct
#pragma once

#include "ec_kernels_impl.hpp"

namespace ecamd {

// GF(2^16) encode: <= 2 rows per pass need only the low dword of each table
// entry (Gf16<1>); 5..8 rows run in one eight-row pass (Gf16x8).  A pass is
// built for 2, 4 or 8 rows; the rows past p.nrows are dropped
// (ec_kernels_impl.hpp parity_row), so 1, 3, 5..7 rows need no kernels of
// their own.
#define ECAMD_ENC16(K)                                                      \
  hipError_t launch_enc16_##K(const EncodeParams& p, hipStream_t s) {       \
    switch (p.nrows) {                                                      \
      case 1: case 2: return launch_encode_k<Gf16<1>, K, 2>(p, s);          \
      case 3: case 4: return launch_encode_k<Gf16<2>, K, 4>(p, s);          \
      case 5: case 6: case 7: case 8:                                       \
        return launch_encode_k<Gf16x8, K, 8>(p, s);                         \
      default: return hipErrorInvalidValue;                                 \
    }                                                                       \
  }

// GF(2^16) decode: reconstruct has one row (Gf16<1>); decode with m <= 2 has
// at most 2 rows per pass; the generic (multi-pass) mode exists only for
// m > 4, so always 4-row entries.
#define ECAMD_DEC16(K)                                                          \
  hipError_t launch_dec16_##K(const DecodeParams& p, hipStream_t s) {           \
    const bool narrow = std::min<uint32_t>(p.m, kRowsPerPass) <= 2;            \
    switch (p.mode) {                                                           \
      case kReconstruct: return launch_decode_mode<Gf16<1>, K, kReconstruct>(p, s); \
      case kDecode:                                                             \
        return narrow ? launch_decode_mode<Gf16<1>, K, kDecode>(p, s)          \
                      : launch_decode_mode<Gf16<2>, K, kDecode>(p, s);         \
      default: return launch_decode_mode<Gf16<2>, K, kDecodeGeneric>(p, s);     \
    }                                                                           \
  }

// GF(2^8): one table entry carries four rows whatever the pass holds, so
// every pass runs the four-row kernel (rows past p.nrows dropped).
#define ECAMD_ENC8(K)                                                 \
  hipError_t launch_enc8_##K(const EncodeParams& p, hipStream_t s) {  \
    if (p.nrows < 1 || p.nrows > 4) return hipErrorInvalidValue;      \
    return launch_encode_k<Gf8, K, 4>(p, s);                          \
  }

#define ECAMD_DEC8(K)                                                           \
  hipError_t launch_dec8_##K(const DecodeParams& p, hipStream_t s) {            \
    switch (p.mode) {                                                           \
      case kReconstruct: return launch_decode_mode<Gf8, K, kReconstruct>(p, s); \
      case kDecode: return launch_decode_mode<Gf8, K, kDecode>(p, s);           \
      default: return launch_decode_mode<Gf8, K, kDecodeGeneric>(p, s);         \
    }                                                                           \
  }

}  // namespace ecamd
