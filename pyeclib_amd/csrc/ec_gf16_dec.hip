// GF(2^16) decode / reconstruct instantiations (liberasurecode_rs_vand).
#include "ec_kernels_impl.hpp"

namespace ecamd {

hipError_t launch_decode_gf16(const DecodeParams& p, hipStream_t stream) {
  // every object's n_out is <= 4; the row count only selects the entry width
  const uint32_t rows = p.reconstruct ? 1u : std::min<uint32_t>(p.m, kRowsPerPass);
  const bool narrow = rows <= 2;
  switch (p.k) {
#define X(K)                                               \
  case K:                                                  \
    return narrow ? launch_decode_k<Gf16<1>, K>(p, stream) \
                  : launch_decode_k<Gf16<2>, K>(p, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ecamd
