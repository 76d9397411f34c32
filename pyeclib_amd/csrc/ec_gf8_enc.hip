// GF(2^8) encode instantiations (ISA-L layout: isa_l_rs_vand / isa_l_rs_cauchy).
#include "ec_kernels_impl.hpp"

namespace ecamd {

hipError_t launch_encode_gf8(const EncodeParams& p, hipStream_t stream) {
  switch (p.k) {
#define X(K) \
  case K:    \
    return launch_encode_rows<Gf8, K>(p, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ecamd
