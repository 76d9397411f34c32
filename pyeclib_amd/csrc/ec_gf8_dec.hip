// GF(2^8) decode / reconstruct instantiations (ISA-L layout).
#include "ec_kernels_impl.hpp"

namespace ecamd {

hipError_t launch_decode_gf8(const DecodeParams& p, hipStream_t stream) {
  switch (p.k) {
#define X(K) \
  case K:    \
    return launch_decode_k<Gf8, K>(p, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ecamd
