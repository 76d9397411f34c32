// GF(2^16) encode instantiations (liberasurecode_rs_vand).
#include "ec_kernels_impl.hpp"

namespace ecamd {

namespace {
template <int K>
hipError_t encode_gf16_k(const EncodeParams& p, hipStream_t stream) {
  // <= 2 rows per pass: the low dword of each table entry is enough
  switch (p.nrows) {
    case 1:
      return launch_encode_k<Gf16<1>, K, 1>(p, stream);
    case 2:
      return launch_encode_k<Gf16<1>, K, 2>(p, stream);
    case 3:
      return launch_encode_k<Gf16<2>, K, 3>(p, stream);
    case 4:
      return launch_encode_k<Gf16<2>, K, 4>(p, stream);
    default:
      return hipErrorInvalidValue;
  }
}
}  // namespace

hipError_t launch_encode_gf16(const EncodeParams& p, hipStream_t stream) {
  switch (p.k) {
#define X(K) \
  case K:    \
    return encode_gf16_k<K>(p, stream);
    ECAMD_K_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace ecamd
