// Field dispatch of the region kernels (ec_kernels.hpp).
#include "ec_kernels.hpp"

namespace ecamd {

hipError_t launch_encode(const EncodeParams& p, hipStream_t stream) {
  return p.w == 8 ? launch_encode_gf8(p, stream) : launch_encode_gf16(p, stream);
}

hipError_t launch_decode(const DecodeParams& p, hipStream_t stream) {
  return p.w == 8 ? launch_decode_gf8(p, stream) : launch_decode_gf16(p, stream);
}

}  // namespace ecamd
