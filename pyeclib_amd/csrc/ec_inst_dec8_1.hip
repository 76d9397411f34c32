// GF(2^8) decode / reconstruct instantiations, k = 9..14 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC8(9) ECAMD_DEC8(10) ECAMD_DEC8(11) ECAMD_DEC8(12) ECAMD_DEC8(13) ECAMD_DEC8(14)
}  // namespace ecamd
