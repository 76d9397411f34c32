// GF(2^8) decode / reconstruct instantiations, k = 22..31 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC8(22) ECAMD_DEC8(23) ECAMD_DEC8(24) ECAMD_DEC8(25) ECAMD_DEC8(26) ECAMD_DEC8(27) ECAMD_DEC8(28) ECAMD_DEC8(29) ECAMD_DEC8(30) ECAMD_DEC8(31)
}  // namespace ecamd
