// GF(2^8) decode / reconstruct instantiations, k = 1..8 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC8(1) ECAMD_DEC8(2) ECAMD_DEC8(3) ECAMD_DEC8(4) ECAMD_DEC8(5) ECAMD_DEC8(6) ECAMD_DEC8(7) ECAMD_DEC8(8)
}  // namespace ecamd
