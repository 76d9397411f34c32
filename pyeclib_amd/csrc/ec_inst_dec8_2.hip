// GF(2^8) decode / reconstruct instantiations, k = 15..21 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC8(15) ECAMD_DEC8(16) ECAMD_DEC8(17) ECAMD_DEC8(18) ECAMD_DEC8(19) ECAMD_DEC8(20) ECAMD_DEC8(21)
}  // namespace ecamd
