// GF(2^16) decode / reconstruct instantiations, k = 22..31 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC16(22) ECAMD_DEC16(23) ECAMD_DEC16(24) ECAMD_DEC16(25) ECAMD_DEC16(26) ECAMD_DEC16(27) ECAMD_DEC16(28) ECAMD_DEC16(29) ECAMD_DEC16(30) ECAMD_DEC16(31)
}  // namespace ecamd
