// GF(2^16) decode / reconstruct instantiations, k = 1..8 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC16(1) ECAMD_DEC16(2) ECAMD_DEC16(3) ECAMD_DEC16(4) ECAMD_DEC16(5) ECAMD_DEC16(6) ECAMD_DEC16(7) ECAMD_DEC16(8)
}  // namespace ecamd
