// GF(2^16) decode / reconstruct instantiations, k = 15..21 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC16(15) ECAMD_DEC16(16) ECAMD_DEC16(17) ECAMD_DEC16(18) ECAMD_DEC16(19) ECAMD_DEC16(20) ECAMD_DEC16(21)
}  // namespace ecamd
