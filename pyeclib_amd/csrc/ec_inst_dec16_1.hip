// GF(2^16) decode / reconstruct instantiations, k = 9..14 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_DEC16(9) ECAMD_DEC16(10) ECAMD_DEC16(11) ECAMD_DEC16(12) ECAMD_DEC16(13) ECAMD_DEC16(14)
}  // namespace ecamd
