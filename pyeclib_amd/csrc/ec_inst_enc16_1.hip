// GF(2^16) encode instantiations, k = 9..14 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC16(9) ECAMD_ENC16(10) ECAMD_ENC16(11) ECAMD_ENC16(12) ECAMD_ENC16(13) ECAMD_ENC16(14)
}  // namespace ecamd
