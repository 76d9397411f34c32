// GF(2^16) encode instantiations, k = 22..31 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC16(22) ECAMD_ENC16(23) ECAMD_ENC16(24) ECAMD_ENC16(25) ECAMD_ENC16(26) ECAMD_ENC16(27) ECAMD_ENC16(28) ECAMD_ENC16(29) ECAMD_ENC16(30) ECAMD_ENC16(31)
}  // namespace ecamd
