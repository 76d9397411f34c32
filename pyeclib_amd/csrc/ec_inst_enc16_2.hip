// GF(2^16) encode instantiations, k = 15..21 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC16(15) ECAMD_ENC16(16) ECAMD_ENC16(17) ECAMD_ENC16(18) ECAMD_ENC16(19) ECAMD_ENC16(20) ECAMD_ENC16(21)
}  // namespace ecamd
