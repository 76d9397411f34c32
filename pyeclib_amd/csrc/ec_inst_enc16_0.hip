// GF(2^16) encode instantiations, k = 1..8 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC16(1) ECAMD_ENC16(2) ECAMD_ENC16(3) ECAMD_ENC16(4) ECAMD_ENC16(5) ECAMD_ENC16(6) ECAMD_ENC16(7) ECAMD_ENC16(8)
}  // namespace ecamd
