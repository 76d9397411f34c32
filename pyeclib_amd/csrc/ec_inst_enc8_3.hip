// GF(2^8) encode instantiations, k = 22..31 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC8(22) ECAMD_ENC8(23) ECAMD_ENC8(24) ECAMD_ENC8(25) ECAMD_ENC8(26) ECAMD_ENC8(27) ECAMD_ENC8(28) ECAMD_ENC8(29) ECAMD_ENC8(30) ECAMD_ENC8(31)
}  // namespace ecamd
