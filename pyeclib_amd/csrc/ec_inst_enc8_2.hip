// GF(2^8) encode instantiations, k = 15..21 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC8(15) ECAMD_ENC8(16) ECAMD_ENC8(17) ECAMD_ENC8(18) ECAMD_ENC8(19) ECAMD_ENC8(20) ECAMD_ENC8(21)
}  // namespace ecamd
