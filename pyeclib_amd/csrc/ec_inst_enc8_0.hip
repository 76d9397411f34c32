// GF(2^8) encode instantiations, k = 1..8 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC8(1) ECAMD_ENC8(2) ECAMD_ENC8(3) ECAMD_ENC8(4) ECAMD_ENC8(5) ECAMD_ENC8(6) ECAMD_ENC8(7) ECAMD_ENC8(8)
}  // namespace ecamd
