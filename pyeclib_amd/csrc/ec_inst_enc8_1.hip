// GF(2^8) encode instantiations, k = 9..14 (see ec_inst.hpp).
#include "ec_inst.hpp"

namespace ecamd {
ECAMD_ENC8(9) ECAMD_ENC8(10) ECAMD_ENC8(11) ECAMD_ENC8(12) ECAMD_ENC8(13) ECAMD_ENC8(14)
}  // namespace ecamd
