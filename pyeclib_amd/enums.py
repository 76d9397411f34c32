"""Backend and checksum enumerations (reference: src/pyeclib/enums.py).

Values mirror liberasurecode's ``ec_backend_id_t`` and
``ec_checksum_type_t``; ``amd_rs_vand`` (11) is the new ec_type served by the
MI355X kernels.  Its fragments are byte-identical to liberasurecode_rs_vand's
(they carry backend_id 6), so either name can decode the other's output.
"""
from enum import Enum, unique

_BACKENDS = [
    ("jerasure_rs_vand", 1), ("jerasure_rs_cauchy", 2), ("flat_xor_hd", 3),
    ("isa_l_rs_vand", 4), ("shss", 5), ("liberasurecode_rs_vand", 6),
    ("isa_l_rs_cauchy", 7), ("libphazr", 8), ("isa_l_rs_vand_inv", 9),
    ("isa_l_rs_lrc", 10), ("amd_rs_vand", 11),
]

# Functional API keeps member order = value order (values start at 1: 0 is falsy).
PyECLib_EC_Types = unique(Enum("PyECLib_EC_Types", _BACKENDS, module=__name__))

PyECLib_FRAGHDRCHKSUM_Types = unique(
    Enum("PyECLib_FRAGHDRCHKSUM_Types", [("none", 1), ("inline_crc32", 2)], module=__name__)
)

# ec_types whose arithmetic this package runs on the GPU: GF(2^16) rs_vand,
# and the GF(2^8) ISA-L Vandermonde / Cauchy codes
GPU_EC_TYPES = ("liberasurecode_rs_vand", "amd_rs_vand", "isa_l_rs_vand", "isa_l_rs_cauchy")
