"""ECDriver: the public erasure-coding API (reference: src/pyeclib/ec_iface.py).

Same keyword-only constructor, argument checks, messages, plugin loading and
method surface as the reference ``ECDriver`` (ec_iface.py:81-464); the default
plugin is the MI355X driver (``pyeclib_amd.core.ECPyECLibDriver``).  The new
ec_type is ``amd_rs_vand``; ``liberasurecode_rs_vand`` is served by the same
kernels since the two produce identical fragments.
"""
from __future__ import annotations

import warnings
from typing import Any, Collection, Sequence

from .enums import PyECLib_EC_Types, PyECLib_FRAGHDRCHKSUM_Types
from .exceptions import (ECBackendInitializationError, ECBackendInstanceInUse,  # noqa: F401
                         ECBackendInstanceNotAvailable, ECBackendNotSupported,
                         ECBadFragmentChecksum, ECDriverError, ECDriverErrorWithPosition,
                         ECInsufficientFragments, ECInvalidFragmentMetadata, ECInvalidParameter,
                         ECMethodNotImplemented, ECOutOfMemory)
from .utils import create_instance, positive_int_value

DEFAULT_DRIVER = "pyeclib_amd.core.ECPyECLibDriver"
PYECLIB_MAX_DATA = 32
PYECLIB_MAX_PARITY = 32

REQUIRED_METHODS = (
    "decode", "encode", "reconstruct", "fragments_needed", "min_parity_fragments_needed",
    "get_metadata", "verify_stripe_metadata", "get_segment_info",
)

# ec_type aliases that select a Hamming distance (ec_iface.py:145-152)
_HD_ALIASES = {"flat_xor_hd": ("flat_xor_hd", 3), "flat_xor_hd_3": ("flat_xor_hd", 3),
               "flat_xor_hd_4": ("flat_xor_hd", 4), "libphazr": ("libphazr", 1)}


def PyECLibVersion(z: int, y: int, x: int) -> int:
    return (z << 16) + (y << 8) + x


PYECLIB_MAJOR, PYECLIB_MINOR, PYECLIB_REV = 1, 8, 0
PYECLIB_VERSION = PyECLibVersion(PYECLIB_MAJOR, PYECLIB_MINOR, PYECLIB_REV)
__version__ = "%d.%d.%d" % (PYECLIB_MAJOR, PYECLIB_MINOR, PYECLIB_REV)


class ECDriver:
    """Encode, decode and reconstruct erasure-coded data."""

    def __init__(self, *, ec_type: str | None = None,
                 library_import_str: str = DEFAULT_DRIVER, k: int, m: int,
                 chksum_type: str = "none", validate: bool = False, local_parity: int = 0):
        self.k = self.m = self.hd = -1
        self.ec_type: Any = None
        self.chksum_type: Any = None
        if ec_type is None and library_import_str == DEFAULT_DRIVER:
            raise ECDriverError("Invalid Argument: either ec_type or library_import_str "
                                "must be provided")
        try:
            self.k = positive_int_value(k)
        except ValueError:
            raise ECDriverError("Invalid number of data fragments (k)")
        try:
            self.m = positive_int_value(m)
        except ValueError:
            raise ECDriverError("Invalid number of parity fragments (m)")
        self.local_parity = int(local_parity)

        if ec_type:
            if ec_type in _HD_ALIASES:
                ec_type, self.hd = _HD_ALIASES[ec_type]
            if ec_type not in PyECLib_EC_Types.__members__:
                raise ECBackendNotSupported("%s is not a valid EC type for PyECLib!" % ec_type)
            self.ec_type = PyECLib_EC_Types[ec_type]
            if ec_type in ("jerasure_rs_vand", "jerasure_rs_cauchy"):
                warnings.warn("Jerasure support is deprecated and may be removed in a "
                              "future release", FutureWarning, stacklevel=2)

        if chksum_type not in PyECLib_FRAGHDRCHKSUM_Types.__members__:
            raise ECDriverError("%s is not a valid checksum type for PyECLib!" % chksum_type)
        self.chksum_type = PyECLib_FRAGHDRCHKSUM_Types[chksum_type]
        self.validate = validate
        if self.hd == -1:
            self.hd = self.m
        self.library_import_str = library_import_str

        self.ec_lib_reference = create_instance(
            library_import_str, k=self.k, m=self.m, hd=self.hd, ec_type=self.ec_type,
            chksum_type=self.chksum_type, validate=int(self.validate),
            local_parity=self.local_parity)
        missing = " ".join(name for name in REQUIRED_METHODS
                           if not callable(getattr(self.ec_lib_reference, name, None)))
        if missing:
            raise ECDriverError("The following required methods are not implemented in %s: %s"
                                % (library_import_str, missing))

    def __repr__(self) -> str:
        if self.ec_type is None:
            name = "None"
        elif self.ec_type.name == "flat_xor_hd":
            name = "flat_xor_hd_%s" % self.hd
        else:
            name = self.ec_type.name
        return "%s(ec_type=%r, k=%d, m=%d)" % (type(self).__name__, name, self.k, self.m)

    def close(self) -> None:
        self.ec_lib_reference.close()

    def encode(self, data_bytes: bytes) -> list[bytes]:
        """k data fragments followed by m parity fragments."""
        return self.ec_lib_reference.encode(data_bytes)

    def decode(self, fragment_payloads: Sequence[bytes],
               ranges: list[tuple[int, int]] | None = None,
               force_metadata_checks: bool = False) -> bytes | list[bytes]:
        """The original buffer (or inclusive byte ranges of it) from any k fragments."""
        return self.ec_lib_reference.decode(fragment_payloads, ranges, force_metadata_checks)

    def reconstruct(self, available_fragment_payloads: Collection[bytes],
                    missing_fragment_indexes: list[int]) -> list[bytes]:
        """Rebuilt fragments, ordered by index, byte-identical to encode()'s."""
        return self.ec_lib_reference.reconstruct(available_fragment_payloads,
                                                 missing_fragment_indexes)

    def fragments_needed(self, reconstruction_indexes: list[int],
                         exclude_indexes: list[int] | None = None) -> list[int]:
        return self.ec_lib_reference.fragments_needed(reconstruction_indexes,
                                                      exclude_indexes or [])

    def min_parity_fragments_needed(self) -> int:
        return self.ec_lib_reference.min_parity_fragments_needed()

    def get_metadata(self, fragment: bytes, formatted: int = 0) -> bytes | dict:
        return self.ec_lib_reference.get_metadata(fragment, formatted)

    def verify_stripe_metadata(self, fragment_metadata_list: Sequence[bytes]) -> dict:
        return self.ec_lib_reference.verify_stripe_metadata(fragment_metadata_list)

    def get_segment_info(self, data_len: int, segment_size: int) -> dict:
        return self.ec_lib_reference.get_segment_info(data_len, segment_size)

    def get_segment_info_byterange(self, ranges: list[tuple[int, int]], data_len: int,
                                   segment_size: int) -> dict:
        """Per-range recipe {segment index: (begin, end)} (ec_iface.py:389-464)."""
        seg = self.ec_lib_reference.get_segment_info(data_len, segment_size)["segment_size"]
        recipe = {}
        for begin, end in ranges:
            first, last = begin // seg, end // seg
            if first == last:
                recipe[(begin, end)] = {first: (begin % seg, end % seg)}
                continue
            plan = {first: (begin % seg, seg - 1)}
            for mid in range(first + 1, last):
                plan[mid] = (0, seg - 1)
            plan[last] = (0, end % seg)
            recipe[(begin, end)] = plan
        return recipe


ALL_EC_TYPES = [
    "jerasure_rs_vand", "jerasure_rs_cauchy", "flat_xor_hd_3", "flat_xor_hd_4",
    "isa_l_rs_vand", "shss", "liberasurecode_rs_vand", "isa_l_rs_cauchy", "libphazr",
    "isa_l_rs_vand_inv", "isa_l_rs_lrc", "amd_rs_vand",
]


def check_backend_available(backend_name: str) -> bool:
    from . import _native
    key = "flat_xor_hd" if backend_name.startswith("flat_xor_hd") else backend_name
    member = PyECLib_EC_Types[key]
    return bool(member) and _native.check_backend_available(member.value)


def _valid_ec_types() -> list[str]:
    return [name for name in ALL_EC_TYPES if check_backend_available(name)]


def _liberasurecode_version() -> str:
    from . import _native
    v = _native.get_liberasurecode_version()
    return "%d.%d.%d" % ((v >> 16) & 0xFF, (v >> 8) & 0xFF, v & 0xFF)


VALID_EC_TYPES = _valid_ec_types()
LIBERASURECODE_VERSION = _liberasurecode_version()
