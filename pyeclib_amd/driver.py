"""ECAMDDriver: the driver plugin behind ``ECDriver`` for the GPU ec_types.

Reference counterpart: ``pyeclib.core.ECPyECLibDriver`` (src/pyeclib/core.py:
40-215).  Same constructor signature (what ECDriver passes through
``create_instance``, ec_iface.py:179-188), same eight required methods
(ec_iface.py:193-214), same validation and error messages; the work is done
by libpyeclib_amd.so through ``_native``.

It also plugs into an unmodified upstream pyeclib:
``pyeclib.ec_iface.ECDriver(k=10, m=4, ec_type='liberasurecode_rs_vand',
library_import_str='pyeclib_amd.driver.ECAMDDriver')``.
"""
from __future__ import annotations

from typing import Any, Collection

from . import _native
from .exceptions import ECDriverErrorWithPosition

_CLOSED_MESSAGE = "erasure coding handle is closed"


def _wants_crc(chksum_type: Any) -> bool:
    # accept this package's enum, upstream pyeclib's enum, or a plain name
    name = getattr(chksum_type, "name", chksum_type)
    return name == "inline_crc32"


class ECAMDDriver:
    def __init__(self, k: int, m: int, hd: int, ec_type: Any = None,
                 chksum_type: Any = "none", validate: bool = False, local_parity: int = 0):
        self.k = k
        self.m = m
        self.hd = hd
        self.local_parity = local_parity
        self.ec_type = ec_type
        self.chksum_type = chksum_type
        self.inline_chksum = 1 if _wants_crc(chksum_type) else 0
        self.algsig_chksum = 0
        backend = getattr(ec_type, "value", ec_type)
        self._handle: _native.PyECLibHandle | None = _native.init(
            k, m, backend, hd, self.inline_chksum, self.algsig_chksum, int(bool(validate)),
            local_parity)

    def __repr__(self) -> str:
        return "%s(k=%r, m=%r, hd=%r, ec_type=%r, chksum_type=%r)" % (
            type(self).__name__, self.k, self.m, self.hd, self.ec_type, self.chksum_type)

    # -- lifecycle (core.py:86-97) --
    def close(self) -> None:
        handle, self._handle = self._handle, None
        if handle is not None:
            _native.destroy(handle)

    @property
    def handle(self) -> _native.PyECLibHandle:
        if self._handle is None:
            raise _native._exception_class("ECBackendInstanceNotAvailable")(_CLOSED_MESSAGE)
        return self._handle

    # -- helpers --
    def _fragment_len(self, method: str, fragments: list[bytes]) -> int:
        """All fragments must be non-empty and of equal length (core.py:102-124)."""
        where = "ECPyECLibDriver.%s" % method
        if not fragments:
            raise _native._exception_class("ECDriverError")("No fragments payload in %s" % where)
        size = len(fragments[0])
        if size == 0:
            raise _position_error("Invalid fragment payload in %s" % where, 0)
        for pos, frag in enumerate(fragments[1:], start=2):
            if len(frag) != size:
                raise _position_error("Invalid fragment payload in %s" % where, pos)
        return size

    # -- the eight required methods --
    def encode(self, data_bytes: bytes) -> list[bytes]:
        return _native.encode(self.handle, data_bytes)

    def decode(self, fragment_payloads: Collection[bytes],
               ranges: list[tuple[int, int]] | None = None,
               force_metadata_checks: bool = False) -> bytes | list[bytes]:
        frags = list(fragment_payloads)
        size = self._fragment_len("decode", frags)
        if len(frags) < self.k:
            raise _native._exception_class("ECInsufficientFragments")(
                "Not enough fragments given in ECPyECLibDriver.decode")
        return _native.decode(self.handle, frags, size, ranges, force_metadata_checks)

    def reconstruct(self, fragment_payloads: Collection[bytes],
                    indexes_to_reconstruct: list[int]) -> list[bytes]:
        """One index at a time, ascending, each result fed back as an input
        (core.py:150-176) -- so parity can be rebuilt after missing data."""
        frags = list(fragment_payloads)
        size = self._fragment_len("reconstruct", frags)
        indexes_to_reconstruct.sort()  # the reference sorts the caller's list in place
        rebuilt = []
        for idx in list(indexes_to_reconstruct):
            frag = _native.reconstruct(self.handle, frags, size, idx)
            rebuilt.append(frag)
            frags.append(frag)
        return rebuilt

    def fragments_needed(self, reconstruct_indexes: list[int],
                         exclude_indexes: list[int]) -> list[int]:
        return _native.get_required_fragments(self.handle, reconstruct_indexes, exclude_indexes)

    def min_parity_fragments_needed(self) -> int:
        return 1

    def get_metadata(self, fragment: bytes, formatted: int = 0) -> bytes | dict:
        return _native.get_metadata(self.handle, fragment, formatted)

    def verify_stripe_metadata(self, fragment_metadata_list: list[bytes]) -> dict:
        return _native.check_metadata(self.handle, fragment_metadata_list)

    def get_segment_info(self, data_len: int, segment_size: int) -> dict:
        return _native.get_segment_info(self.handle, data_len, segment_size)


def _position_error(msg: str, pos: int) -> Exception:
    cls = _native._exception_class("ECDriverErrorWithPosition")
    return cls(msg, pos) if cls is not None else ECDriverErrorWithPosition(msg, pos)
