"""Python binding of libpyeclib_amd.so -- the counterpart of pyeclib's
``pyeclib_c`` extension (src/pyeclib_c/pyeclib_c.c) for the MI355X backend.

It exposes the same eleven module functions as the reference method table
(pyeclib_c.c:1221-1234) with the same argument meaning, return shapes and
error behaviour, but binds them through ctypes to the liberasurecode-shaped
C ABI declared in include/erasurecode_amd.h instead of to liberasurecode.

The shared library is mandatory: importing this module raises ImportError
when it is missing or cannot be loaded, and there is no CPU fallback for the
GF(2^16) arithmetic.
"""
from __future__ import annotations

import ctypes
import math
import os
import threading
from typing import Any, Sequence

from . import exceptions as _local_exc

_LIB_NAME = "libpyeclib_amd.so"
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), _LIB_NAME)
# Developer A/B runs only (tools/ab_bench.py): load another build of the
# same C ABI, e.g. tools/build/libpyeclib_amd_ab.so (`make -C
# pyeclib_amd/csrc ab`).  The product library has no switches of its own.
if os.environ.get("PYECLIB_AMD_LIBRARY"):
    _LIB_PATH = os.path.abspath(os.environ["PYECLIB_AMD_LIBRARY"])

if not os.path.exists(_LIB_PATH):
    raise ImportError(
        f"{_LIB_PATH} is missing: build it with `make -C pyeclib_amd/csrc` "
        "(or __graft_entry__.build()); pyeclib_amd has no CPU fallback"
    )



def _share_torch_hip_runtime() -> None:
    """Use the HIP runtime PyTorch ships, when PyTorch is installed.

    Both this library (SONAME dependency libamdhip64.so.7) and torch's
    libtorch_hip need a HIP runtime; two copies in one process (ROCm's and
    torch's bundled one) make whichever initialises second fail.  Loading
    torch's copy first by path (without importing torch) lets our dependency
    bind to it by SONAME, and torch later re-uses the same file.  Set
    PYECLIB_AMD_HIP_RUNTIME=system to keep ROCm's runtime instead.
    """
    if os.environ.get("PYECLIB_AMD_HIP_RUNTIME") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    for loc in (spec.submodule_search_locations or []) if spec else []:
        cand = os.path.join(loc, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            return


_share_torch_hip_runtime()
lib = ctypes.CDLL(_LIB_PATH)


def build_id() -> str:
    """First 16 hex digits of the SHA-256 of the loaded library file (ties
    profiles/pmc_summary.json counters to the build they were measured on)."""
    import hashlib
    with open(_LIB_PATH, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]

# ---- liberasurecode constants (include/erasurecode_amd.h) ----
EBACKENDNOTSUPP = 200
EECMETHODNOTIMPL = 201
EBACKENDINITERR = 202
EBACKENDINUSE = 203
EBACKENDNOTAVAIL = 204
EBADCHKSUM = 205
EINVALIDPARAMS = 206
EBADHEADER = 207
EINSUFFFRAGS = 208
ENOMEM = 12
EDEADLK = 35
EINVAL = 22

CHKSUM_NONE = 1
CHKSUM_CRC32 = 2
CHKSUM_MD5 = 3
HEADER_SIZE = 80
METADATA_SIZE = 59


class ECArgs(ctypes.Structure):
    class _Priv(ctypes.Union):
        class _Null(ctypes.Structure):
            _fields_ = [("arg1", ctypes.c_uint64)]

        class _Reserved(ctypes.Structure):
            _fields_ = [("x", ctypes.c_uint64), ("y", ctypes.c_uint64),
                        ("z", ctypes.c_uint64), ("a", ctypes.c_uint64)]

        _fields_ = [("null_args", _Null), ("reserved", _Reserved)]

    _fields_ = [("k", ctypes.c_int), ("m", ctypes.c_int), ("w", ctypes.c_int),
                ("hd", ctypes.c_int), ("priv_args1", _Priv),
                ("priv_args2", ctypes.c_void_p), ("ct", ctypes.c_int)]


class FragmentMetadata(ctypes.Structure):
    _pack_ = 1
    _fields_ = [("idx", ctypes.c_uint32), ("size", ctypes.c_uint32),
                ("frag_backend_metadata_size", ctypes.c_uint32),
                ("orig_data_size", ctypes.c_uint64), ("chksum_type", ctypes.c_uint8),
                ("chksum", ctypes.c_uint32 * 8), ("chksum_mismatch", ctypes.c_uint8),
                ("backend_id", ctypes.c_uint8), ("backend_version", ctypes.c_uint32)]


assert ctypes.sizeof(FragmentMetadata) == METADATA_SIZE

_P = ctypes.POINTER
_cpp = _P(ctypes.c_char_p)
_sig = {
    "liberasurecode_backend_available": (ctypes.c_int, [ctypes.c_int]),
    "liberasurecode_instance_create": (ctypes.c_int, [ctypes.c_int, _P(ECArgs)]),
    "liberasurecode_instance_destroy": (ctypes.c_int, [ctypes.c_int]),
    "liberasurecode_encode": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                             _P(_P(ctypes.c_void_p)), _P(_P(ctypes.c_void_p)),
                                             _P(ctypes.c_uint64)]),
    "liberasurecode_encode_cleanup": (ctypes.c_int, [ctypes.c_int, _P(ctypes.c_void_p),
                                                     _P(ctypes.c_void_p)]),
    "liberasurecode_decode": (ctypes.c_int, [ctypes.c_int, _cpp, ctypes.c_int, ctypes.c_uint64,
                                             ctypes.c_int, _P(ctypes.c_void_p),
                                             _P(ctypes.c_uint64)]),
    "liberasurecode_decode_cleanup": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p]),
    "liberasurecode_reconstruct_fragment": (ctypes.c_int, [ctypes.c_int, _cpp, ctypes.c_int,
                                                           ctypes.c_uint64, ctypes.c_int,
                                                           ctypes.c_void_p]),
    "liberasurecode_fragments_needed": (ctypes.c_int, [ctypes.c_int, _P(ctypes.c_int),
                                                       _P(ctypes.c_int), _P(ctypes.c_int)]),
    "liberasurecode_get_fragment_metadata": (ctypes.c_int, [ctypes.c_void_p,
                                                            _P(FragmentMetadata)]),
    "liberasurecode_verify_stripe_metadata": (ctypes.c_int, [ctypes.c_int, _cpp, ctypes.c_int]),
    "liberasurecode_get_aligned_data_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64]),
    "liberasurecode_get_minimum_encode_size": (ctypes.c_int, [ctypes.c_int]),
    "liberasurecode_get_fragment_size": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "liberasurecode_get_version": (ctypes.c_uint32, []),
    "ecamd_blocksize": (ctypes.c_uint64, [ctypes.c_int, ctypes.c_uint64]),
    "ecamd_device": (ctypes.c_int, [ctypes.c_int]),
    "ecamd_decode_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           _P(ctypes.c_int), ctypes.c_int,
                                           _P(ctypes.c_uint16), _P(ctypes.c_int)]),
    "ecamd_layout_supported": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_uint64]),
    "ecamd_encode_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_void_p]),
    "ecamd_decode_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                          _P(ctypes.c_uint32), ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p]),
    "ecamd_reconstruct_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                               _P(ctypes.c_uint32), _P(ctypes.c_int),
                                               ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_void_p]),
    "ecamd_encode_host_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_uint64]),
    "ecamd_decode_host_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint64, ctypes.c_int,
                                               _P(ctypes.c_uint32), ctypes.c_void_p,
                                               ctypes.c_uint64]),
    "ecamd_reconstruct_host_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p,
                                                    ctypes.c_uint64, ctypes.c_uint64,
                                                    ctypes.c_int, _P(ctypes.c_uint32),
                                                    _P(ctypes.c_int), ctypes.c_void_p,
                                                    ctypes.c_uint64]),
}
_sig.update({
    "ecamd_encode_into": (ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64,
                                         _P(ctypes.c_void_p), ctypes.c_uint64]),
    "ecamd_decode_into": (ctypes.c_int, [ctypes.c_int, _cpp, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]),
    "ecamd_call_phases": (ctypes.c_int, [ctypes.c_int, _P(ctypes.c_double), ctypes.c_int]),
    "ecamd_last_device_error": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64]),
    "ecamd_instance_stats": (ctypes.c_int, [ctypes.c_int, _P(ctypes.c_uint64), ctypes.c_int]),
})
EXPORTS = tuple(_sig)
for _name, (_res, _args) in _sig.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

# ---- error mapping: pyeclib_c_seterr (pyeclib_c.c:125-183) ----
_ERRORS = {
    -EBACKENDNOTAVAIL: ("ECBackendInstanceNotAvailable", "Backend instance not found"),
    -EINSUFFFRAGS: ("ECInsufficientFragments", "Insufficient number of fragments"),
    -EBACKENDNOTSUPP: ("ECBackendNotSupported", "Backend not supported"),
    -EINVALIDPARAMS: ("ECInvalidParameter", "Invalid arguments"),
    -EBADCHKSUM: ("ECBadFragmentChecksum", "Fragment integrity check failed"),
    -EBADHEADER: ("ECInvalidFragmentMetadata", "Fragment integrity check failed"),
    -ENOMEM: ("ECOutOfMemory", "Out of memory"),
    EDEADLK: ("ECDriverError", "Thread already owns lock"),
    EINVAL: ("ECDriverError", "Invalid read-write lock"),
}


def _exception_class(name: str) -> type:
    """Resolve the exception class by name at raise time, as the reference
    does (pyeclib_c.c:176 imports pyeclib.exceptions).  When the upstream
    pyeclib package is importable its classes are used, so callers that catch
    pyeclib.exceptions.* keep working with this backend plugged in."""
    try:
        import pyeclib.exceptions as upstream  # type: ignore
        cls = getattr(upstream, name, None)
        if cls is not None:
            return cls
    except ImportError:
        pass
    return getattr(_local_exc, name)


def last_device_error() -> tuple[int, str]:
    """The device-runtime error behind this thread's last -EBACKENDINITERR
    (ecamd_last_device_error): (code, "name: text"), code 0 when none."""
    buf = ctypes.create_string_buffer(256)
    code = int(lib.ecamd_last_device_error(buf, len(buf)))
    return code, buf.value.decode(errors="replace")


def instance_stats(handle: "PyECLibHandle") -> dict:
    """ecamd_instance_stats: the instance's stream marks, the process's
    pinned staging bytes and budget, and its single-object calls that staged
    through HBM (tests)."""
    out = (ctypes.c_uint64 * 5)()
    ret = lib.ecamd_instance_stats(handle.desc, out, 5)
    if ret < 0:
        raise_error(ret, "ecamd_instance_stats")
    return {"marks": out[0], "pinned_bytes": out[1], "dma_calls": out[2], "pinned_budget": out[3],
            "direct_calls": out[4]}


def raise_error(ret: int, prefix: str) -> None:
    name, msg = _ERRORS.get(ret, ("ECDriverError", "Unknown error"))
    if ret == -EBACKENDINITERR:
        # pyeclib says "Unknown error" here (pyeclib_c.c:170-173); a device
        # fault behind it is named, so the cause is not lost in the mapping
        code, text = last_device_error()
        if code:
            msg = f"{msg} (device: {text})"
    cls = _exception_class(name)
    raise cls(f"{prefix} ERROR: {msg}. Please inspect syslog for liberasurecode error report.")


# ---- handle (the reference's PyCapsule "pyeclib_handle", pyeclib_c.h:30-37) ----
class PyECLibHandle:
    __slots__ = ("desc", "k", "m", "hd", "ct", "_lock", "__weakref__")

    def __init__(self, desc: int, k: int, m: int, hd: int, ct: int):
        self.desc = desc
        self.k = k
        self.m = m
        self.hd = hd
        self.ct = ct
        self._lock = threading.Lock()

    def __del__(self):  # capsule destructor: best-effort destroy
        try:
            lib.liberasurecode_instance_destroy(self.desc)
        except Exception:
            pass


def _handle(obj: Any, fn: str) -> PyECLibHandle:
    if not isinstance(obj, PyECLibHandle):
        raise_error(-EINVALIDPARAMS, fn)
    return obj


def _as_buffer(data: Any) -> tuple[Any, int]:
    """Argument parsing of "y#" (pyeclib_c.c:49): bytes-like objects only."""
    if isinstance(data, bytes):
        return data, len(data)
    if isinstance(data, (bytearray, memoryview)):
        b = bytes(data)
        return b, len(b)
    raise TypeError


def _frag_array(frags: Sequence[bytes]) -> ctypes.Array:
    return (ctypes.c_char_p * len(frags))(*frags)


# New bytes objects whose storage the library fills (the C-API pattern
# PyBytes_FromStringAndSize(NULL, n), then write, then share): pyeclib_c
# copies liberasurecode's fragment buffers into new bytes objects
# (Py_BuildValue("y#"), pyeclib_c.c:544-560); here the library writes the
# fragments (or the decoded object) into the bytes objects' own storage, and
# that whole-object copy is gone.  Only ever called with n >= 1, and the
# objects are not shared before they are filled.
_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.restype = ctypes.py_object
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_bytes_ptr = ctypes.pythonapi.PyBytes_AsString
_bytes_ptr.restype = ctypes.c_void_p
_bytes_ptr.argtypes = [ctypes.py_object]


# ---- the eleven module functions ----

def init(k: int, m: int, backend_id: int, hd: int = 0, use_inline_chksum: int = 0,
         use_algsig_chksum: int = 0, validate: int = 0, local_parity: int = 0) -> PyECLibHandle:
    """pyeclib_c_init (pyeclib_c.c:221-286)."""
    try:
        args = ECArgs()
        args.k, args.m, args.hd = int(k), int(m), int(hd)
        args.ct = CHKSUM_CRC32 if use_inline_chksum else CHKSUM_NONE
        args.priv_args1.reserved.x = int(local_parity)
        bid = int(backend_id)
    except (TypeError, ValueError):
        raise_error(-EINVALIDPARAMS, "pyeclib_c_init")
    desc = lib.liberasurecode_instance_create(bid, ctypes.byref(args))
    if desc <= 0:
        raise_error(desc, "pyeclib_c_init")
    return PyECLibHandle(desc, args.k, args.m, args.hd, args.ct)


def destroy(handle: PyECLibHandle) -> None:
    """pyeclib_c_destroy (pyeclib_c.c:289-344)."""
    if not isinstance(handle, PyECLibHandle):
        raise_error(-1, "pyeclib_c_destroy")
    ret = lib.liberasurecode_instance_destroy(handle.desc)
    if ret != 0:
        raise_error(ret, "pyeclib_c_destroy")


def encode(handle: PyECLibHandle, data: Any) -> list[bytes]:
    """pyeclib_c_encode (pyeclib_c.c:512-565)."""
    fn = "pyeclib_c_encode"
    h = _handle(handle, fn)
    try:
        buf, n = _as_buffer(data)
    except TypeError:
        raise_error(-EINVALIDPARAMS, fn)
    # liberasurecode_encode's fragments, written straight into the bytes
    # objects returned (ecamd_encode_into: same bytes, no copy out)
    fl = int(lib.ecamd_blocksize(h.desc, n)) + HEADER_SIZE
    out = [_new_bytes(None, fl) for _ in range(h.k + h.m)]
    ptrs = (ctypes.c_void_p * len(out))(*[_bytes_ptr(b) for b in out])
    ret = lib.ecamd_encode_into(h.desc, buf, n, ptrs, fl)
    if ret < 0:
        raise_error(ret, fn)
    return out


def decode(handle: PyECLibHandle, fragments: list[bytes], fragment_len: int,
           ranges: list[tuple[int, int]] | None = None,
           force_metadata_checks: bool = False) -> bytes | list[bytes]:
    """pyeclib_c_decode (pyeclib_c.c:770-922), ranges inclusive (:855-856)."""
    fn = "pyeclib_c_decode"
    h = _handle(handle, fn)
    if not isinstance(fragments, list):
        raise_error(-EINVALIDPARAMS, fn)
    if h.k > len(fragments):
        raise_error(-EINSUFFFRAGS, fn)
    spans: list[tuple[int, int]] = []
    for r in ranges or []:
        if not isinstance(r, tuple) or len(r) != 2:
            raise_error(-EINVALIDPARAMS, "pyeclib_c_decode invalid range")
        if not all(isinstance(v, int) for v in r):
            raise_error(-EINVALIDPARAMS, "pyeclib_c_decode invalid range")
        spans.append((r[0], r[1] - r[0] + 1))
    try:
        arr = _frag_array(fragments)
    except TypeError:
        raise_error(-EINVALIDPARAMS, fn)
    fl = int(fragment_len)
    n_out = _decoded_len(fragments, fl, h.k)
    if n_out is not None:
        # into a new bytes object of the decoded length (ecamd_decode_into)
        res = _new_bytes(None, n_out) if n_out else b""
        ret = lib.ecamd_decode_into(h.desc, arr, len(fragments), fl,
                                    1 if force_metadata_checks else 0,
                                    _bytes_ptr(res) if n_out else None, n_out)
        if ret < 0:
            raise_error(ret, fn)
        if not spans:
            return res
        pieces = []
        for off, length in spans:
            if off < 0 or length < 0 or off + length > n_out:
                raise_error(-EINVALIDPARAMS, "pyeclib_c_decode invalid range")
            pieces.append(res[off:off + length])
        return pieces
    out = ctypes.c_void_p()
    olen = ctypes.c_uint64(0)
    ret = lib.liberasurecode_decode(h.desc, arr, len(fragments), int(fragment_len),
                                    1 if force_metadata_checks else 0, ctypes.byref(out),
                                    ctypes.byref(olen))
    if ret < 0:
        raise_error(ret, fn)
    try:
        n = olen.value
        if not spans:
            return ctypes.string_at(out.value, n) if n else b""
        pieces = []
        for off, length in spans:
            if off < 0 or length < 0 or off + length > n:
                raise_error(-EINVALIDPARAMS, "pyeclib_c_decode invalid range")
            pieces.append(ctypes.string_at(out.value + off, length) if length else b"")
        return pieces
    finally:
        lib.liberasurecode_decode_cleanup(h.desc, out)


def _decoded_len(fragments: list[bytes], fragment_len: int, k: int) -> int | None:
    """orig_data_size from the first fragment's header when it is plausible
    (the payload sizes of k fragments hold it); None sends the call through
    liberasurecode_decode, whose checks produce the error a bad header deserves."""
    f = fragments[0]
    if not isinstance(f, bytes) or len(f) < HEADER_SIZE or fragment_len < HEADER_SIZE:
        return None
    n = int.from_bytes(f[12:20], "little")
    return n if n <= k * (fragment_len - HEADER_SIZE) else None


def reconstruct(handle: PyECLibHandle, fragments: list[bytes], fragment_len: int,
                destination_idx: int) -> bytes:
    """pyeclib_c_reconstruct (pyeclib_c.c:681-758)."""
    fn = "pyeclib_c_reconstruct"
    h = _handle(handle, fn)
    if not isinstance(fragments, list):
        raise_error(-EINVALIDPARAMS, fn)
    try:
        arr = _frag_array(fragments)
    except TypeError:
        raise_error(-EINVALIDPARAMS, fn)
    fl = int(fragment_len)
    out = ctypes.create_string_buffer(max(fl, 1))
    ret = lib.liberasurecode_reconstruct_fragment(h.desc, arr, len(fragments), fl,
                                                  int(destination_idx), out)
    if ret < 0:
        raise_error(ret, fn)
    return out.raw[:fl]


def get_required_fragments(handle: PyECLibHandle, reconstruct_list: list[int],
                           exclude_list: list[int]) -> list[int]:
    """pyeclib_c_get_required_fragments (pyeclib_c.c:577-664)."""
    fn = "pyeclib_c_get_required_fragments"
    h = _handle(handle, fn)
    miss = (ctypes.c_int * (len(reconstruct_list) + 1))(*reconstruct_list, -1)
    excl = (ctypes.c_int * (len(exclude_list) + 1))(*exclude_list, -1)
    need = (ctypes.c_int * (h.k + h.m + 1))()
    ret = lib.liberasurecode_fragments_needed(h.desc, miss, excl, need)
    if ret < 0:
        raise_error(ret, fn)
    out = []
    for v in need:
        if v < 0:
            break
        out.append(v)
    return out


def get_segment_info(handle: PyECLibHandle, data_len: int, segment_size: int) -> dict:
    """pyeclib_c_get_segment_info (pyeclib_c.c:387-502): C int arithmetic."""
    fn = "pyeclib_c_get_segment_info"
    h = _handle(handle, fn)
    try:
        data_len, segment_size = int(data_len), int(segment_size)
    except (TypeError, ValueError):
        raise_error(-EINVALIDPARAMS, fn)
    min_seg = lib.liberasurecode_get_minimum_encode_size(h.desc)
    if min_seg < 0:
        raise_error(-EINVALIDPARAMS, fn)
    num_segments = int(math.ceil(data_len / segment_size))
    if num_segments == 2 and data_len < segment_size + min_seg:
        num_segments -= 1
    if num_segments == 1:
        fragment_size = lib.liberasurecode_get_fragment_size(h.desc, data_len)
        if fragment_size < 0:
            raise_error(-EINVALIDPARAMS, fn)
        segment_size = data_len
        last_segment_size = segment_size
        last_fragment_size = fragment_size
    else:
        fragment_size = lib.liberasurecode_get_fragment_size(h.desc, segment_size)
        if fragment_size < 0:
            raise_error(-EINVALIDPARAMS, fn)
        last_segment_size = data_len - segment_size * (num_segments - 1)
        if last_segment_size < min_seg:
            num_segments -= 1
            last_segment_size += segment_size
        last_fragment_size = lib.liberasurecode_get_fragment_size(h.desc, last_segment_size)
    return {
        "segment_size": segment_size,
        "last_segment_size": last_segment_size,
        "fragment_size": fragment_size + HEADER_SIZE,
        "last_fragment_size": last_fragment_size + HEADER_SIZE,
        "num_segments": num_segments,
    }


_CHKSUM_NAMES = {CHKSUM_NONE: "none", CHKSUM_CRC32: "crc32", CHKSUM_MD5: "md5"}
_CHKSUM_LEN = {CHKSUM_CRC32: 4, CHKSUM_MD5: 16}
_BACKEND_NAMES = {
    0: "null", 1: "jerasure_rs_vand", 2: "jerasure_rs_cauchy", 3: "flat_xor_hd",
    4: "isa_l_rs_vand", 5: "shss", 6: "liberasurecode_rs_vand", 7: "isa_l_rs_cauchy",
    8: "libphazr", 9: "isa_l_rs_vand_inv", 10: "isa_l_rs_lrc",
}


def _metadata_dict(md: FragmentMetadata) -> dict:
    """fragment_metadata_to_dict (pyeclib_c.c:1029-1052)."""
    raw = bytes(md.chksum)
    return {
        "index": md.idx,
        "size": md.size,
        "orig_data_size": md.orig_data_size,
        "chksum_type": _CHKSUM_NAMES.get(md.chksum_type, "unknown"),
        "chksum": raw[: _CHKSUM_LEN.get(md.chksum_type, 0)].hex(),
        "chksum_mismatch": md.chksum_mismatch,
        "backend_id": _BACKEND_NAMES.get(md.backend_id, "unknown"),
        "backend_version": md.backend_version,
    }


def get_metadata(handle: PyECLibHandle, fragment: Any, formatted: int = 0) -> bytes | dict:
    """pyeclib_c_get_metadata (pyeclib_c.c:1062-1100)."""
    fn = "pyeclib_c_get_metadata"
    _handle(handle, fn)
    try:
        buf, n = _as_buffer(fragment)
    except TypeError:
        raise_error(-EINVALIDPARAMS, fn)
    if n < HEADER_SIZE:
        raise_error(-EBADHEADER, fn)
    # the C entry point trusts the header's payload size; do not let it read past the bytes
    size = int.from_bytes(buf[4:8], "little")
    if buf[20] == CHKSUM_CRC32 and HEADER_SIZE + size > n:
        raise_error(-EBADHEADER, fn)
    md = FragmentMetadata()
    ret = lib.liberasurecode_get_fragment_metadata(buf, ctypes.byref(md))
    if ret < 0:
        raise_error(ret, fn)
    if formatted:
        return _metadata_dict(md)
    return ctypes.string_at(ctypes.addressof(md), METADATA_SIZE)


def check_metadata(handle: PyECLibHandle, fragment_metadata_list: list[bytes]) -> dict:
    """pyeclib_c_check_metadata (pyeclib_c.c:1114-1197)."""
    fn = "pyeclib_c_check_metadata"
    h = _handle(handle, fn)
    n = h.k + h.m
    if not isinstance(fragment_metadata_list, list) or len(fragment_metadata_list) != n:
        raise_error(-EINVALIDPARAMS, fn)
    if any(not isinstance(b, bytes) or len(b) < METADATA_SIZE for b in fragment_metadata_list):
        raise_error(-EINVALIDPARAMS, fn)
    ret = lib.liberasurecode_verify_stripe_metadata(h.desc, _frag_array(fragment_metadata_list), n)
    if ret == 0:
        return {"status": 0}
    if ret == -EBADCHKSUM:
        bad = [int.from_bytes(b[0:4], "little") for b in fragment_metadata_list if b[53] == 1]
        return {"status": ret, "reason": "Bad checksum", "bad_fragments": bad}
    raise_error(ret, fn)


def check_backend_available(backend_id: int) -> bool:
    """pyeclib_c_check_backend_available (pyeclib_c.c:1199-1214)."""
    try:
        bid = int(backend_id)
    except (TypeError, ValueError):
        raise_error(-EINVALIDPARAMS, "pyeclib_c_check_backend_available")
    return bool(lib.liberasurecode_backend_available(bid))


def get_liberasurecode_version() -> int:
    """pyeclib_c_liberasurecode_version (pyeclib_c.c:1216-1219)."""
    return int(lib.liberasurecode_get_version())
