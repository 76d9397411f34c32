"""TEST INFRASTRUCTURE ONLY -- ctypes view of the C oracle (rs_vand_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The
product (``pyeclib_amd``) never imports it.

Every function mirrors one liberasurecode 1.8.0 entry point that pyeclib's C
binding calls (src/pyeclib_c/pyeclib_c.c:537 encode, :878 decode,
:735 reconstruct, :441 fragment size); see the header of rs_vand_oracle.c for
the upstream files each piece restates and for the parity status.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle_rs_vand.so")
_SO8 = os.path.join(_HERE, "build", "liboracle_isal.so")

HDR = 80
LIBEC_VERSION = 0x010800
CHKSUM_NONE = 1
CHKSUM_CRC32 = 2

_lib = None
_lib8 = None

# GF(2^8) ISA-L codes (isal_oracle.c): backend ids of the two matrix kinds
ISAL_VAND = 4
ISAL_CAUCHY = 7


def build() -> str:
    """Compile the oracle with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u8p = ctypes.c_void_p
        L.orc_blocksize.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.orc_blocksize.restype = ctypes.c_uint64
        L.orc_fragment_len.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.orc_fragment_len.restype = ctypes.c_uint64
        L.orc_generator.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.orc_gf_mul.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_gf_div.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_invert.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.orc_crc32.argtypes = [u8p, ctypes.c_uint64]
        L.orc_crc32.restype = ctypes.c_uint32
        L.orc_crc32_legacy.argtypes = [u8p, ctypes.c_uint64]
        L.orc_crc32_legacy.restype = ctypes.c_uint32
        L.orc_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                 u8p, ctypes.c_uint64, u8p]
        L.orc_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                 ctypes.c_int, ctypes.c_uint64, u8p, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                      ctypes.c_uint64, ctypes.c_int, u8p]
        _lib = L
    return _lib


def blocksize(k: int, length: int) -> int:
    return lib().orc_blocksize(k, length)


def fragment_len(k: int, length: int) -> int:
    return lib().orc_fragment_len(k, length)


def generator(k: int, m: int) -> list[list[int]]:
    buf = (ctypes.c_int * ((k + m) * k))()
    assert lib().orc_generator(k, m, buf) == 0
    return [list(buf[r * k:(r + 1) * k]) for r in range(k + m)]


def gf_mul(a: int, b: int) -> int:
    return lib().orc_gf_mul(a, b)


def gf_div(a: int, b: int) -> int:
    return lib().orc_gf_div(a, b)


def invert(mat: list[list[int]]) -> list[list[int]]:
    n = len(mat)
    a = (ctypes.c_int * (n * n))(*[v for row in mat for v in row])
    o = (ctypes.c_int * (n * n))()
    if lib().orc_invert(a, o, n) != 0:
        raise ValueError("singular")
    return [list(o[r * n:(r + 1) * n]) for r in range(n)]


def crc32(data: bytes) -> int:
    return lib().orc_crc32(data, len(data))


def crc32_legacy(data: bytes) -> int:
    return lib().orc_crc32_legacy(data, len(data))


def legacy_headers(frag: bytes) -> bytes:
    """An inline_crc32 fragment as liberasurecode writes it with
    LIBERASURECODE_WRITE_LEGACY_CRC set: payload checksum and metadata
    checksum from liberasurecode_crc32_alt (erasurecode_helpers.c
    set_checksum / set_metadata_chksum)."""
    size = int.from_bytes(frag[4:8], "little")
    h = bytearray(frag[:HDR])
    h[21:25] = crc32_legacy(frag[HDR:HDR + size]).to_bytes(4, "little")
    h[67:71] = crc32_legacy(bytes(h[:59])).to_bytes(4, "little")
    return bytes(h) + frag[HDR:]


def encode(k: int, m: int, data: bytes, ct: int = CHKSUM_NONE,
           libec_version: int = LIBEC_VERSION) -> list[bytes]:
    """liberasurecode_encode restated: k data + m parity fragments (with headers)."""
    fl = fragment_len(k, len(data))
    out = ctypes.create_string_buffer(fl * (k + m))
    rc = lib().orc_encode(k, m, ct, libec_version, data, len(data), out)
    if rc != 0:
        raise RuntimeError(f"orc_encode rc={rc}")
    raw = out.raw
    return [raw[i * fl:(i + 1) * fl] for i in range(k + m)]


def decode(k: int, m: int, frags: list[bytes]) -> bytes:
    if not frags:
        raise ValueError("no fragments")
    fl = len(frags[0])
    arr = (ctypes.c_char_p * len(frags))(*frags)
    orig = int.from_bytes(frags[0][12:20], "little") if fl >= HDR else 0
    out = ctypes.create_string_buffer(max(orig, 1))
    olen = ctypes.c_uint64(0)
    rc = lib().orc_decode(k, m, arr, len(frags), fl, out, ctypes.byref(olen))
    if rc != 0:
        raise RuntimeError(f"orc_decode rc={rc}")
    return out.raw[:olen.value]


def reconstruct(k: int, m: int, frags: list[bytes], dest: int, ct: int = CHKSUM_NONE,
                libec_version: int = LIBEC_VERSION) -> bytes:
    fl = len(frags[0])
    arr = (ctypes.c_char_p * len(frags))(*frags)
    out = ctypes.create_string_buffer(fl)
    rc = lib().orc_reconstruct(k, m, ct, libec_version, arr, len(frags), fl, dest, out)
    if rc != 0:
        raise RuntimeError(f"orc_reconstruct rc={rc}")
    return out.raw


def encode_payloads_into(k: int, m: int, data_ptr: int, length: int, out_ptr: int,
                         ct: int = CHKSUM_NONE) -> None:
    """Raw-pointer encode used by bench.py's cpu_baseline leg (no Python copies)."""
    rc = lib().orc_encode(k, m, ct, LIBEC_VERSION, ctypes.c_void_p(data_ptr), length,
                          ctypes.c_void_p(out_ptr))
    if rc != 0:
        raise RuntimeError(f"orc_encode rc={rc}")


# ---------------- GF(2^8) ISA-L codes (isal_oracle.c) ----------------

def lib8() -> ctypes.CDLL:
    global _lib8
    if _lib8 is None:
        if not os.path.exists(_SO8):
            build()
        L = ctypes.CDLL(_SO8)
        u8p = ctypes.c_void_p
        L.o8_blocksize.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.o8_blocksize.restype = ctypes.c_uint64
        L.o8_generator.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
        L.o8_gf_mul.argtypes = [ctypes.c_int, ctypes.c_int]
        L.o8_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_uint32, u8p, ctypes.c_uint64, u8p]
        L.o8_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, u8p,
                                ctypes.POINTER(ctypes.c_uint64)]
        L.o8_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint32, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.c_int, ctypes.c_uint64, ctypes.c_int, u8p]
        _lib8 = L
    return _lib8


def isal_blocksize(k: int, length: int) -> int:
    return lib8().o8_blocksize(k, length)


def isal_generator(kind: int, k: int, m: int) -> list[list[int]]:
    buf = ctypes.create_string_buffer((k + m) * k)
    assert lib8().o8_generator(kind, k, m, buf) == 0
    raw = buf.raw
    return [list(raw[r * k:(r + 1) * k]) for r in range(k + m)]


def isal_gf_mul(a: int, b: int) -> int:
    return lib8().o8_gf_mul(a, b)


def isal_encode(kind: int, k: int, m: int, data: bytes, ct: int = CHKSUM_NONE,
                libec_version: int = LIBEC_VERSION) -> list[bytes]:
    fl = isal_blocksize(k, len(data)) + HDR
    out = ctypes.create_string_buffer(fl * (k + m))
    rc = lib8().o8_encode(kind, k, m, ct, libec_version, data, len(data), out)
    if rc != 0:
        raise RuntimeError(f"o8_encode rc={rc}")
    raw = out.raw
    return [raw[i * fl:(i + 1) * fl] for i in range(k + m)]


def isal_decode(kind: int, k: int, m: int, frags: list[bytes]) -> bytes:
    arr = (ctypes.c_char_p * len(frags))(*frags)
    orig = int.from_bytes(frags[0][12:20], "little")
    out = ctypes.create_string_buffer(max(orig, 1))
    olen = ctypes.c_uint64(0)
    rc = lib8().o8_decode(kind, k, m, arr, len(frags), out, ctypes.byref(olen))
    if rc != 0:
        raise RuntimeError(f"o8_decode rc={rc}")
    return out.raw[:olen.value]


def isal_reconstruct(kind: int, k: int, m: int, frags: list[bytes], dest: int,
                     ct: int = CHKSUM_NONE, libec_version: int = LIBEC_VERSION) -> bytes:
    fl = len(frags[0])
    arr = (ctypes.c_char_p * len(frags))(*frags)
    out = ctypes.create_string_buffer(fl)
    rc = lib8().o8_reconstruct(kind, k, m, ct, libec_version, arr, len(frags), fl, dest, out)
    if rc != 0:
        raise RuntimeError(f"o8_reconstruct rc={rc}")
    return out.raw
