"""The upgrade path of SURVEY.md section 8(c): when a system liberasurecode is
installed (`ctypes.util.find_library("erasurecode")`), its own
`liberasurecode_encode` is the true reference for this path -- parity pinned
against real liberasurecode instead of the CPU restatement.  This image has
none (nor ISA-L), so the probe reports null and the tests that use it skip;
a box or a user installation that has it runs them unchanged.

Test and measurement infrastructure only: the product path never loads it.
The ctypes signatures are the ones pyeclib_c.c binds (pyeclib_c.c:259, :537,
:562, :322), with the ec_args layout of include/erasurecode_amd.h."""
import ctypes
import ctypes.util

from . import _native

BACKEND_IDS = {"liberasurecode_rs_vand": 6, "isa_l_rs_vand": 4, "isa_l_rs_cauchy": 7}
HEADER_BYTES = 80


def probe():
    """Path of the system liberasurecode, or None."""
    return ctypes.util.find_library("erasurecode")


class SystemLibrary:
    def __init__(self, path=None):
        path = path or probe()
        if path is None:
            raise OSError("no system liberasurecode (ctypes.util.find_library('erasurecode'))")
        self.path = path
        lib = self.lib = ctypes.CDLL(path)
        P = ctypes.POINTER
        lib.liberasurecode_instance_create.restype = ctypes.c_int
        lib.liberasurecode_instance_create.argtypes = [ctypes.c_int, P(_native.ECArgs)]
        lib.liberasurecode_instance_destroy.restype = ctypes.c_int
        lib.liberasurecode_instance_destroy.argtypes = [ctypes.c_int]
        lib.liberasurecode_encode.restype = ctypes.c_int
        lib.liberasurecode_encode.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_uint64,
                                              P(P(ctypes.c_char_p)), P(P(ctypes.c_char_p)),
                                              P(ctypes.c_uint64)]
        lib.liberasurecode_encode_cleanup.restype = ctypes.c_int
        lib.liberasurecode_encode_cleanup.argtypes = [ctypes.c_int, P(ctypes.c_char_p),
                                                      P(ctypes.c_char_p)]

    def encode(self, k, m, data, ec_type="liberasurecode_rs_vand", crc32=False):
        """liberasurecode_encode's k + m fragments (80-byte header + payload)."""
        args = _native.ECArgs()
        args.k, args.m, args.w, args.hd = k, m, 16 if ec_type == "liberasurecode_rs_vand" else 8, m
        args.ct = 2 if crc32 else 1
        desc = self.lib.liberasurecode_instance_create(BACKEND_IDS[ec_type], ctypes.byref(args))
        if desc <= 0:
            raise OSError(f"liberasurecode_instance_create: {desc}")
        try:
            dp, pp = ctypes.POINTER(ctypes.c_char_p)(), ctypes.POINTER(ctypes.c_char_p)()
            flen = ctypes.c_uint64()
            rc = self.lib.liberasurecode_encode(desc, data, len(data), ctypes.byref(dp),
                                                ctypes.byref(pp), ctypes.byref(flen))
            if rc != 0:
                raise OSError(f"liberasurecode_encode: {rc}")
            n = flen.value
            frags = [ctypes.string_at(dp[i], n) for i in range(k)]
            frags += [ctypes.string_at(pp[i], n) for i in range(m)]
            self.lib.liberasurecode_encode_cleanup(desc, dp, pp)
            return frags
        finally:
            self.lib.liberasurecode_instance_destroy(desc)


def comparable(frag):
    """A fragment without the fields that name the library's version: the
    header's libec_version (offset 63) and the metadata checksum over it
    (offset 67) -- payload, sizes, index, checksum type and payload CRC stay."""
    return frag[:63] + frag[71:]
