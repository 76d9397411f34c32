"""Host-side checks that need no GPU: the C-ABI library loads and exports
every symbol include/erasurecode_amd.h declares, the ECDriver argument
handling and plugin seam (reference src/pyeclib/ec_iface.py:81-214), error
mapping (pyeclib_c.c:125-183) and the byte-range recipe (ec_iface.py:389-464).
No GF compute is called here."""
import ctypes
import os
import re
import warnings

import pytest

import pyeclib_amd
from pyeclib_amd import ECDriver, _native
from pyeclib_amd import exceptions as X
from pyeclib_amd.enums import PyECLib_EC_Types, PyECLib_FRAGHDRCHKSUM_Types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "erasurecode_amd.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b((?:liberasurecode|ecamd)_\w+)\s*\(", text, re.M)))


def test_header_parses():
    names = declared_functions()
    assert "liberasurecode_encode" in names and "ecamd_encode_batch" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native._LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(_native.EXPORTS)


def test_struct_layouts():
    assert ctypes.sizeof(_native.FragmentMetadata) == 59
    assert _native.FragmentMetadata.chksum_mismatch.offset == 53
    assert _native.FragmentMetadata.backend_version.offset == 55
    assert ctypes.sizeof(_native.ECArgs) == 64


def test_version_and_enums():
    assert _native.get_liberasurecode_version() == 0x010800
    assert pyeclib_amd.api.LIBERASURECODE_VERSION == "1.8.0"
    assert PyECLib_EC_Types.liberasurecode_rs_vand.value == 6
    assert PyECLib_EC_Types.amd_rs_vand.value == 11
    assert PyECLib_FRAGHDRCHKSUM_Types.inline_crc32.value == 2
    assert "amd_rs_vand" in pyeclib_amd.ALL_EC_TYPES


def _gpu_present():
    return bool(_native.lib.liberasurecode_backend_available(6))


@pytest.mark.skipif(_gpu_present(), reason="checks the no-GPU behaviour")
def test_no_gpu_means_backend_unavailable():
    assert pyeclib_amd.VALID_EC_TYPES == []
    assert not _native.check_backend_available(6)
    with pytest.raises(X.ECBackendInstanceNotAvailable) as ctx:
        ECDriver(k=4, m=2, ec_type="amd_rs_vand")
    assert str(ctx.value) == ("pyeclib_c_init ERROR: Backend instance not found. Please "
                              "inspect syslog for liberasurecode error report.")


def test_instance_create_argument_errors():
    args = _native.ECArgs()
    args.k, args.m, args.hd, args.ct = 30, 3, 3, 1
    assert _native.lib.liberasurecode_instance_create(6, ctypes.byref(args)) == -206
    args.k, args.m = 4, 2
    assert _native.lib.liberasurecode_instance_create(99, ctypes.byref(args)) == -200
    assert _native.lib.liberasurecode_instance_create(1, ctypes.byref(args)) == -204
    assert _native.lib.liberasurecode_instance_create(6, None) == -206
    assert _native.lib.liberasurecode_instance_destroy(12345) == -204


def test_missing_required_args():  # test_pyeclib_api.py:123-150
    with pytest.raises(X.ECDriverError) as ctx:
        ECDriver(k=1, m=1)
    assert str(ctx.value) == ("Invalid Argument: either ec_type or library_import_str "
                              "must be provided")
    with pytest.raises(TypeError, match="missing 1 required keyword-only argument: 'k'"):
        ECDriver(ec_type="amd_rs_vand", m=1)
    with pytest.raises(TypeError, match="missing 1 required keyword-only argument: 'm'"):
        ECDriver(ec_type="amd_rs_vand", k=1)


def test_invalid_km_and_types():  # :152-166, :241-243
    with pytest.raises(X.ECDriverError, match=r"Invalid number of data fragments \(k\)"):
        ECDriver(ec_type="amd_rs_vand", k=-100, m=1)
    with pytest.raises(X.ECDriverError, match=r"Invalid number of parity fragments \(m\)"):
        ECDriver(ec_type="amd_rs_vand", k=1, m=-100)
    with pytest.raises(X.ECBackendNotSupported):
        ECDriver(k=10, m=5, ec_type="invalid_algo")
    with pytest.raises(X.ECDriverError, match="crc64 is not a valid checksum type"):
        ECDriver(k=10, m=5, ec_type="amd_rs_vand", chksum_type="crc64")


class DummyDriver:
    """A plugin with every required method (the seam ECDriver loads through
    library_import_str, ec_iface.py:179-214)."""

    def __init__(self, k, m, hd, ec_type, chksum_type, validate, local_parity):
        self.args = (k, m, hd, ec_type, chksum_type, validate, local_parity)

    def encode(self, data):
        return [data]

    def decode(self, frags, ranges=None, force=False):
        return b"".join(frags)

    def reconstruct(self, frags, idx):
        return frags

    def fragments_needed(self, r, e):
        return [r, e]

    def min_parity_fragments_needed(self):
        return 1

    def get_metadata(self, f, formatted=0):
        return b""

    def verify_stripe_metadata(self, md):
        return {"status": 0}

    def get_segment_info(self, data_len, segment_size):
        return {"segment_size": segment_size}

    def close(self):
        pass


class HalfDriver:
    def __init__(self, **kw):
        pass

    def encode(self, data):
        return [data]


def test_plugin_seam_and_repr():
    d = ECDriver(k=8, m=2, library_import_str="tests.test_host.DummyDriver")
    assert d.ec_lib_reference.args == (8, 2, 2, None, PyECLib_FRAGHDRCHKSUM_Types.none, 0, 0)
    assert repr(d) == "ECDriver(ec_type='None', k=8, m=2)"
    assert d.encode(b"x") == [b"x"]
    assert d.fragments_needed([1]) == [[1], []]
    d2 = ECDriver(k=4, m=2, ec_type="flat_xor_hd_4", library_import_str="tests.test_host.DummyDriver")
    assert d2.hd == 4 and repr(d2) == "ECDriver(ec_type='flat_xor_hd_4', k=4, m=2)"
    with pytest.raises(X.ECDriverError) as ctx:
        ECDriver(k=4, m=2, library_import_str="tests.test_host.HalfDriver")
    assert str(ctx.value).startswith("The following required methods are not implemented in "
                                     "tests.test_host.HalfDriver: decode reconstruct")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        ECDriver(k=4, m=2, ec_type="jerasure_rs_vand", library_import_str="tests.test_host.DummyDriver")
    assert any(issubclass(x.category, FutureWarning) for x in w)


def test_segment_byterange_recipe():  # test_pyeclib_api.py:650-699
    d = ECDriver(k=8, m=2, library_import_str="tests.test_host.DummyDriver")
    seg = 3 * 1024
    ranges = [(0, 1), (1, 12), (10, 1000), (0, seg - 1), (1, seg + 1), (seg - 1, 2 * seg)]
    got = d.get_segment_info_byterange(ranges, 1024 * 1024, seg)
    assert got == {
        (0, 1): {0: (0, 1)}, (1, 12): {0: (1, 12)}, (10, 1000): {0: (10, 1000)},
        (0, seg - 1): {0: (0, seg - 1)}, (1, seg + 1): {0: (1, seg - 1), 1: (0, 1)},
        (seg - 1, 2 * seg): {0: (seg - 1, seg - 1), 1: (0, seg - 1), 2: (0, 0)},
    }


def test_error_mapping():
    cases = {-204: "ECBackendInstanceNotAvailable", -208: "ECInsufficientFragments",
             -200: "ECBackendNotSupported", -206: "ECInvalidParameter",
             -205: "ECBadFragmentChecksum", -207: "ECInvalidFragmentMetadata",
             -12: "ECOutOfMemory", -1: "ECDriverError", -202: "ECDriverError"}
    for code, name in cases.items():
        with pytest.raises(getattr(X, name)) as ctx:
            _native.raise_error(code, "pyeclib_c_encode")
        assert type(ctx.value).__name__ == name
        assert str(ctx.value).startswith("pyeclib_c_encode ERROR: ")
        assert str(ctx.value).endswith(". Please inspect syslog for liberasurecode error report.")
    e = X.ECDriverErrorWithPosition("Invalid fragment payload in ECPyECLibDriver.decode", 2)
    assert str(e) == "Invalid fragment payload in ECPyECLibDriver.decode (position 2)"


def test_positive_int_value():
    from pyeclib_amd.utils import positive_int_value
    assert positive_int_value("7") == 7
    for bad in (None, 0, -1, "x"):
        with pytest.raises(ValueError):
            positive_int_value(bad)


def test_batch_layout_helpers():
    from pyeclib_amd import batch
    assert batch.blocksize(10, 4 * 1024 * 1024) == 419432
    assert batch.blocksize(4, 1024 * 1024) == 262144
    assert batch.blocksize(12, 16 * 1024 * 1024) == 1398102
    fs = batch.frag_stride(419432)
    assert fs % 128 == 0 and fs >= 80 + 419440
    assert (batch.PAYLOAD_SKEW + 80) % 128 == 0


def test_layout_guard_32bit_offsets():
    """The kernels use 32-bit buffer offsets (object slices below 2^31,
    stripes below 2^32): layouts past them are refused with -EINVALIDPARAMS
    instead of wrapping (run_encode / run_decode apply the same
    check).  Needs no GPU."""
    from pyeclib_amd import batch
    f = _native.lib.ecamd_layout_supported
    bad = -_native.EINVALIDPARAMS
    L = 4 * 1024 * 1024
    assert f(10, 4, 16, L, batch.frag_stride(419432), 256) == 0
    # a 1.9 GiB object still fits; 2 GiB does not (decode's output window)
    big = 1900 * 2**20
    assert f(10, 4, 16, big, batch.frag_stride(batch.blocksize(10, big)), 1) == 0
    assert f(10, 4, 16, 2**31, batch.frag_stride(batch.blocksize(10, 2**31)), 1) == bad
    # a stripe span (k+m)*frag_stride past 4 GiB
    assert f(4, 28, 16, 2**30, batch.frag_stride(batch.blocksize(4, 2**30)), 1) == bad
    # a batch whose 4 KiB work items overflow 31 bits
    assert f(10, 4, 16, L, batch.frag_stride(419432), 2**25) == bad
    # bad codes
    assert f(0, 4, 16, L, 1 << 20, 1) == bad
    assert f(10, 4, 12, L, 1 << 20, 1) == bad


def test_batch_rejects_strided_views():
    """A fragment group must be packed at k * frag_stride per object: the C
    API takes only the fragment stride, so a view like stripes[:, :k] is
    refused rather than read as the wrong bytes."""
    import torch
    from pyeclib_amd import batch
    k, m, fs = 4, 2, 256
    stripes = torch.zeros((3, k + m, fs), dtype=torch.uint8)
    chk = batch.BatchCodec._check_rows
    chk("f", stripes[:, :k])                      # device path: any object stride
    chk("f", stripes[:, :k].contiguous(), k)      # host path: packed group
    with pytest.raises(X.ECInvalidParameter):
        chk("f", stripes[:, :k], k)               # host path: strided group
    with pytest.raises(X.ECInvalidParameter):
        chk("f", stripes[:, :, ::2])              # bytes not contiguous
    with pytest.raises(X.ECInvalidParameter):
        chk("f", stripes[:, :k + 1].contiguous(), k)  # wrong group size
    chk("f", stripes[:1, :k], k)                  # one object: stride(0) unused
