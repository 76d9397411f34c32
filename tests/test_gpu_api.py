"""The reference's ECDriver test suite, re-expressed against the MI355X backend.

Each test names the reference test it follows (test/test_pyeclib_api.py and
test/test_pyeclib_c.py in /root/reference) and keeps its invariant: round
trips, reconstruct == original fragment byte for byte, metadata fields,
checksum verification, segment sizing, error classes and messages.  On top of
the reference's self-consistency checks, fragments are compared with the CPU
oracle where the reference had nothing to compare against.
"""
import itertools
import os
import queue
import random
import string
import threading

import pytest

from pyeclib_amd import ECDriver
from pyeclib_amd import _native
from pyeclib_amd.exceptions import (ECBackendInstanceNotAvailable, ECDriverError,
                                    ECInsufficientFragments, ECInvalidFragmentMetadata,
                                    ECInvalidParameter)

pytestmark = pytest.mark.gpu

EC_TYPES = ["liberasurecode_rs_vand", "amd_rs_vand"]
# reference get_pyeclib_testspec() for liberasurecode_rs_vand (test_pyeclib_api.py:259-272)
SPECS = [(12, 2), (11, 2), (10, 2), (8, 4)]


def drivers(csum="none", ec_type="amd_rs_vand"):
    return [ECDriver(k=k, m=m, ec_type=ec_type, chksum_type=csum) for k, m in SPECS]


def ascii_bytes(n, seed):
    rng = random.Random(seed)
    return "".join(rng.choice(string.ascii_letters) for _ in range(n)).encode("ascii")


def test_valid_ec_types_on_gpu():
    from pyeclib_amd import VALID_EC_TYPES
    # ALL_EC_TYPES order (ec_iface.py:468-480, amd_rs_vand appended)
    assert VALID_EC_TYPES == ["isa_l_rs_vand", "liberasurecode_rs_vand", "isa_l_rs_cauchy",
                              "amd_rs_vand"]


def test_use_after_close():  # test_pyeclib_api.py:386-409
    for drv in drivers():
        frags = drv.encode(b"testdata")
        assert drv.reconstruct(frags[1:], [0])[0] == frags[0]
        drv.close()
        for call in (lambda: drv.encode(b"testdata"), lambda: drv.decode(frags),
                     lambda: drv.reconstruct(frags[1:], [0])):
            with pytest.raises(ECBackendInstanceNotAvailable) as ctx:
                call()
            assert str(ctx.value) == "erasure coding handle is closed"


@pytest.mark.parametrize("ec_type", EC_TYPES)
def test_small_encode(oracle, ec_type):  # :411-420
    for drv in drivers(ec_type=ec_type):
        for s in [b"a", b"hello", b"hellohyhi", b"yo"]:
            frags = drv.encode(s)
            assert frags == oracle.encode(drv.k, drv.m, s)
            assert drv.decode(frags) == s


def test_empty_encode_roundtrip(oracle):
    drv = ECDriver(k=4, m=2, ec_type="amd_rs_vand")
    frags = drv.encode(b"")
    assert frags == oracle.encode(4, 2, b"")
    assert all(len(f) == 80 for f in frags)
    assert drv.decode(frags[2:]) == b""


def test_encode_invalid_params():  # :422-429
    for drv in drivers():
        for bad in ["\U0001f0a1", 3, object(), None, {}, []]:
            with pytest.raises(ECInvalidParameter):
                drv.encode(bad)


def test_decode_reconstruct_with_fragment_iterator():  # :462-505
    for drv in drivers():
        for s in [b"a", b"hello", b"hellohyhi", b"yo"]:
            frags = drv.encode(s)
            lost = random.sample(range(drv.k + drv.m), 2)
            avail = [f for i, f in enumerate(frags) if i not in lost]
            it = iter(avail)
            assert drv.decode(it) == s
            with pytest.raises(ECDriverError) as ctx:
                drv.decode(it)
            assert str(ctx.value) == "No fragments payload in ECPyECLibDriver.decode"
            it = iter(avail)
            rebuilt = drv.reconstruct(it, lost)
            assert len(rebuilt) == 2
            for i, frag in zip(sorted(lost), rebuilt):
                assert frag == frags[i]
            with pytest.raises(ECDriverError) as ctx:
                drv.reconstruct(it, lost)
            assert str(ctx.value) == "No fragments payload in ECPyECLibDriver.reconstruct"


@pytest.mark.parametrize("k,m", [(12, 2), (8, 4)])
def test_get_metadata_formatted(k, m):  # :507-572
    data = ascii_bytes(3 * 1024 * 1024, k)
    drv = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand", chksum_type="inline_crc32")
    for i, frag in enumerate(drv.encode(data)):
        md = drv.get_metadata(frag, 1)
        assert md["index"] == i
        assert md["chksum_mismatch"] == 0
        assert md["backend_id"] == "liberasurecode_rs_vand"
        assert md["orig_data_size"] == 3145728
        assert md["chksum_type"] == "crc32"
        assert md["size"] == len(frag) - 80
        assert md["backend_version"] == 0x10000
        assert len(md["chksum"]) == 8
        raw = drv.get_metadata(frag)
        assert raw == frag[:59]


def test_verify_fragment_inline_chksum_fail():  # :574-622
    data = ascii_bytes(3 * 1024 * 1024, 5)
    for drv in drivers("inline_crc32"):
        frags = drv.encode(data)
        first = random.randint(0, len(frags))
        bad = sorted((first + i) % len(frags) for i in range(3))
        mds = []
        for i, frag in enumerate(frags):
            if i in bad:
                frag = frag[:100] + bytes([(frag[100] + 1) % 128]) + frag[101:]
            mds.append(drv.get_metadata(frag))
        assert drv.verify_stripe_metadata(mds) == {
            "status": -205, "reason": "Bad checksum", "bad_fragments": bad}


def test_verify_fragment_inline_chksum_succeed():  # :624-648
    data = ascii_bytes(3 * 1024 * 1024, 6)
    for drv in drivers("inline_crc32"):
        mds = [drv.get_metadata(f) for f in drv.encode(data)]
        assert drv.verify_stripe_metadata(mds) == {"status": 0}


def test_get_segment_info():  # :701-774
    segs = {seg: ascii_bytes(2 * seg, seg) for seg in [3 * 1024, 1024 * 1024]}
    for drv in drivers():
        for file_size in [1024 * 1024, 2 * 1024 * 1024, 10 * 1024 * 1024, 10 * 1024 * 1024 + 7]:
            for seg, payload in segs.items():
                info = drv.get_segment_info(file_size, seg)
                n, ss = info["num_segments"], info["segment_size"]
                assert (n - 1) * ss + info["last_segment_size"] == file_size
                body = payload[:ss] if ss <= len(payload) else os.urandom(ss)
                assert info["fragment_size"] == len(drv.encode(body)[0])
                last = info["last_segment_size"]
                if last > 0:
                    tail = payload[:last] if last <= len(payload) else os.urandom(last)
                    assert info["last_fragment_size"] == len(drv.encode(tail)[0])


def test_greedy_decode_reconstruct_combination(oracle):  # :776-825
    data = os.urandom(1024)
    for drv in drivers():
        frags = drv.encode(data)
        assert frags == oracle.encode(drv.k, drv.m, data)
        n = drv.k + drv.m
        for keep in itertools.combinations(range(n), n - drv.m):
            check = [frags[i] for i in keep]
            assert drv.decode(check) == data, keep
            for hole in (i for i in range(n) if i not in keep):
                assert drv.reconstruct(check, [hole])[0] == frags[hole], (keep, hole)


def test_rs():  # :827-903
    data = ascii_bytes(100 * 1000, 11)
    for drv in drivers():
        orig = drv.encode(data)
        for _ in range(20):
            lost = sorted(random.sample(range(drv.k + drv.m), 2), reverse=True)
            frags = orig[:]
            for i in lost:
                frags.pop(i)
            assert drv.decode(frags) == data
            rebuilt = drv.reconstruct(frags, lost)
            for i, frag in zip(sorted(lost), rebuilt):
                assert frag == orig[i]
            first = random.randint(0, len(frags))
            count = min(len(frags), drv.m + 1)
            for j in [(first + i) % len(frags) for i in range(count)]:
                frags[j] = b"0" * len(frags[j])
            with pytest.raises(ECInvalidFragmentMetadata):
                drv.decode(frags, force_metadata_checks=True)


def test_insufficient_frags_error():  # :915-931
    data = ascii_bytes(100 * 1000, 12)
    drv = ECDriver(k=10, m=5, ec_type="liberasurecode_rs_vand", chksum_type="inline_crc32")
    frags = drv.encode(data)
    with pytest.raises(ECInsufficientFragments):
        drv.reconstruct([frags[0]], [1, 2, 3, 4, 5, 6])
    with pytest.raises(ECInsufficientFragments):
        drv.decode(frags[:9])


def test_min_parity_and_repr():  # :932-954
    drv = ECDriver(k=10, m=5, ec_type="liberasurecode_rs_vand")
    assert drv.min_parity_fragments_needed() == 1
    for d in drivers():
        assert repr(d) == "ECDriver(ec_type='amd_rs_vand', k=%d, m=%d)" % (d.k, d.m)


def test_create_in_threads():  # :192-218
    for ec_type in EC_TYPES:
        q = queue.Queue()
        threads = [threading.Thread(target=lambda: q.put(ECDriver(ec_type=ec_type, k=10, m=5)))
                   for _ in range(5)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        assert q.qsize() == 5


def test_threaded_encode_decode(oracle):
    """Concurrent calls on one instance and on separate instances (the GIL is
    released inside ctypes calls, unlike the reference's C extension)."""
    shared = ECDriver(k=10, m=4, ec_type="amd_rs_vand")
    errors = []

    def work(seed, drv):
        try:
            data = os.urandom(100000 + seed)
            frags = drv.encode(data)
            assert frags == oracle.encode(10, 4, data)
            assert drv.decode(frags[3:]) == data
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=work, args=(i, shared if i % 2 else
                                              ECDriver(k=10, m=4, ec_type="amd_rs_vand")))
          for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors


def test_destroy_semantics():  # test_pyeclib_c.py:544-593
    data = ascii_bytes(101 * 1000, 13)
    h = _native.init(4, 2, 6, 2)
    _native.encode(h, data)
    _native.destroy(h)
    with pytest.raises(ECBackendInstanceNotAvailable) as ctx:
        _native.destroy(h)
    assert str(ctx.value) == ("pyeclib_c_destroy ERROR: Backend instance not found. Please "
                              "inspect syslog for liberasurecode error report.")
    with pytest.raises(ECBackendInstanceNotAvailable) as ctx:
        _native.encode(h, data)
    assert str(ctx.value) == ("pyeclib_c_encode ERROR: Backend instance not found. Please "
                              "inspect syslog for liberasurecode error report.")
    h1, h2 = _native.init(4, 2, 6, 2), _native.init(4, 2, 6, 2)
    _native.encode(h1, data)
    _native.destroy(h1)
    _native.encode(h2, data)
    _native.destroy(h2)


def test_required_fragments():  # test_pyeclib_c.py:430-455 (made non-vacuous)
    for k, m in [(12, 2), (12, 3), (12, 4)]:
        h = _native.init(k, m, 6, m)
        for _ in range(20):
            missing = random.sample(range(k + m), random.randint(0, m))
            expected = [i for i in range(k + m) if i not in missing][:k]
            assert _native.get_required_fragments(h, missing, []) == expected
        with pytest.raises(ECDriverError):
            _native.get_required_fragments(h, list(range(m + 1)), [])


def test_range_decode():  # test_pyeclib_c.py:218-260
    drv = ECDriver(k=12, m=3, ec_type="amd_rs_vand")
    data = ascii_bytes(303 * 1000, 14)
    frags = drv.encode(data)
    ranges = [(0, 0), (5, 1000), (1000, 303 * 1000 - 1), (77777, 77777 + 4095)]
    got = drv.decode(frags[2:], ranges=ranges)
    assert got == [data[a:b + 1] for a, b in ranges]
    with pytest.raises(ECInvalidParameter):
        drv.decode(frags, ranges=[(0, len(data))])


def test_fragments_interchangeable_between_ec_types():
    a = ECDriver(k=10, m=4, ec_type="amd_rs_vand")
    b = ECDriver(k=10, m=4, ec_type="liberasurecode_rs_vand")
    data = os.urandom(50000)
    fa = a.encode(data)
    assert fa == b.encode(data)
    assert b.decode(fa[4:]) == data


@pytest.mark.parametrize("pinned_max", ["0", str(1 << 40), ""])
@pytest.mark.parametrize("n", [1, 4093, 65536 + 3, 1 << 20, (2 << 20) + 11])
def test_single_object_staging_paths(oracle, monkeypatch, pinned_max, n):
    """Single-object encode / decode / reconstruct through both staging paths:
    DMA copies through HBM (ECAMD_SINGLE_PINNED_MAX=0), zero-copy pinned host
    memory (any size), and the default split at 1 MiB -- bit-exact against the
    oracle, decode with data fragments missing so the kernels run."""
    monkeypatch.setenv("ECAMD_SINGLE_PINNED_MAX", pinned_max)
    k, m = 10, 4
    drv = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand")
    data = os.urandom(n)
    frags = drv.encode(data)
    assert frags == oracle.encode(k, m, data)
    assert drv.decode(frags[m:]) == data
    assert drv.decode(frags[2:2 + k]) == data
    assert drv.reconstruct(frags[1:k + 1], [0])[0] == frags[0]
    assert drv.reconstruct(frags[:k], [k + 2])[0] == frags[k + 2]
    drv.close()


@pytest.mark.parametrize("n", [1, 4093, (1 << 20) + 5, (4 << 20) + 17])
def test_liberasurecode_entry_points_match_into_forms(oracle, n):
    """The entry points pyeclib_c.c binds (liberasurecode_encode / _decode /
    _cleanup, pyeclib_c.c:537, :562, :878, :919) called through ctypes, as
    the reference binding calls them: the same fragments as the oracle and as
    the ecamd_*_into forms the Python binding uses, and the same decoded bytes."""
    import ctypes
    P = ctypes.POINTER
    k, m = 10, 4
    drv = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand")
    desc = drv.ec_lib_reference.handle.desc
    data = os.urandom(n)
    dat, par = P(ctypes.c_void_p)(), P(ctypes.c_void_p)()
    flen = ctypes.c_uint64(0)
    assert _native.lib.liberasurecode_encode(desc, data, n, ctypes.byref(dat), ctypes.byref(par),
                                             ctypes.byref(flen)) == 0
    fl = flen.value
    frags = [ctypes.string_at(dat[i], fl) for i in range(k)] + \
            [ctypes.string_at(par[i], fl) for i in range(m)]
    assert _native.lib.liberasurecode_encode_cleanup(desc, dat, par) == 0
    assert frags == oracle.encode(k, m, data)
    assert drv.encode(data) == frags  # ecamd_encode_into
    for avail in (frags[m:m + k], frags[:k]):  # GPU path, concatenation fast path
        arr = (ctypes.c_char_p * k)(*avail)
        out, olen = ctypes.c_void_p(), ctypes.c_uint64(0)
        assert _native.lib.liberasurecode_decode(desc, arr, k, fl, 0, ctypes.byref(out),
                                                 ctypes.byref(olen)) == 0
        assert olen.value == n and ctypes.string_at(out.value, n) == data
        assert _native.lib.liberasurecode_decode_cleanup(desc, out) == 0
        assert drv.decode(avail) == data  # ecamd_decode_into
    drv.close()
