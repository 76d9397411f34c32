"""Parity against a SYSTEM liberasurecode, when one is installed (SURVEY.md
section 8(c), upgrade path).  This image has none, so these tests skip here
and on the GPU boxes of this pool; where liberasurecode exists they pin the
oracle (CPU) and the GPU path (gpu) to the real library's bytes."""
import numpy as np
import pytest

from pyeclib_amd import system_liberasurecode as S

pytestmark = pytest.mark.skipif(S.probe() is None, reason="no system liberasurecode")

CASES = [(4, 2, 1), (4, 2, 1000), (10, 4, 4 << 20), (10, 4, 999999), (12, 6, 65537), (8, 8, 12345)]


def _data(n):
    return np.random.Generator(np.random.PCG64(n)).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("k,m,n", CASES)
@pytest.mark.parametrize("crc32", [False, True])
def test_oracle_matches_system_liberasurecode(oracle, k, m, n, crc32):
    ref = S.SystemLibrary().encode(k, m, _data(n), crc32=crc32)
    got = oracle.encode(k, m, _data(n), ct=oracle.CHKSUM_CRC32 if crc32 else oracle.CHKSUM_NONE)
    assert [S.comparable(f) for f in got] == [S.comparable(f) for f in ref]


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,n", CASES)
def test_gpu_matches_system_liberasurecode(k, m, n):
    from pyeclib_amd import ECDriver
    ref = S.SystemLibrary().encode(k, m, _data(n))
    got = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand").encode(_data(n))
    assert [S.comparable(f) for f in got] == [S.comparable(f) for f in ref]
