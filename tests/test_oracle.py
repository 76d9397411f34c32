"""CPU oracle checks (no GPU): the C restatement against an independent numpy
restatement, the structural known answers of the rs_vand construction, the
80-byte header format and the committed golden fixtures."""
import hashlib
import json
import os
import zlib

import numpy as np
import pytest

from oracle import oracle_np as N

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "rs_vand_golden.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_gf_field_basics(oracle):
    # x * x^15 = x^16 = 0x1100B - 0x10000 = 0x100B (primitive polynomial, rs_galois.c)
    assert oracle.gf_mul(2, 0x8000) == 0x100B
    for a, b in [(0x1234, 0x5678), (3, 7), (0xFFFF, 0xFFFF), (1, 0xBEEF), (0, 77)]:
        assert oracle.gf_mul(a, b) == N.gf_mul(a, b)
        if b:
            assert oracle.gf_mul(oracle.gf_div(a, b), b) == a


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (4, 2), (10, 4), (12, 2), (11, 2), (8, 4),
                                 (3, 5), (6, 9), (20, 4), (28, 4), (16, 16)])
def test_generator_matches_independent_restatement(oracle, k, m):
    g = oracle.generator(k, m)
    assert g == N.generator(k, m)
    assert g[:k] == [[int(i == j) for j in range(k)] for i in range(k)]  # systematic
    assert g[k] == [1] * k  # first parity row all ones -> parity 0 = XOR of data
    assert all(v != 0 for row in g[k:] for v in row)  # MDS: no zero coefficient


@pytest.mark.parametrize("k,m,n", [(4, 2, 1000), (10, 4, 4099), (3, 5, 77), (12, 2, 65536 + 6)])
def test_encode_matches_numpy(oracle, k, m, n):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    frags = oracle.encode(k, m, data)
    assert [f[80:] for f in frags] == N.encode_payloads(k, m, data)


def test_structural_known_answers(oracle):
    k, m, n = 10, 4, 100003
    data = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8).tobytes()
    frags = oracle.encode(k, m, data)
    bs = oracle.blocksize(k, n)
    assert bs == 2 * -(-n // (2 * k))
    assert all(len(f) == 80 + bs for f in frags)
    padded = data + bytes(k * bs - n)
    for j in range(k):
        assert frags[j][80:] == padded[j * bs:(j + 1) * bs]
    x = np.zeros(bs, dtype=np.uint8)
    for j in range(k):
        x ^= np.frombuffer(frags[j][80:], dtype=np.uint8)
    assert frags[k][80:] == x.tobytes()


def test_header_layout(oracle):
    k, m, n = 4, 2, 12345
    data = os.urandom(n)
    for ct in (oracle.CHKSUM_NONE, oracle.CHKSUM_CRC32):
        for i, f in enumerate(oracle.encode(k, m, data, ct=ct)):
            h = f[:80]
            bs = len(f) - 80
            assert int.from_bytes(h[0:4], "little") == i
            assert int.from_bytes(h[4:8], "little") == bs
            assert int.from_bytes(h[8:12], "little") == 0
            assert int.from_bytes(h[12:20], "little") == n
            assert h[20] == ct
            want = zlib.crc32(f[80:]) if ct == oracle.CHKSUM_CRC32 else 0
            assert int.from_bytes(h[21:25], "little") == want
            assert h[25:53] == bytes(28)
            assert h[53] == 0 and h[54] == 6
            assert int.from_bytes(h[55:59], "little") == 0x00010000
            assert int.from_bytes(h[59:63], "little") == 0xB0C5ECC
            assert int.from_bytes(h[63:67], "little") == 0x010800
            assert int.from_bytes(h[67:71], "little") == zlib.crc32(h[:59])
            assert h[71:80] == bytes(9)


def test_oracle_roundtrips(oracle):
    import itertools
    k, m = 6, 3
    data = os.urandom(5001)
    frags = oracle.encode(k, m, data)
    for lost in itertools.combinations(range(k + m), m):
        avail = [f for i, f in enumerate(frags) if i not in lost]
        assert oracle.decode(k, m, avail) == data
        for i in lost:
            assert oracle.reconstruct(k, m, avail, i) == frags[i]


def test_golden_generators(oracle, golden):
    for key, rows in golden["generator"].items():
        k, m = map(int, key.split(","))
        assert oracle.generator(k, m)[k:] == rows
    for a, b, c in golden["gf_mul"]:
        assert oracle.gf_mul(a, b) == c == N.gf_mul(a, b)


def test_golden_small_vectors(oracle, golden):
    for case in golden["small"]:
        frags = oracle.encode(case["k"], case["m"], bytes.fromhex(case["data"]))
        assert [f.hex() for f in frags] == case["fragments"]


def test_golden_digests(oracle, golden):
    pdf = open(os.path.join(HERE, "golden", "storer-storagess06.pdf"), "rb").read()
    for case in golden["sha"]:
        src = case["source"]
        if src.startswith("file:"):
            data = pdf
        else:
            _, seed, n = src.split(":")
            data = np.random.Generator(np.random.PCG64(int(seed))).integers(
                0, 256, int(n), dtype=np.uint8).tobytes()
        assert hashlib.sha256(data).hexdigest() == case["data_sha256"]
        frags = oracle.encode(case["k"], case["m"], data)
        assert [hashlib.sha256(f).hexdigest() for f in frags] == case["fragments_sha256"]


# ---------------- GF(2^8) ISA-L oracle (isal_oracle.c) ----------------

@pytest.mark.parametrize("kind,name", [(4, "vand"), (7, "cauchy")])
@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (12, 4), (8, 4), (12, 2), (11, 7)])
def test_isal_oracle_matches_numpy(oracle, kind, name, k, m):
    g = oracle.isal_generator(kind, k, m)
    assert g == N.isal_generator(name, k, m)
    assert g[:k] == [[int(i == j) for j in range(k)] for i in range(k)]
    data = np.random.default_rng(k * 100 + m).integers(0, 256, 5003, dtype=np.uint8).tobytes()
    frags = oracle.isal_encode(kind, k, m, data)
    assert [f[80:] for f in frags] == N.isal_encode_payloads(name, k, m, data)
    bs = -(-len(data) // k)  # ISA-L alignment: multiple of k bytes (w = 8)
    assert all(len(f) == 80 + bs for f in frags)
    for i, f in enumerate(frags):
        assert int.from_bytes(f[0:4], "little") == i and f[54] == kind


def test_isal_known_answers(oracle):
    # gf_gen_rs_matrix: first parity row all ones, second row powers of 2
    g = oracle.isal_generator(4, 6, 3)
    assert g[6] == [1] * 6
    assert g[7] == [1, 2, 4, 8, 16, 32]
    assert g[8] == [1, 4, 16, 64, 29, 116]  # 4^j over 0x11D: 4^4 = 256 ^ 0x11D = 29
    # gf_gen_cauchy1_matrix: 1 / (i ^ j); 4 * 71 = 1 in GF(2^8)/0x11D
    c = oracle.isal_generator(7, 4, 2)
    assert c[4][0] == 71 and oracle.isal_gf_mul(4, 71) == 1
    assert all(oracle.isal_gf_mul(c[i][j], i ^ j) == 1 for i in (4, 5) for j in range(4))


def test_isal_oracle_roundtrips(oracle):
    import itertools
    k, m = 6, 3
    data = os.urandom(4001)
    for kind in (4, 7):
        frags = oracle.isal_encode(kind, k, m, data)
        for lost in itertools.combinations(range(k + m), m):
            avail = [f for i, f in enumerate(frags) if i not in lost]
            assert oracle.isal_decode(kind, k, m, avail) == data
            for i in lost:
                assert oracle.isal_reconstruct(kind, k, m, avail, i) == frags[i]
