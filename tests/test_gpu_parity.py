"""GPU parity: the MI355X path (through the C ABI) against the CPU oracle.

Bit-exact comparisons of whole fragments (80-byte header + payload), decoded
objects and reconstructed fragments, on seeded inputs at sizes the oracle
finishes in seconds.  Every call below goes through libpyeclib_amd.so.
"""
import itertools
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# m = 5..8 (rs_vand): one eight-row encode pass (Gf16x8); m = 9: four-row passes
CONFIGS = [(4, 2), (10, 4), (12, 2), (11, 2), (10, 2), (8, 4), (12, 4), (3, 5), (6, 9), (20, 4),
           (1, 1), (2, 1), (28, 4), (10, 5), (12, 6), (8, 8), (7, 7), (24, 8)]
LENGTHS = [1, 2, 9, 31, 100, 1000, 4099, 8192, 65536 + 3, 262144, 1 << 20]


def _data(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


@pytest.fixture(scope="module")
def amd():
    from pyeclib_amd import ECDriver
    return ECDriver


@pytest.mark.parametrize("k,m", CONFIGS)
def test_encode_matches_oracle(amd, oracle, k, m):
    drv = amd(k=k, m=m, ec_type="amd_rs_vand")
    for i, n in enumerate(LENGTHS):
        data = _data(n, 1000 * k + 10 * m + i)
        got = drv.encode(data)
        want = oracle.encode(k, m, data)
        assert len(got) == k + m
        for idx, (g, w) in enumerate(zip(got, want)):
            assert g == w, f"k={k} m={m} len={n} fragment {idx} differs"


@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (12, 2), (8, 4), (3, 5), (6, 9), (10, 5),
                                 (12, 6), (8, 8)])
def test_decode_reconstruct_random_erasures(amd, oracle, k, m):
    drv = amd(k=k, m=m, ec_type="liberasurecode_rs_vand")
    rng = random.Random(k * 31 + m)
    for n in (1, 77, 4099, 300001):
        data = _data(n, n + k)
        frags = oracle.encode(k, m, data)
        for _ in range(6):
            lost = sorted(rng.sample(range(k + m), rng.randint(1, m)))
            avail = [f for i, f in enumerate(frags) if i not in lost]
            rng.shuffle(avail)
            assert drv.decode(avail) == data
            rebuilt = drv.reconstruct(avail, list(lost))
            for idx, frag in zip(lost, rebuilt):
                assert frag == frags[idx], f"reconstruct {idx} k={k} m={m} len={n}"


def test_exhaustive_erasures_k10_m4(amd, oracle):
    k, m = 10, 4
    drv = amd(k=k, m=m, ec_type="amd_rs_vand")
    data = _data(10000, 7)
    frags = drv.encode(data)
    assert frags == oracle.encode(k, m, data)
    for lost in itertools.combinations(range(k + m), m):
        avail = [f for i, f in enumerate(frags) if i not in lost]
        assert drv.decode(avail) == data, lost
    for lost in itertools.combinations(range(k + m), 2):
        avail = [f for i, f in enumerate(frags) if i not in lost]
        for idx in lost:
            assert drv.reconstruct(avail, [idx])[0] == frags[idx]


def test_inline_crc32_headers(amd, oracle):
    for k, m in [(12, 2), (8, 4)]:
        drv = amd(k=k, m=m, ec_type="amd_rs_vand", chksum_type="inline_crc32")
        data = _data(3 * 1024 * 1024, 3)
        got = drv.encode(data)
        assert got == oracle.encode(k, m, data, ct=oracle.CHKSUM_CRC32)
        lost = [1, k]
        avail = [f for i, f in enumerate(got) if i not in lost]
        for idx, frag in zip(lost, drv.reconstruct(avail, lost)):
            assert frag == got[idx]


# ---------------- device-resident batch API ----------------

def _batch_layout(k, m, n_obj, obj_len):
    from pyeclib_amd import batch
    bs = batch.blocksize(k, obj_len)
    obj_stride = (obj_len + 15) // 16 * 16
    frag_stride = batch.frag_stride(bs)
    return bs, obj_stride, frag_stride


@pytest.mark.parametrize("k,m,obj_len", [(10, 4, 1 << 20), (10, 4, 4 * 1024 * 1024 // 7),
                                         (4, 2, 100001), (12, 4, 999999), (6, 9, 65538),
                                         (3, 1, 17), (10, 4, 10 * 4096 * 3),
                                         (8, 3, 8 * 8192), (10, 4, 10 * 4096 + 2),
                                         # prime k: padded stream slots (NB = 4)
                                         (7, 3, 7 * 4096 * 5 + 13), (11, 4, 1 << 20),
                                         (13, 3, (2 << 20) + 6),
                                         # one eight-row encode pass (m = 5..8)
                                         (10, 5, 1 << 20), (12, 6, 999999), (8, 8, 8 * 4096 * 7 + 10),
                                         (5, 7, 65536 + 6)])
def test_batch_encode_decode_reconstruct(oracle, gpu, k, m, obj_len):
    import torch
    from pyeclib_amd import batch
    n_obj = 5
    codec = batch.BatchCodec(k, m)
    bs, obj_stride, frag_stride = _batch_layout(k, m, n_obj, obj_len)
    host = torch.from_numpy(np.random.default_rng(obj_len).integers(
        0, 256, (n_obj, obj_stride), dtype=np.uint8))
    objs = host.to(gpu)
    frags = torch.zeros((n_obj, k + m, frag_stride), dtype=torch.uint8, device=gpu)
    codec.encode(objs, obj_len, parity=frags[:, k:], data=frags[:, :k])
    torch.cuda.synchronize()
    fl = 80 + bs
    got = frags.cpu().numpy()
    for o in range(n_obj):
        want = oracle.encode(k, m, host[o, :obj_len].numpy().tobytes())
        for i in range(k + m):
            assert got[o, i, :fl].tobytes() == want[i], f"obj {o} fragment {i}"
    # decode with per-object erasures (all patterns different)
    rng = random.Random(obj_len)
    masks = []
    for o in range(n_obj):
        lost = rng.sample(range(k + m), rng.randint(0, m))
        masks.append(sum(1 << i for i in range(k + m) if i not in lost))
    out = torch.zeros((n_obj, obj_stride), dtype=torch.uint8, device=gpu)
    codec.decode(frags, obj_len, masks, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :obj_len].cpu(), host[:, :obj_len])
    # reconstruct one missing fragment per object
    dest = [rng.randrange(k + m) for _ in range(n_obj)]
    masks2 = [mk & ~(1 << d) for mk, d in zip(masks, dest)]
    masks2 = [mk if bin(mk).count("1") >= k else ((1 << (k + m)) - 1) & ~(1 << d)
              for mk, d in zip(masks2, dest)]
    rec = torch.zeros((n_obj, frag_stride), dtype=torch.uint8, device=gpu)
    codec.reconstruct(frags, obj_len, masks2, dest, rec)
    torch.cuda.synchronize()
    rec = rec.cpu().numpy()
    for o in range(n_obj):
        assert rec[o, :fl].tobytes() == got[o, dest[o], :fl].tobytes(), f"obj {o} dest {dest[o]}"


def test_golden_fixtures_on_gpu(amd):
    """The committed golden vectors (tests/golden, made by the oracle) through
    the GPU path: full fragments for small inputs, SHA-256 digests for the
    4 MiB / 1 MiB PCG64 objects and for the reference's PDF test file."""
    import hashlib
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    golden = json.load(open(os.path.join(here, "rs_vand_golden.json")))
    for case in golden["small"]:
        drv = amd(k=case["k"], m=case["m"], ec_type="amd_rs_vand")
        assert [f.hex() for f in drv.encode(bytes.fromhex(case["data"]))] == case["fragments"]
    pdf = open(os.path.join(here, "storer-storagess06.pdf"), "rb").read()
    for case in golden["sha"]:
        if case["source"].startswith("file:"):
            data = pdf
        else:
            _, seed, n = case["source"].split(":")
            data = np.random.Generator(np.random.PCG64(int(seed))).integers(
                0, 256, int(n), dtype=np.uint8).tobytes()
        drv = amd(k=case["k"], m=case["m"], ec_type="amd_rs_vand")
        frags = drv.encode(data)
        assert [hashlib.sha256(f).hexdigest() for f in frags] == case["fragments_sha256"]
    for case in golden["decode"]:
        k, m = case["k"], case["m"]
        drv = amd(k=k, m=m, ec_type="amd_rs_vand")
        frags = drv.encode(pdf)
        avail = [f for i, f in enumerate(frags) if i not in case["lost"]]
        assert drv.decode(avail) == pdf
        rebuilt = drv.reconstruct(avail, list(case["lost"]))
        assert [hashlib.sha256(f).hexdigest() for f in rebuilt] == case["rebuilt_sha256"]


@pytest.mark.parametrize("obj_len", [4 * 1024 * 1024, 4194560, 3 * 1024 * 1024 + 22,
                                     10 * 4096 * 102])
def test_batch_full_size_properties(gpu, obj_len):
    """Full-size batch (64 x ~4 MiB, k=10 m=4): size-independent properties
    instead of the oracle -- parity row 0 == XOR of the data fragments, every
    erasure pattern class decodes back to the objects, and reconstructed
    fragments equal the encoded ones."""
    import torch
    from pyeclib_amd import batch
    k, m, n_obj = 10, 4, 64
    codec = batch.BatchCodec(k, m)
    bs = batch.blocksize(k, obj_len)
    stride = (obj_len + 255) // 256 * 256
    objs = torch.randint(0, 256, (n_obj, stride), dtype=torch.uint8, device=gpu)
    objs[:, obj_len:] = 0
    stripes = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(objs, obj_len, parity=stripes[:, k:], data=stripes[:, :k])
    payload = stripes[:, :, 80:80 + bs]
    x = payload[:, 0].clone()
    for j in range(1, k):
        x ^= payload[:, j]
    assert torch.equal(x, payload[:, k])
    rng = random.Random(obj_len)
    full = (1 << (k + m)) - 1
    masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), o % (m + 1)))
             for o in range(n_obj)]
    out = torch.zeros_like(objs)
    codec.decode(stripes, obj_len, masks, out)
    assert torch.equal(out[:, :obj_len], objs[:, :obj_len])
    dest = [rng.randrange(k + m) for _ in range(n_obj)]
    masks2 = [full & ~(1 << d) for d in dest]
    rec = torch.zeros((n_obj, stripes.shape[2]), dtype=torch.uint8, device=gpu)
    codec.reconstruct(stripes, obj_len, masks2, dest, rec)
    for o in range(n_obj):
        assert torch.equal(rec[o, :80 + bs], stripes[o, dest[o], :80 + bs]), o


# ---------------- GF(2^8) ISA-L codes (isa_l_rs_vand / isa_l_rs_cauchy) ----------------

ISAL = [("isa_l_rs_vand", 4), ("isa_l_rs_cauchy", 7)]


@pytest.mark.parametrize("ec_type,kind", ISAL)
@pytest.mark.parametrize("k,m", [(4, 2), (10, 4), (12, 4), (12, 2), (8, 4), (11, 2), (3, 5)])
def test_isal_encode_matches_oracle(amd, oracle, ec_type, kind, k, m):
    drv = amd(k=k, m=m, ec_type=ec_type)
    for i, n in enumerate([1, 2, 9, 31, 100, 1000, 4099, 65536 + 3, 262144 + 7, 1 << 20]):
        data = _data(n, 7000 + 10 * k + m + i)
        got = drv.encode(data)
        want = oracle.isal_encode(kind, k, m, data)
        for idx, (g, w) in enumerate(zip(got, want)):
            assert g == w, f"{ec_type} k={k} m={m} len={n} fragment {idx} differs"


@pytest.mark.parametrize("ec_type,kind", ISAL)
@pytest.mark.parametrize("k,m", [(4, 2), (12, 4), (8, 4)])
def test_isal_decode_reconstruct(amd, oracle, ec_type, kind, k, m):
    drv = amd(k=k, m=m, ec_type=ec_type)
    rng = random.Random(k * 7 + m + kind)
    for n in (1, 77, 4099, 300001):
        data = _data(n, n + k + kind)
        frags = oracle.isal_encode(kind, k, m, data)
        for _ in range(5):
            lost = sorted(rng.sample(range(k + m), rng.randint(1, m)))
            avail = [f for i, f in enumerate(frags) if i not in lost]
            rng.shuffle(avail)
            assert drv.decode(avail) == data
            for idx, frag in zip(lost, drv.reconstruct(avail, list(lost))):
                assert frag == frags[idx], f"{ec_type} reconstruct {idx} k={k} m={m} len={n}"


@pytest.mark.parametrize("k,m,obj_len", [(12, 4, 1 << 20), (12, 4, 999999), (10, 4, 65537),
                                         (6, 2, 12 * 4096 * 3 + 5), (11, 3, (1 << 20) + 3),
                                         (7, 4, 7 * 4096 * 9)])
def test_isal_cauchy_batch(oracle, gpu, k, m, obj_len):
    """Device-resident batch API on the GF(2^8) Cauchy code (BASELINE config 4
    shape at a small batch): encode vs oracle, decode, reconstruct."""
    import torch
    from pyeclib_amd import batch
    n_obj = 4
    codec = batch.BatchCodec(k, m, ec_type="isa_l_rs_cauchy")
    bs = batch.blocksize(k, obj_len, w=8)
    stride = (obj_len + 15) // 16 * 16
    host = torch.from_numpy(np.random.default_rng(obj_len).integers(
        0, 256, (n_obj, stride), dtype=np.uint8))
    objs = host.to(gpu)
    frags = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(objs, obj_len, parity=frags[:, k:], data=frags[:, :k])
    torch.cuda.synchronize()
    got = frags.cpu().numpy()
    for o in range(n_obj):
        want = oracle.isal_encode(7, k, m, host[o, :obj_len].numpy().tobytes())
        for i in range(k + m):
            assert got[o, i, :80 + bs].tobytes() == want[i], f"obj {o} fragment {i}"
    rng = random.Random(obj_len)
    full = (1 << (k + m)) - 1
    masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), m)) for _ in range(n_obj)]
    out = torch.zeros((n_obj, stride), dtype=torch.uint8, device=gpu)
    codec.decode(frags, obj_len, masks, out)
    torch.cuda.synchronize()
    assert torch.equal(out[:, :obj_len].cpu(), host[:, :obj_len])
    dest = [rng.randrange(k + m) for _ in range(n_obj)]
    rec = torch.zeros((n_obj, frags.shape[2]), dtype=torch.uint8, device=gpu)
    codec.reconstruct(frags, obj_len, [full & ~(1 << d) for d in dest], dest, rec)
    torch.cuda.synchronize()
    rec = rec.cpu().numpy()
    for o in range(n_obj):
        assert rec[o, :80 + bs].tobytes() == got[o, dest[o], :80 + bs].tobytes()


# ---------------- inline CRC-32 on the batch path (GPU payload CRC kernel) ----------------

@pytest.mark.parametrize("ec_type,k,m,obj_len,n_obj", [
    ("amd_rs_vand", 10, 4, 4 * 1024 * 1024, 3), ("amd_rs_vand", 4, 2, 100001, 3),
    ("amd_rs_vand", 12, 2, 4096 * 12 * 2, 3), ("amd_rs_vand", 3, 1, 17, 3),
    ("isa_l_rs_cauchy", 12, 4, 999999, 3), ("isa_l_rs_vand", 8, 4, 65537, 3),
    # many objects per launch (the loader / consumer kernels; the stream
    # kernels take the small batches above), multi-pass parity (m > 4)
    ("amd_rs_vand", 10, 4, 4 * 1024 * 1024, 160), ("amd_rs_vand", 6, 6, 300000, 40),
    ("isa_l_rs_cauchy", 12, 4, 3 * 1024 * 1024 + 5, 48)])
def test_batch_inline_crc32(oracle, gpu, ec_type, k, m, obj_len, n_obj):
    """chksum_type inline_crc32 on device-resident batches: every header
    (payload CRC-32 + metadata checksum) equals the oracle's, for encode with
    data fragments, encode of the parity alone, and reconstruct.  Each launch
    stores its 1 KiB chunks' CRCs and a finishing pass sets the headers
    (ec_crc.hip); no pass re-reads the payloads."""
    _check_batch_crc(oracle, gpu, ec_type, k, m, obj_len, n_obj, legacy=False)


@pytest.mark.parametrize("ec_type,k,m,obj_len,n_obj", [
    ("amd_rs_vand", 10, 4, 1 << 20, 5), ("amd_rs_vand", 10, 4, 4 * 1024 * 1024, 12),
    ("amd_rs_vand", 6, 6, 300001, 4), ("isa_l_rs_vand", 8, 4, 65537, 3)])
def test_batch_legacy_crc32(oracle, gpu, monkeypatch, ec_type, k, m, obj_len, n_obj):
    """LIBERASURECODE_WRITE_LEGACY_CRC=1: the batch encode and reconstruct
    write liberasurecode's legacy CRC (liberasurecode_crc32_alt) into the
    payload and metadata checksums, as the reference path does in every call
    (pyeclib_c.c:248)."""
    monkeypatch.setenv("LIBERASURECODE_WRITE_LEGACY_CRC", "1")
    _check_batch_crc(oracle, gpu, ec_type, k, m, obj_len, n_obj, legacy=True)


def _check_batch_crc(oracle, gpu, ec_type, k, m, obj_len, n_obj, legacy):
    import torch
    from pyeclib_amd import batch
    codec = batch.BatchCodec(k, m, inline_crc32=True, ec_type=ec_type)
    bs = codec.blocksize(obj_len)
    stride = (obj_len + 15) // 16 * 16
    host = torch.from_numpy(np.random.default_rng(obj_len + k).integers(
        0, 256, (n_obj, stride), dtype=np.uint8))
    frags = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(host.to(gpu), obj_len, parity=frags[:, k:], data=frags[:, :k])
    torch.cuda.synchronize()
    got = frags.cpu().numpy()
    for o in range(n_obj):
        data = host[o, :obj_len].numpy().tobytes()
        if codec.w == 8:
            kind = 7 if ec_type == "isa_l_rs_cauchy" else 4
            want = oracle.isal_encode(kind, k, m, data, ct=oracle.CHKSUM_CRC32)
        else:
            want = oracle.encode(k, m, data, ct=oracle.CHKSUM_CRC32)
        if legacy:
            want = [oracle.legacy_headers(f) for f in want]
        for i in range(k + m):
            assert got[o, i, :80 + bs].tobytes() == want[i], f"obj {o} fragment {i}"
    # the parity alone (no data fragments): same parity fragments
    par = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(host.to(gpu), obj_len, parity=par[:, k:])
    torch.cuda.synchronize()
    assert np.array_equal(par[:, k:].cpu().numpy()[:, :, :80 + bs], got[:, k:, :80 + bs])
    full = (1 << (k + m)) - 1
    dest = [(o * 5 + 1) % (k + m) for o in range(n_obj)]
    rec = torch.zeros((n_obj, frags.shape[2]), dtype=torch.uint8, device=gpu)
    codec.reconstruct(frags, obj_len, [full & ~(1 << d) for d in dest], dest, rec)
    torch.cuda.synchronize()
    rec = rec.cpu().numpy()
    for o in range(n_obj):
        assert rec[o, :80 + bs].tobytes() == got[o, dest[o], :80 + bs].tobytes()


# ---------------- large single-object calls ----------------

@pytest.mark.parametrize("ec_type,k,m,n", [
    ("liberasurecode_rs_vand", 10, 4, (2 << 20) + 2), ("amd_rs_vand", 12, 6, 3 * (1 << 20) + 7),
    ("amd_rs_vand", 6, 9, (2 << 20) + 1), ("amd_rs_vand", 3, 5, (2 << 20) + 33),
    ("amd_rs_vand", 28, 4, 5 * (1 << 20) + 9), ("isa_l_rs_cauchy", 12, 4, (4 << 20) + 5),
    ("isa_l_rs_vand", 8, 3, (2 << 20) + 1), ("liberasurecode_rs_vand", 10, 4, 4 << 20)])
def test_single_object_large(oracle, ec_type, k, m, n):
    """Single-object encode / decode / reconstruct of 2-5 MiB objects (the
    pinned staging path), multi-pass parity and multi-pass decode (m > 4)
    included, both fields: fragments and decoded bytes against the oracle.
    (Round 5 also ran these calls in windows of payload positions, staging
    window w + 1 while the GPU ran window w: slower at 1 and 4 MiB, because
    the copy pool's wake-up per window cost more than the overlap gained --
    profiles/r05h_single_probe_windows.txt, r05i_single_probe_windows.txt -- so not kept.)"""
    from pyeclib_amd import ECDriver
    drv = ECDriver(k=k, m=m, ec_type=ec_type)
    data = _data(n, n + 7 * k)
    frags = drv.encode(data)
    if ec_type.startswith("isa_l"):
        want = oracle.isal_encode(7 if ec_type == "isa_l_rs_cauchy" else 4, k, m, data)
    else:
        want = oracle.encode(k, m, data)
    assert frags == want
    rng = random.Random(n)
    for _ in range(3):
        lost = sorted(rng.sample(range(k + m), m))
        avail = [f for i, f in enumerate(frags) if i not in lost]
        rng.shuffle(avail)
        assert drv.decode(avail) == data
        assert drv.reconstruct(avail, lost[:2]) == [frags[i] for i in lost[:2]]
    drv.close()


@pytest.mark.parametrize("n_obj,obj_len", [(64, 4 << 20), (7, 300001)])
def test_back_to_back_calls_with_erased_bytes(gpu, n_obj, obj_len):
    """Decodes and reconstructs issued back to back with no synchronisation,
    each call with new erasure masks over its own copy of the stripes whose
    erased fragments are ZEROED: a call that ran with another call's
    descriptors or table sets (the upload ring, the host-side upload waits,
    round 5) would read zeros and differ.  The batch tests' stripes keep every
    fragment intact, so any valid pattern decodes them -- they cannot see
    that.  64 x 4 MiB takes the loader / consumer decode, 7 x 300 KB the
    stream kernels."""
    import torch
    from pyeclib_amd import batch
    k, m, rounds = 10, 4, 8
    codec = batch.BatchCodec(k, m)
    bs, obj_stride, frag_stride = _batch_layout(k, m, n_obj, obj_len)
    g = torch.Generator(device="cpu").manual_seed(obj_len)
    objs = torch.randint(0, 256, (n_obj, obj_stride), dtype=torch.uint8, generator=g).to(gpu)
    frags = torch.zeros((n_obj, k + m, frag_stride), dtype=torch.uint8, device=gpu)
    codec.encode(objs, obj_len, parity=frags[:, k:], data=frags[:, :k])
    torch.cuda.synchronize()
    rng = np.random.default_rng(n_obj)
    jobs = []
    for r in range(rounds):
        lost = [rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False) for _ in range(n_obj)]
        masks = [sum(1 << i for i in range(k + m) if i not in ls) for ls in lost]
        st = frags.clone()
        gone = torch.zeros((n_obj, k + m), dtype=torch.bool)
        for o, ls in enumerate(lost):
            gone[o, torch.as_tensor(ls)] = True
        st[gone.to(gpu)] = 0
        out = torch.zeros((n_obj, obj_stride), dtype=torch.uint8, device=gpu)
        dest = [int(ls[0]) for ls in lost]
        rec = torch.zeros((n_obj, frag_stride), dtype=torch.uint8, device=gpu)
        jobs.append((st, masks, out, dest, rec))
    torch.cuda.synchronize()
    for st, masks, out, dest, rec in jobs:  # no synchronisation between the calls
        codec.decode(st, obj_len, masks, out)
        codec.reconstruct(st, obj_len, masks, dest, rec)
    torch.cuda.synchronize()
    fl = 80 + bs
    for r, (st, masks, out, dest, rec) in enumerate(jobs):
        assert torch.equal(out[:, :obj_len], objs[:, :obj_len]), f"round {r} decode"
        want = frags[torch.arange(n_obj, device=gpu), torch.as_tensor(dest, device=gpu), :fl]
        assert torch.equal(rec[:, :fl], want), f"round {r} reconstruct"
