"""BASELINE configs at their real sizes, plus the host-resident paths and the
decode table-pool recycling, on the GPU through the C ABI.

Full-size batches are checked object by object against the CPU oracle with
the same routine bench.py uses on its timed batch (bench.oracle_pass): every
fragment (80-byte header + payload) of every object, and every decoded object
or rebuilt fragment.
"""
import argparse
import os
import random
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _inputs(B, n, k, m, erasures, seed):
    import bench
    rng = np.random.Generator(np.random.PCG64(seed))
    host = np.zeros((B, (n + 255) // 256 * 256), dtype=np.uint8)
    host[:, :n] = rng.integers(0, 256, size=(B, n), dtype=np.uint8)
    masks = bench.erasure_masks(rng, B, k, m, erasures)
    dests = [int(d) for d in rng.integers(0, k + m, size=B)]
    return host, masks, dests


def _device_batch(gpu, ec_type, k, m, n, B, second, erasures=4, seed=20261015):
    """Encode (data fragments materialised) + decode / reconstruct a batch on
    the GPU; returns what bench.oracle_pass needs."""
    import torch
    from pyeclib_amd import batch
    host, masks, dests = _inputs(B, n, k, m, erasures, seed)
    full = (1 << (k + m)) - 1
    if second == "reconstruct":
        masks = [full & ~(1 << d) for d in dests]
    codec = batch.BatchCodec(k, m, ec_type=ec_type)
    bs = codec.blocksize(n)
    fl = 80 + bs
    objs = torch.from_numpy(host).to(gpu)
    stripes = batch.stripe_buffer(B, k, m, bs, device=gpu)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    if second == "decode":
        out = torch.zeros_like(objs)
        codec.decode(stripes, n, masks, out)
        g2 = out[:, :n]
    else:
        out = torch.zeros((B, stripes.shape[2]), dtype=torch.uint8, device=gpu)
        codec.reconstruct(stripes, n, masks, dests, out)
        g2 = out[:, :fl]
    torch.cuda.synchronize()
    gf = stripes[:, :, :fl].cpu().numpy()
    g2 = g2.cpu().numpy()
    del stripes, out, objs
    args = argparse.Namespace(ec_type=ec_type, k=k, m=m, obj_bytes=n, second=second)
    return args, host, masks, dests, gf, g2


def test_config1_2_full_batch_256x4MiB(gpu):
    """configs[1] + configs[2]: k=10 m=4 rs_vand, 256 x 4 MiB, decode with 4
    random erasures per object -- the bench's exact workload."""
    import bench
    args, host, masks, dests, gf, g2 = _device_batch(gpu, "amd_rs_vand", 10, 4, 4 << 20, 256,
                                                     "decode")
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=256)
    assert bad == []


def test_config3_per_gpu_shard_128x16MiB_cauchy(gpu):
    """configs[3] as one GPU's shard of 1024 objects over 8 GPUs: k=12 m=4
    isa_l_rs_cauchy (GF(2^8)), 128 x 16 MiB, encode + reconstruct of one
    random fragment per object."""
    import bench
    args, host, masks, dests, gf, g2 = _device_batch(gpu, "isa_l_rs_cauchy", 12, 4, 16 << 20,
                                                     128, "reconstruct")
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=128)
    assert bad == []


def test_decode_pool_recycles_safely(gpu, oracle, monkeypatch):
    """More distinct erasure patterns in one call than the decode table pool
    holds (forced to 5 slots), and patterns carried over between calls: the
    runtime must launch the objects holding slots before recycling the pool.
    k=28 m=4 has C(32,4) = 35,960 patterns."""
    import torch
    from pyeclib_amd import batch
    monkeypatch.setenv("ECAMD_POOL_SLOTS", "5")
    k, m, n, B = 28, 4, 28 * 2 * 300 + 6, 23
    codec = batch.BatchCodec(k, m)
    bs = codec.blocksize(n)
    host, _, _ = _inputs(B, n, k, m, 0, 11)
    rng = random.Random(5)
    full = (1 << (k + m)) - 1
    objs = torch.from_numpy(host).to(gpu)
    stripes = batch.stripe_buffer(B, k, m, bs, device=gpu)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    for call in range(3):
        masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), m)) for _ in range(B)]
        if call == 2:
            masks[:6] = masks[6:12]  # cached patterns mixed with new ones
        out = torch.zeros_like(objs)
        codec.decode(stripes, n, masks, out)
        dest = [rng.randrange(k + m) for _ in range(B)]
        rmasks = [full & ~(1 << d) & ~(1 << ((d + 1 + o) % (k + m))) for o, d in enumerate(dest)]
        rec = torch.zeros((B, stripes.shape[2]), dtype=torch.uint8, device=gpu)
        codec.reconstruct(stripes, n, rmasks, dest, rec)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :n].cpu(), torch.from_numpy(host[:, :n])), f"call {call}"
        got = rec.cpu().numpy()
        want = stripes.cpu().numpy()
        for o in range(B):
            assert got[o, :80 + bs].tobytes() == want[o, dest[o], :80 + bs].tobytes(), (call, o)
    # and the parity itself is the oracle's
    frags = oracle.encode(k, m, host[0, :n].tobytes())
    assert stripes[0, k, :80 + bs].cpu().numpy().tobytes() == frags[k]


@pytest.mark.parametrize("ec_type,k,m,n", [("amd_rs_vand", 10, 4, 4 << 20),
                                           ("amd_rs_vand", 6, 2, 65536 + 10),
                                           ("amd_rs_vand", 12, 4, 999999),
                                           ("isa_l_rs_cauchy", 12, 4, 1 << 20),
                                           ("amd_rs_vand", 4, 2, 17)])
@pytest.mark.parametrize("path", ["direct", "staged", "staged_out"])
@pytest.mark.parametrize("crc", [False, True])
def test_host_resident_encode_decode_reconstruct(gpu, oracle, monkeypatch, ec_type, k, m, n,
                                                 path, crc):
    """ecamd_{encode,decode,reconstruct}_host_batch: pinned host in and out,
    against the oracle (encode, reconstruct) and the objects (decode).  Paths:
    kernels on the mapped host arrays (default), the copy-engine pipeline with
    kernels writing host outputs, and the pipeline with D2H-staged outputs.
    crc: inline_crc32 headers (the parity CRC fused into the encode launch,
    its finishing pass reading the payloads it wrote, wherever they are)."""
    import torch
    from pyeclib_amd import batch
    if path != "direct":
        monkeypatch.setenv("ECAMD_HOST_STAGED", "1")
    if path == "staged_out":
        monkeypatch.setenv("ECAMD_HOST_STAGED_OUT", "1")
    B = 13
    host, masks, dests = _inputs(B, n, k, m, m, 97 + n)
    codec = batch.BatchCodec(k, m, ec_type=ec_type, inline_crc32=crc)
    ct = oracle.CHKSUM_CRC32 if crc else oracle.CHKSUM_NONE
    bs = codec.blocksize(n)
    fs = batch.frag_stride(bs)
    fl = 80 + bs
    pinned = torch.from_numpy(host).pin_memory()
    par = torch.zeros((B, m, fs), dtype=torch.uint8).pin_memory()
    codec.encode_host(pinned, n, par)
    want = []
    for o in range(B):
        data = host[o, :n].tobytes()
        if codec.w == 8:
            w = oracle.isal_encode(oracle.ISAL_CAUCHY, k, m, data, ct=ct)
        else:
            w = oracle.encode(k, m, data, ct=ct)
        want.append(w)
        for p in range(m):
            assert par[o, p, :fl].numpy().tobytes() == w[k + p], (o, p)
    # the k fragments each object's decode reads (first k available), compact
    hfr = torch.zeros((B, k, fs), dtype=torch.uint8).pin_memory()
    for o in range(B):
        idx = [i for i in range(k + m) if masks[o] >> i & 1][:k]
        for c, i in enumerate(idx):
            hfr[o, c, :fl] = torch.frombuffer(bytearray(want[o][i]), dtype=torch.uint8)
    out = torch.zeros((B, host.shape[1]), dtype=torch.uint8).pin_memory()
    codec.decode_host(hfr, n, masks, out)
    assert torch.equal(out[:, :n], pinned[:, :n])
    # reconstruct a fragment each object lost
    full = (1 << (k + m)) - 1
    dest = [next(i for i in range(k + m) if not masks[o] >> i & 1) for o in range(B)]
    rec = torch.zeros((B, fs), dtype=torch.uint8).pin_memory()
    codec.reconstruct_host(hfr, n, masks, dest, rec)
    for o in range(B):
        assert rec[o, :fl].numpy().tobytes() == want[o][dest[o]], o
    assert full  # (all masks had m erasures)


def test_swift_mix_reduced_host_stream(gpu, oracle):
    """configs[4] shape at a reduced count: k in {6,10,12} x m in {2,4},
    objects 64 KiB .. 16 MiB (plus ragged sizes), streamed host -> host
    through encode_host and read back through decode_host; parity checked
    against the oracle, objects round-tripped."""
    import torch
    from pyeclib_amd import batch
    rng = random.Random(2026)
    for k, m in [(6, 2), (10, 4), (12, 4), (12, 2)]:
        codec = batch.BatchCodec(k, m)
        for n in (64 << 10, (256 << 10) + 3, 1 << 20, (4 << 20) - 2, 16 << 20):
            B = 2 if n >= (4 << 20) - 2 else 4
            host, _, _ = _inputs(B, n, k, m, 0, n + k)
            bs = codec.blocksize(n)
            fs = batch.frag_stride(bs)
            fl = 80 + bs
            pinned = torch.from_numpy(host).pin_memory()
            par = torch.zeros((B, m, fs), dtype=torch.uint8).pin_memory()
            codec.encode_host(pinned, n, par)
            masks, hfr = [], torch.zeros((B, k, fs), dtype=torch.uint8).pin_memory()
            for o in range(B):
                frags = oracle.encode(k, m, host[o, :n].tobytes())
                for p in range(m):
                    assert par[o, p, :fl].numpy().tobytes() == frags[k + p], (k, m, n, o, p)
                lost = set(rng.sample(range(k + m), m))
                idx = [i for i in range(k + m) if i not in lost][:k]
                masks.append(sum(1 << i for i in range(k + m) if i not in lost))
                for c, i in enumerate(idx):
                    hfr[o, c, :fl] = torch.frombuffer(bytearray(frags[i]), dtype=torch.uint8)
            out = torch.zeros((B, host.shape[1]), dtype=torch.uint8).pin_memory()
            codec.decode_host(hfr, n, masks, out)
            assert torch.equal(out[:, :n], pinned[:, :n]), (k, m, n)


def test_swift_mix_tool_verifies(gpu):
    """tools/swift_mix.py (configs[4] driver) on a reduced mix: its own
    verification (parity vs the oracle, every decoded object) must pass."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "swift_mix.py"),
                        "--group-mib", "8", "--passes", "1", "--schemes", "6:2,12:4",
                        "--sizes", "65536,1048576,16777216"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["verified"] is True
    assert out["encode_GiBps"] > 0 and out["decode_GiBps"] > 0
    assert len(out["groups"]) == 6
