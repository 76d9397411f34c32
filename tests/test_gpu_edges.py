"""Launch shapes around the edge items, on the GPU through the C ABI.

Round 3 runs a launch's edge items (payload tails, zero padding, headers) in
blocks of their own, at most one per CU, ahead of the interior blocks
(ec_kernels_impl.hpp launch_edges_apart).  These batches have more edge items
than the GPU has CUs (so each edge block walks several), objects with no
interior tile at all (the launch falls back to every block taking its share
of the edges), and the round-2 form forced with ECAMD_EDGE_BLOCKS=0 -- each
checked object by object against the CPU oracle (bench.oracle_pass: every
fragment, header included, and every decoded object or rebuilt fragment).
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


@pytest.mark.parametrize("ec_type,k,m,n,B,second,edge_blocks", [
    ("amd_rs_vand", 10, 4, 102437, 600, "decode", None),
    ("amd_rs_vand", 10, 4, 102437, 600, "reconstruct", None),
    ("isa_l_rs_cauchy", 12, 4, 50000, 700, "reconstruct", None),
    ("isa_l_rs_vand", 6, 3, 40001, 520, "decode", None),
    ("amd_rs_vand", 8, 3, 3000, 1000, "decode", None),   # no interior tile at all
    ("amd_rs_vand", 10, 4, 102437, 600, "decode", "0"),  # round-2 form
])
def test_many_edge_items(gpu, monkeypatch, ec_type, k, m, n, B, second, edge_blocks):
    import bench
    from test_gpu_configs import _device_batch
    if edge_blocks is not None:
        monkeypatch.setenv("ECAMD_EDGE_BLOCKS", edge_blocks)
    args, host, masks, dests, gf, g2 = _device_batch(gpu, ec_type, k, m, n, B, second,
                                                     erasures=min(4, m), seed=n + B)
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=B)
    assert bad == []


@pytest.mark.parametrize("edge_blocks", [None, "0"])
def test_inline_crc32_parity_only_many_objects(gpu, oracle, monkeypatch, edge_blocks):
    """The bench's --inline-crc32 encode (parity fragments only, CRC fused
    into the encode launch) with 600 objects: more edge items than CUs and
    many block ranges cut at object boundaries.  Every parity fragment,
    header included, equals the oracle's."""
    import torch
    from pyeclib_amd import batch
    if edge_blocks is not None:
        monkeypatch.setenv("ECAMD_EDGE_BLOCKS", edge_blocks)
    k, m, n, B = 10, 4, 102437, 600
    codec = batch.BatchCodec(k, m, inline_crc32=True)
    bs = codec.blocksize(n)
    stride = (n + 15) // 16 * 16
    host = np.random.default_rng(99).integers(0, 256, (B, stride), dtype=np.uint8)
    stripes = batch.stripe_buffer(B, k, m, bs, device=gpu)
    codec.encode(torch.from_numpy(host).to(gpu), n, parity=stripes[:, k:])
    torch.cuda.synchronize()
    got = stripes[:, k:, :80 + bs].cpu().numpy()
    for o in range(B):
        want = oracle.encode(k, m, host[o, :n].tobytes(), ct=oracle.CHKSUM_CRC32)
        for r in range(m):
            assert got[o, r].tobytes() == want[k + r], f"object {o} parity {r}"
