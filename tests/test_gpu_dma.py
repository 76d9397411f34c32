"""The loader / consumer kernels (encode_dma_kernel, decode_dma_kernel,
encode_crc_dma_kernel: 16 KiB items, LDS-DMA ring) against the CPU oracle.

The launchers take them when a batch has at least one 16 KiB interior item
per CU (256 on MI355X), so every case here is sized past that line at a few
MiB per object or less: ragged object lengths, k from 4 to 28, m = 1 .. 6
(parity rows 1 .. 4 per pass, and the two-pass m > 4 CRC encode), GF(2^16)
and GF(2^8), parity-only and full-stripe encode, inline_crc32 headers.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

MIN_ITEMS = 256  # 16 KiB interior items per launch for the DMA kernels (one per CU)


def _dma_items(codec, k, n, n_obj):
    bs = codec.blocksize(n)
    room = min(n - (k - 1) * bs, bs)  # last_room (ec_kernels_impl.hpp)
    return max(room, 0) // 16384 * n_obj


@pytest.mark.parametrize("ec_type,k,m,n,n_obj", [
    ("amd_rs_vand", 10, 4, 1 << 20, 48),
    ("amd_rs_vand", 4, 2, 512 * 1024, 40),
    ("amd_rs_vand", 6, 3, (1 << 20) + 3, 40),
    ("amd_rs_vand", 16, 4, 1 << 20, 64),
    ("amd_rs_vand", 28, 4, 2 << 20, 64),
    ("isa_l_rs_cauchy", 12, 4, (2 << 20) + 5, 32),
    ("isa_l_rs_vand", 8, 1, 1 << 20, 32),
    # many small objects: one 16 KiB item each, plus an edge tile
    ("amd_rs_vand", 10, 4, 200 * 1024 + 6, 600),
    ("amd_rs_vand", 30, 2, 2 << 20, 64),
])
def test_dma_encode_decode(gpu, ec_type, k, m, n, n_obj):
    """Full-stripe encode (DATA variant), parity-only encode and decode with
    min(m, 4) random erasures per object, every object against the oracle."""
    import torch
    import bench
    from pyeclib_amd import batch
    from test_gpu_configs import _device_batch
    codec = batch.BatchCodec(k, m, ec_type=ec_type)
    assert _dma_items(codec, k, n, n_obj) >= MIN_ITEMS, "case must reach the DMA kernels"
    args, host, masks, dests, gf, g2 = _device_batch(gpu, ec_type, k, m, n, n_obj, "decode",
                                                     erasures=min(m, 4))
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=n_obj)
    assert bad == []
    # parity-only launch (no data fragments): the same parity payloads
    bs = codec.blocksize(n)
    objs = torch.from_numpy(host).to(gpu)
    stripes = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(objs, n, parity=stripes[:, k:])
    torch.cuda.synchronize()
    par = stripes[:, k:, 80:80 + bs].cpu().numpy()
    assert np.array_equal(par, gf[:, k:, 80:80 + bs])


@pytest.mark.parametrize("ec_type,k,m,n,n_obj", [
    ("amd_rs_vand", 10, 4, 1 << 20, 48),
    ("amd_rs_vand", 8, 6, 1 << 20, 64),        # two parity passes (rows 0-3, 4-5)
    ("isa_l_rs_vand", 10, 4, (1 << 20) + 1, 48),
    ("amd_rs_vand", 5, 3, 777777, 64),
    ("amd_rs_vand", 10, 4, 200 * 1024 + 6, 600),  # runs end at every object
])
def test_dma_inline_crc32(oracle, gpu, ec_type, k, m, n, n_obj):
    """The fused-CRC loader / consumer encode: every header of a sample of
    objects (first, last, and every fifth) equals the oracle's."""
    import torch
    from pyeclib_amd import batch
    codec = batch.BatchCodec(k, m, inline_crc32=True, ec_type=ec_type)
    assert _dma_items(codec, k, n, n_obj) >= MIN_ITEMS, "case must reach the DMA kernels"
    bs = codec.blocksize(n)
    stride = (n + 15) // 16 * 16
    host = torch.from_numpy(np.random.default_rng(n + k).integers(0, 256, (n_obj, stride),
                                                                  dtype=np.uint8))
    frags = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(host.to(gpu), n, parity=frags[:, k:], data=frags[:, :k])
    par_only = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(host.to(gpu), n, parity=par_only[:, k:])
    torch.cuda.synchronize()
    got = frags.cpu().numpy()
    got_par = par_only[:, k:].cpu().numpy()
    for o in sorted(set(range(0, n_obj, 5)) | {n_obj - 1}):
        data = host[o, :n].numpy().tobytes()
        if codec.w == 8:
            want = oracle.isal_encode(4, k, m, data, ct=oracle.CHKSUM_CRC32)
        else:
            want = oracle.encode(k, m, data, ct=oracle.CHKSUM_CRC32)
        for i in range(k + m):
            assert got[o, i, :80 + bs].tobytes() == want[i], f"obj {o} fragment {i}"
        for p in range(m):
            assert got_par[o, p, :80 + bs].tobytes() == want[k + p], f"obj {o} parity {p}"


@pytest.mark.parametrize("ec_type,k,m,n,n_obj", [
    ("amd_rs_vand", 10, 4, 1 << 20, 48),
    ("amd_rs_vand", 4, 2, 512 * 1024, 40),
    ("isa_l_rs_cauchy", 12, 4, (2 << 20) + 5, 32),
    ("amd_rs_vand", 9, 3, 999999, 64),
])
def test_reconstruct_dma_sized_batches(gpu, ec_type, k, m, n, n_obj):
    """Reconstruct (one random fragment per object, header included) at the
    batch sizes that take the loader / consumer kernels for encode and decode
    -- reconstruct itself keeps the stream kernel, which measured faster --
    every object against the oracle."""
    import bench
    from pyeclib_amd import batch
    from test_gpu_configs import _device_batch
    codec = batch.BatchCodec(k, m, ec_type=ec_type)
    assert codec.blocksize(n) // 16384 * n_obj >= MIN_ITEMS, "case must reach the DMA kernels"
    args, host, masks, dests, gf, g2 = _device_batch(gpu, ec_type, k, m, n, n_obj, "reconstruct")
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=n_obj)
    assert bad == []
