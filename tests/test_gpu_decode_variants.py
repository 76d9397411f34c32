"""GPU decode object stores: the streaming decode kernel's slice stores (every
slice alignment: 16-B aligned, 8 mod 16, odd for GF(2^8)), its dropped stores
(parity inputs, rows past the missing count) and the edge items must rebuild
the objects bit-exactly and write nothing outside [0, obj_len) of each
object's output row.

Encode parity itself is pinned against the oracle in test_gpu_parity.py;
here the decoded bytes are compared with the objects.
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [
    ("amd_rs_vand", 10, 4, 4 * 1024 * 1024),     # bench shape: slices 8 mod 16
    ("amd_rs_vand", 10, 4, 1 << 20),
    ("amd_rs_vand", 10, 4, 4 * 1024 * 1024 // 7),
    ("amd_rs_vand", 10, 4, 10 * 4096 * 3),        # slices 16-B aligned
    ("amd_rs_vand", 12, 4, 999999),
    ("amd_rs_vand", 6, 3, 3 * 1024 * 1024 + 22),
    ("amd_rs_vand", 16, 4, 2 * 1024 * 1024 + 6),
    ("amd_rs_vand", 4, 2, 100001),
    ("isa_l_rs_vand", 10, 4, 4 * 1024 * 1024 + 3),  # GF(2^8): odd slice offsets
    ("isa_l_rs_cauchy", 12, 4, 1 << 20),
    ("isa_l_rs_cauchy", 8, 3, 777777),
]


@pytest.mark.parametrize("ec_type,k,m,obj_len", CASES)
def test_decode_object_stores(gpu, ec_type, k, m, obj_len):
    import torch
    from pyeclib_amd import batch
    n_obj = 6
    codec = batch.BatchCodec(k, m, ec_type=ec_type)
    bs = codec.blocksize(obj_len)
    stride = (obj_len + 255) // 256 * 256 + 256
    gen = torch.Generator(device=gpu).manual_seed(obj_len + k)
    objs = torch.randint(0, 256, (n_obj, stride), dtype=torch.uint8, device=gpu, generator=gen)
    stripes = batch.stripe_buffer(n_obj, k, m, bs, device=gpu)
    codec.encode(objs, obj_len, parity=stripes[:, k:], data=stripes[:, :k])
    rng = random.Random(obj_len * 7 + k)
    full = (1 << (k + m)) - 1
    # o % (m + 1) erasures: every count from none to m, random positions
    masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), o % (m + 1)))
             for o in range(n_obj)]
    out = torch.full((n_obj, stride), 0xA5, dtype=torch.uint8, device=gpu)
    codec.decode(stripes, obj_len, masks, out)
    torch.cuda.synchronize()
    for o in range(n_obj):
        assert torch.equal(out[o, :obj_len], objs[o, :obj_len]), f"object {o} mask {masks[o]:x}"
        tail = out[o, obj_len:].cpu().numpy()
        assert np.all(tail == 0xA5), f"object {o}: bytes written past obj_len"
