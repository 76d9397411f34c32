#!/usr/bin/env python3
"""Debug aid: decode a small batch under the current ECAMD_* environment and
report where the output differs from the objects (slice, offset in slice,
offset mod 1024 / 16)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pyeclib_amd import batch
    k, m, n, B = 10, 4, 4 * 1024 * 1024, int(os.environ.get("DIFF_B", "8"))
    dev = torch.device("cuda:0")
    bs = batch.blocksize(k, n)
    stride = (n + 255) // 256 * 256
    rng = np.random.default_rng(3)
    objs = torch.from_numpy(rng.integers(0, 256, size=(B, stride), dtype=np.uint8)).to(dev)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    codec = batch.BatchCodec(k, m)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    full = (1 << (k + m)) - 1
    masks = [full & ~int(sum(1 << int(i) for i in rng.choice(k + m, 4, replace=False)))
             for _ in range(B)]
    out = torch.zeros_like(objs)
    codec.decode(stripes, n, masks, out)
    torch.cuda.synchronize()
    a = out[:, :n].cpu().numpy()
    b = objs[:, :n].cpu().numpy()
    for o in range(B):
        bad = np.nonzero(a[o] != b[o])[0]
        lost = [i for i in range(k + m) if not masks[o] >> i & 1]
        if len(bad) == 0:
            print(f"obj {o}: ok (lost {lost})")
            continue
        sl = bad // bs
        pos = bad - sl * bs
        print(f"obj {o}: {len(bad)} bad bytes, lost {lost}, slices {sorted(set(sl.tolist()))}")
        for s in sorted(set(sl.tolist()))[:4]:
            p = pos[sl == s]
            print(f"   slice {s}: n={len(p)} first {p[:6].tolist()} mod1024 {sorted(set((p % 1024).tolist()))[:12]}"
                  f" obj%16 {sorted(set(((s * bs + p) % 16).tolist()))}"
                  f" range [{int(p.min())}, {int(p.max())}] 16K-items {sorted(set((p // 16384).tolist()))[:12]}"
                  f" KiB-in-item {sorted(set(((p % 16384) // 1024).tolist()))}")


if __name__ == "__main__":
    main()
