#!/usr/bin/env python3
"""Where a decode with new erasure masks spends its time (dev tool): the host
call (enqueue) time and the GPU event span, for masks drawn anew per call
(new patterns: decode rows and table sets built on the host), masks
reshuffled per call from 50 patterns already in the device pool (new
descriptors only), and the same masks repeated (cached descriptors), at
bench.py's workload (k=10 m=4, 256 x 4 MiB)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pyeclib_amd import batch
    k, m, n, B = 10, 4, 4 << 20, 256
    dev = torch.device("cuda:0")
    bs = batch.blocksize(k, n)
    objs = torch.randint(0, 256, (B, n), dtype=torch.uint8, device=dev)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    codec = batch.BatchCodec(k, m)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    out = torch.zeros_like(objs)
    full = (1 << (k + m)) - 1

    def masks(seed):
        rng = np.random.default_rng(seed)
        return [full & ~int(sum(1 << int(i) for i in rng.choice(k + m, 4, replace=False)))
                for _ in range(B)]

    pool = masks(3)[:50]  # 50 patterns, cached in the device pool after the first call

    def shuffled(seed):
        rng = np.random.default_rng(seed)
        return [pool[int(i)] for i in rng.integers(0, len(pool), B)]

    for label, seeds, gen in (("fresh", range(100, 112), masks),
                              ("reshuffled", range(200, 212), shuffled),
                              ("repeat", [7] * 12, masks)):
        host_us, span_us = [], []
        for s in seeds:
            mk = gen(s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            codec.decode(stripes, n, mk, out)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            host_us.append((t1 - t0) * 1e6)
            span_us.append(e0.elapsed_time(e1) * 1e3)
        print(f"{label:7s} host call median {np.median(host_us[2:]):8.1f} us  "
              f"event span median {np.median(span_us[2:]):8.1f} us  (first {host_us[0]:.0f} / {span_us[0]:.0f})")
        assert torch.equal(out, objs)
    # back to back (bench.py decode_fresh_ms's shape): 16 calls with no
    # synchronisation between them, masks new every call vs repeated
    for label, gen in (("steady-fresh", lambda i: masks(300 + i)), ("steady-repeat", lambda i: masks(7))):
        mks = [gen(i) for i in range(16)]
        for rep in range(2):  # the first pass brings any new patterns into the pool
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            for mk in mks:
                codec.decode(stripes, n, mk, out)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
        print(f"{label:13s} per call: host {(t1 - t0) * 1e6 / len(mks):8.1f} us  "
              f"event span {e0.elapsed_time(e1) * 1e3 / len(mks):8.1f} us")
        assert torch.equal(out, objs)


if __name__ == "__main__":
    main()
