#!/usr/bin/env python3
"""Host-resident pipeline tuning: pinned H2D/D2H link rates beside
encode_host / decode_host under the runtime's pipeline knobs.

Each positional argument is one variant ("base" or VAR=VAL[,VAR=VAL...] of
ECAMD_HOST_STAGED (copy-engine pipeline instead of kernels on the mapped
host arrays), ECAMD_HOST_CHUNK_MB, ECAMD_HOST_STREAMS, ECAMD_HOST_STAGED_OUT);
the workload is bench.py's (k=10 m=4, 256 x 4 MiB,
4 erasures per object).  Outputs are checked against the device-resident
path.  Prints GiB/s of object bytes per variant (median of --reps).
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
KEYS = ["ECAMD_HOST_CHUNK_MB", "ECAMD_HOST_STREAMS", "ECAMD_HOST_STAGED_OUT", "ECAMD_HOST_STAGED"]


def variant_env(text):
    if text == "base":
        return {}
    return dict(part.split("=", 1) for part in text.split(","))


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()

    import torch
    from pyeclib_amd import batch

    k, m, n, B = 10, 4, 4 * 1024 * 1024, args.batch
    dev = torch.device("cuda:0")
    bs = batch.blocksize(k, n)
    fs = batch.frag_stride(bs)
    rng = np.random.default_rng(5)
    host = torch.from_numpy(rng.integers(0, 256, size=(B, n), dtype=np.uint8)).pin_memory()
    codec = batch.BatchCodec(k, m)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    codec.encode(host.to(dev), n, parity=stripes[:, k:], data=stripes[:, :k])
    full = (1 << (k + m)) - 1
    masks = [full & ~int(sum(1 << int(i) for i in rng.choice(k + m, 4, replace=False)))
             for _ in range(B)]
    idx = torch.tensor([[i for i in range(k + m) if mk >> i & 1][:k] for mk in masks], device=dev)
    hfr = stripes[torch.arange(B, device=dev)[:, None], idx].cpu().pin_memory()
    ref_par = stripes[:, k:, :80 + bs].cpu()
    hpar = torch.zeros((B, m, fs), dtype=torch.uint8).pin_memory()
    hout = torch.zeros((B, n), dtype=torch.uint8).pin_memory()

    # the link alone, as torch moves it (one copy of the whole batch)
    dbuf = torch.empty_like(host, device=dev)
    for name, (dst, src) in (("h2d", (dbuf, host)), ("d2h", (host, dbuf))):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        print(f"link {name}: {3 * host.numel() / (time.perf_counter() - t0) / 2**30:.2f} GiB/s")
    # both directions at once (two streams)
    dbuf2 = torch.empty_like(host, device=dev)
    hsink = torch.empty_like(host).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        with torch.cuda.stream(s1):
            dbuf.copy_(host, non_blocking=True)
        with torch.cuda.stream(s2):
            hsink.copy_(dbuf2, non_blocking=True)
    torch.cuda.synchronize()
    print(f"link h2d+d2h concurrent: {3 * host.numel() / (time.perf_counter() - t0) / 2**30:.2f} "
          "GiB/s each way")
    del dbuf, dbuf2, hsink

    print(f"{'variant':<52} {'enc GiB/s':>10} {'dec GiB/s':>10}")
    for v in args.variants:
        env = variant_env(v)
        for key in KEYS:
            os.environ.pop(key, None)
        os.environ.update(env)
        codec = batch.BatchCodec(k, m)  # the knobs are read when an instance is created
        te, td = [], []
        for r in range(args.reps + 1):
            hpar.zero_()
            t0 = time.perf_counter()
            codec.encode_host(host, n, hpar)
            t1 = time.perf_counter()
            codec.decode_host(hfr, n, masks, hout)
            t2 = time.perf_counter()
            if r == 0:
                assert torch.equal(hpar[:, :, :80 + bs], ref_par), f"{v}: encode_host differs"
                assert torch.equal(hout, host), f"{v}: decode_host differs"
                hout.zero_()
                continue
            te.append(t1 - t0)
            td.append(t2 - t1)
        print(f"{v:<52} {B * n / statistics.median(te) / 2**30:10.2f} "
              f"{B * n / statistics.median(td) / 2**30:10.2f}", flush=True)
    for key in KEYS:
        os.environ.pop(key, None)


if __name__ == "__main__":
    main()
