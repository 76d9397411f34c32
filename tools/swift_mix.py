#!/usr/bin/env python3
"""BASELINE configs[4]: Swift-style mix, streaming encode from host memory.

Schemes k in {6, 10, 12} x m in {2, 4} (rs_vand, GF(2^16)), object sizes
64 KiB, 256 KiB, 1 MiB, 4 MiB and 16 MiB.  Every (scheme, size) group holds
about --group-mib of objects in pinned host memory; one pass encodes every
group through ecamd_encode_host_batch (H2D, kernel and D2H pipelined over
two streams; the data fragments are the host slices themselves, so only
parity fragments come back), exactly the data flow of a Swift proxy that
receives objects from a socket and writes fragments to disk.

One process per GPU (torchrun): every rank streams the whole mix (weak
scaling, no collective on the data path).  Rank 0 prints one JSON line with
the aggregate host-to-host GiB/s (object bytes), the per-group rates and,
for contrast, the device-resident rate of the same groups.

  python tools/swift_mix.py [--group-mib 64] [--passes 3]
  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/swift_mix.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCHEMES = [(6, 2), (6, 4), (10, 2), (10, 4), (12, 2), (12, 4)]
SIZES = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--group-mib", type=int, default=64)
    ap.add_argument("--passes", type=int, default=3)
    args = ap.parse_args()

    from pyeclib_amd import batch, shard
    world, rank, local = shard.init("nccl")
    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rng = np.random.Generator(np.random.PCG64(20261015 + rank))

    groups = []
    for k, m in SCHEMES:
        codec = batch.BatchCodec(k, m)
        for size in SIZES:
            n = max(1, (args.group_mib << 20) // size)
            stride = (size + 255) // 256 * 256
            bs = batch.blocksize(k, size)
            fs = batch.frag_stride(bs)
            objs = torch.from_numpy(rng.integers(0, 256, (n, stride), dtype=np.uint8)).pin_memory()
            parity = torch.zeros((n, m, fs), dtype=torch.uint8).pin_memory()
            groups.append({"k": k, "m": m, "size": size, "n": n, "codec": codec, "objs": objs,
                           "parity": parity, "bs": bs})
    total = sum(g["n"] * g["size"] for g in groups)

    # warm-up (instance tables, staging buffers), then timed passes
    for g in groups:
        g["codec"].encode_host(g["objs"], g["size"], g["parity"])
    shard.barrier()
    t0 = time.perf_counter()
    for _ in range(args.passes):
        for g in groups:
            t = time.perf_counter()
            g["codec"].encode_host(g["objs"], g["size"], g["parity"])
            g.setdefault("t", []).append(time.perf_counter() - t)
    shard.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, device=dev) / args.passes

    # device-resident reference for the same groups
    t_dev = 0.0
    for g in groups:
        d_objs = g["objs"].to(dev)
        d_par = torch.zeros((g["n"], g["m"], g["parity"].shape[2]), dtype=torch.uint8,
                            device=dev)
        g["codec"].encode(d_objs, g["size"], parity=d_par)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.passes):
            g["codec"].encode(d_objs, g["size"], parity=d_par)
        torch.cuda.synchronize()
        t_dev += (time.perf_counter() - t) / args.passes
        del d_objs, d_par

    if rank == 0:
        per_group = [{"k": g["k"], "m": g["m"], "object_bytes": g["size"], "objects": g["n"],
                      "GiBps": round(g["n"] * g["size"] / min(g["t"]) / 2**30, 2)} for g in groups]
        print(json.dumps({
            "metric": "Swift-mix streaming encode GiB/s incl. pinned H2D/D2H (object bytes)",
            "value": round(world * total / elapsed / 2**30, 3),
            "unit": "GiB/s", "n_gpus": world, "passes": args.passes,
            "higher_is_better": True, "scaling": "weak",
            "config": {"schemes": SCHEMES, "object_sizes": SIZES,
                       "group_bytes": args.group_mib << 20, "bytes_per_rank": total,
                       "ec_type": "amd_rs_vand"},
            "device_resident_GiBps_per_gpu": round(total / t_dev / 2**30, 3),
            "groups": per_group,
        }), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
