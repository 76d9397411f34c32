#!/usr/bin/env python3
"""BASELINE configs[4]: Swift-style mix, streaming encode AND decode from host memory.

Schemes k in {6, 10, 12} x m in {2, 4} (rs_vand, GF(2^16)), object sizes
64 KiB, 256 KiB, 1 MiB, 4 MiB and 16 MiB.  Every (scheme, size) group holds
about --group-mib of objects in pinned host memory.  One pass:
  * write path: every group through ecamd_encode_host_batch (H2D, kernel and
    D2H pipelined over three streams; the data fragments are the host slices
    themselves, so only parity fragments come back) -- a Swift proxy PUT:
    object from a socket, fragments to the object servers;
  * read path: every group through ecamd_decode_host_batch from the k
    fragments a GET would fetch (m random fragments lost per object, the
    first k survivors handed over, as pyeclib's decode uses them) -- a
    Swift proxy GET.
Rates are object bytes / wall time of the pass (host to host).

One process per GPU (every rank streams the whole mix; weak scaling, no
collective on the data path).  `--gpus N` without a launcher starts
torch.distributed.run itself as a child (as bench.py does).  Rank 0 prints
one JSON line with the aggregate rates, per-group rates and, for contrast,
the device-resident encode rate of the same groups.

Verification (every rank, outside the timed passes): in every group, EVERY
object's parity fragments (headers included) are compared with the
device-resident batch encode of the same objects (the kernel path bench.py
and tests/ check against the CPU oracle), and EVERY decoded object with the
original bytes; any mismatch exits non-zero.  "verified": true in the JSON
line.  Each rank's CPUs are bound to its GPU's NUMA node before the GPU is
touched (pyeclib_amd/placement.py), so its pinned buffers are first touched
there; the bookkeeping collectives run on gloo (pyeclib_amd/shard.py).

  python tools/swift_mix.py [--group-mib 64] [--passes 3] [--gpus N]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCHEMES = [(6, 2), (6, 4), (10, 2), (10, 4), (12, 2), (12, 4)]
SIZES = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20]


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--group-mib", type=int, default=64)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--no-numa", action="store_true",
                    help="do not bind each rank's CPUs to its GPU's NUMA node")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (exercises the N-rank path on one GPU)")
    ap.add_argument("--schemes", default=None, help="e.g. 6:2,10:4 (default: all six)")
    ap.add_argument("--sizes", default=None, help="e.g. 65536,1048576 (default: all five)")
    return ap.parse_args(argv)


def relaunch(args) -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


def build_groups(args, rank, batch, torch):
    schemes = SCHEMES if not args.schemes else [
        tuple(int(v) for v in s.split(":")) for s in args.schemes.split(",")]
    sizes = SIZES if not args.sizes else [int(v) for v in args.sizes.split(",")]
    rng = np.random.Generator(np.random.PCG64(20261015 + rank))
    pick = random.Random(77 + rank)
    groups = []
    for k, m in schemes:
        codec = batch.BatchCodec(k, m)
        for size in sizes:
            n = max(1, (args.group_mib << 20) // size)
            stride = (size + 255) // 256 * 256
            bs = batch.blocksize(k, size)
            fs = batch.frag_stride(bs)
            objs = torch.from_numpy(rng.integers(0, 256, (n, stride), dtype=np.uint8)).pin_memory()
            parity = torch.zeros((n, m, fs), dtype=torch.uint8).pin_memory()
            masks = []
            for _ in range(n):
                lost = set(pick.sample(range(k + m), m))
                masks.append(sum(1 << i for i in range(k + m) if i not in lost))
            groups.append({"k": k, "m": m, "size": size, "n": n, "codec": codec, "objs": objs,
                           "parity": parity, "bs": bs, "fs": fs, "masks": masks,
                           "frags": torch.zeros((n, k, fs), dtype=torch.uint8).pin_memory(),
                           "out": torch.zeros((n, stride), dtype=torch.uint8).pin_memory()})
    return groups


def fill_read_fragments(g, torch):
    """The k fragments each object's GET hands to decode (first k available,
    ascending), from the host objects (data) and the encoded parity."""
    k, bs, fl = g["k"], g["bs"], 80 + g["bs"]
    from pyeclib_amd import _native  # noqa: F401 (library loaded)
    objs = g["objs"].numpy()
    par = g["parity"].numpy()
    fr = g["frags"].numpy()
    for o in range(g["n"]):
        idx = [i for i in range(k + g["m"]) if g["masks"][o] >> i & 1][:k]
        for c, i in enumerate(idx):
            if i < k:
                # data fragment = header (same fields as parity's, idx i) + padded slice
                hdr = data_header(par[o, 0, :80], i)
                fr[o, c, :80] = hdr
                sl = objs[o, i * bs:min((i + 1) * bs, g["size"])]
                fr[o, c, 80:80 + len(sl)] = sl
                fr[o, c, 80 + len(sl):fl] = 0
            else:
                fr[o, c, :fl] = par[o, i - k, :fl]


def data_header(parity0_hdr, idx):
    """Header of data fragment idx, from parity fragment 0's header (the
    fields differ only in idx and the metadata checksum)."""
    import zlib
    h = bytearray(parity0_hdr.tobytes())
    h[0:4] = idx.to_bytes(4, "little")
    h[67:71] = zlib.crc32(bytes(h[:59])).to_bytes(4, "little")
    return np.frombuffer(bytes(h), dtype=np.uint8)


def verify(groups, dev_parity):
    """Host-resident parity (headers included) == the device-resident
    encode's, for every object; decoded objects == the originals."""
    bad = []
    for g, dp in zip(groups, dev_parity):
        fl = 80 + g["bs"]
        if not np.array_equal(g["parity"][:, :, :fl].numpy(), dp[:, :, :fl]):
            bad.append((g["k"], g["m"], g["size"], "parity"))
        if not np.array_equal(g["out"][:, :g["size"]].numpy(), g["objs"][:, :g["size"]].numpy()):
            bad.append((g["k"], g["m"], g["size"], "decode"))
    return bad


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    from pyeclib_amd import placement, shard
    world, rank, local = shard.rank_info()
    dev_idx = shard.device_index(local, args.same_device)
    numa = {"bound": False, "reason": "--no-numa"} if args.no_numa else \
        placement.bind_to_gpu_numa(dev_idx)
    import torch
    from pyeclib_amd import batch
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    shard.init("gloo")

    groups = build_groups(args, rank, batch, torch)
    total = sum(g["n"] * g["size"] for g in groups)

    # warm-up (instance tables, staging buffers), read-path inputs, then timed passes
    for g in groups:
        g["codec"].encode_host(g["objs"], g["size"], g["parity"])
        fill_read_fragments(g, torch)
        g["codec"].decode_host(g["frags"], g["size"], g["masks"], g["out"])
    shard.barrier()
    t0 = time.perf_counter()
    for _ in range(args.passes):
        for g in groups:
            t = time.perf_counter()
            g["codec"].encode_host(g["objs"], g["size"], g["parity"])
            g.setdefault("te", []).append(time.perf_counter() - t)
    shard.barrier()
    t_write = shard.max_over_ranks(time.perf_counter() - t0) / args.passes
    for g in groups:
        g["out"].zero_()
    shard.barrier()
    t0 = time.perf_counter()
    for _ in range(args.passes):
        for g in groups:
            t = time.perf_counter()
            g["codec"].decode_host(g["frags"], g["size"], g["masks"], g["out"])
            g.setdefault("td", []).append(time.perf_counter() - t)
    shard.barrier()
    t_read = shard.max_over_ranks(time.perf_counter() - t0) / args.passes

    # device-resident encode of the same groups: the reference rate, and the
    # parity the host-resident path must equal
    t_dev = 0.0
    dev_parity = []
    for g in groups:
        d_objs = g["objs"].to(dev)
        d_par = torch.zeros((g["n"], g["m"], g["fs"]), dtype=torch.uint8, device=dev)
        g["codec"].encode(d_objs, g["size"], parity=d_par)
        torch.cuda.synchronize()
        dev_parity.append(d_par.cpu().numpy())
        t = time.perf_counter()
        for _ in range(args.passes):
            g["codec"].encode(d_objs, g["size"], parity=d_par)
        torch.cuda.synchronize()
        t_dev += (time.perf_counter() - t) / args.passes
        del d_objs, d_par

    bad = verify(groups, dev_parity)
    ok = shard.min_over_ranks(0 if bad else 1)
    if bad:
        print(f"rank {rank}: mismatches {bad[:5]}", file=sys.stderr, flush=True)

    if rank == 0:
        per_group = [{"k": g["k"], "m": g["m"], "object_bytes": g["size"], "objects": g["n"],
                      "encode_GiBps": round(g["n"] * g["size"] / min(g["te"]) / 2**30, 2),
                      "decode_GiBps": round(g["n"] * g["size"] / min(g["td"]) / 2**30, 2)}
                     for g in groups]
        print(json.dumps({
            "metric": "Swift-mix streaming encode+decode GiB/s incl. pinned H2D/D2H (object bytes)",
            "value": round(world * 2 * total / (t_write + t_read) / 2**30, 3),
            "unit": "GiB/s", "n_gpus": world, "passes": args.passes,
            "higher_is_better": True, "scaling": "weak",
            "encode_GiBps": round(world * total / t_write / 2**30, 3),
            "decode_GiBps": round(world * total / t_read / 2**30, 3),
            "verified": bool(ok),
            "placement_rank0": numa,
            "config": {"schemes": sorted({(g["k"], g["m"]) for g in groups}),
                       "object_sizes": sorted({g["size"] for g in groups}),
                       "group_bytes": args.group_mib << 20, "bytes_per_rank": total,
                       "ec_type": "amd_rs_vand", "erasures_per_object_on_read": "m"},
            "device_resident_encode_GiBps_per_gpu": round(total / t_dev / 2**30, 3),
            "groups": per_group,
        }), flush=True)
    shard.finish()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
