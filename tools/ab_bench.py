#!/usr/bin/env python3
"""A/B timing of the kernels' tuning switches, interleaved in one process.

Each positional argument is one variant: "base" (no switches) or a
comma-separated list of NAME=VAL switches, e.g.
    python tools/ab_bench.py base ECAMD_ENC_R3=1,ECAMD_DEC_R3=1 ECAMD_XCD=0
The switches exist only in the A/B build of the library (`make -C
pyeclib_amd/csrc ab` -> tools/build/libpyeclib_amd_ab.so, which this tool
loads): its launchers read them, by name, at every launch (ecamd_ab_set;
ec_kernels_impl.hpp launch_*_ab), so the variants run round-robin in one
process on the same buffers (the workload of bench.py: k=10 m=4, 256 x 4
MiB, 4 erasures per object).  The product library has none of them.  Every
variant's decode output is checked against the objects and its parity
against the first variant's (except the memory-only NOCOMP probes, whose
output is wrong by design).  Prints median / min microseconds per launch and
GB/s of algorithmic bytes.
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
AB_LIB = os.path.join(ROOT, "tools", "build", "libpyeclib_amd_ab.so")

KEYS = []  # every switch any variant names


def parse_variant(text):
    if text == "base":
        return {}
    env = {}
    for part in text.split(","):
        key, _, val = part.partition("=")
        env[key] = val
    return env


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed encode + decode steps before the rounds (clock settle)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--obj-bytes", type=int, default=4 * 1024 * 1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--full-stripe", action="store_true",
                    help="encode writes the k data fragments too (liberasurecode_encode's "
                         "full stripe); checked against the first variant's stripes")
    ap.add_argument("--alt", action="store_true",
                    help="alternate encode and decode launches, as bench.py's step does "
                         "(default: each kernel back to back)")
    ap.add_argument("--ec-type", default="amd_rs_vand",
                    help="GPU ec_type (isa_l_rs_vand / isa_l_rs_cauchy: GF(2^8) kernels)")
    ap.add_argument("--crc", action="store_true",
                    help="inline_crc32 instance (parity CRC fused into the encode launch)")
    ap.add_argument("--bench-alloc", action="store_true",
                    help="objects made as bench.py makes them (PCG64 bytes in host memory, "
                         "copied to the GPU) and its reconstruct buffer allocated too")
    ap.add_argument("--flush-mb", type=int, default=0,
                    help="with --alt: read-sweep this many MiB of a clean buffer between "
                         "each decode and the next encode, outside both kernels' events "
                         "(does the encode's alternation cost go away once the decode's "
                         "dirty Infinity-Cache lines are evicted by clean reads?)")
    ap.add_argument("--reconstruct", action="store_true",
                    help="the second kernel rebuilds one random fragment per object "
                         "(header included) instead of decoding; the 'dec' columns time it")
    ap.add_argument("--lib", default=AB_LIB, help="A/B build of the library to load")
    args = ap.parse_args()

    if not os.path.exists(args.lib):
        sys.exit(f"{args.lib} missing: build it with `make -C pyeclib_amd/csrc ab`")
    os.environ["PYECLIB_AMD_LIBRARY"] = args.lib
    import ctypes

    import torch
    from pyeclib_amd import _native, batch
    if hasattr(_native.lib, "ecamd_ab_set"):
        ab_set = _native.lib.ecamd_ab_set
        ab_set.restype = ctypes.c_int
        ab_set.argtypes = [ctypes.c_char_p, ctypes.c_int]
    elif all(v == "base" for v in args.variants):
        ab_set = None  # the product library: only its own behaviour, no switches
    else:
        sys.exit(f"{args.lib} has no A/B switches: only the variant `base` runs on it")

    k, m, n, B = args.k, args.m, args.obj_bytes, args.batch
    dev = torch.device("cuda:0")
    bs = batch.blocksize(k, n, batch._CODES[args.ec_type][1])
    stride = (n + 255) // 256 * 256
    if args.bench_alloc:
        host = np.zeros((B, stride), dtype=np.uint8)
        host[:, :n] = np.random.Generator(np.random.PCG64(20261015)).integers(
            0, 256, size=(B, n), dtype=np.uint8)
        objs = torch.from_numpy(host).to(dev)
        del host
    else:
        gen = torch.Generator(device=dev).manual_seed(20261015)
        objs = torch.randint(0, 256, (B, stride), dtype=torch.uint8, device=dev, generator=gen)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    codec = batch.BatchCodec(k, m, inline_crc32=args.crc, ec_type=args.ec_type)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    ref_stripes = stripes.clone()
    data = stripes[:, :k] if args.full_stripe else None
    rng = np.random.default_rng(7)
    full = (1 << (k + m)) - 1
    masks = [full & ~int(sum(1 << int(i) for i in rng.choice(k + m, min(4, m), replace=False)))
             for _ in range(B)]
    out = torch.zeros_like(objs)
    dests = [int(d) for d in rng.integers(0, k + m, size=B)]
    rmasks = [full & ~(1 << d) for d in dests]
    rec = torch.zeros((B, stripes.shape[2]), dtype=torch.uint8, device=dev)

    def second():
        if args.reconstruct:
            codec.reconstruct(stripes, n, rmasks, dests, rec)
        else:
            codec.decode(stripes, n, masks, out)
    if args.bench_alloc:
        rec = torch.zeros((B, batch.frag_stride(bs)), dtype=torch.uint8, device=dev)  # noqa: F841
    flush = (torch.ones(args.flush_mb << 18, dtype=torch.int32, device=dev)
             if args.flush_mb else None)
    enc_bytes = B * (n + (k + m if args.full_stripe else m) * (bs + 80))
    dec_bytes = B * (k * bs + (bs + 80 if args.reconstruct else n))

    variants = [(v, parse_variant(v)) for v in args.variants]
    for _, env in variants:
        KEYS.extend(key for key in env if key not in KEYS)
    times = {v: {"enc": [], "dec": []} for v, _ in variants}

    def apply(env):
        for key in KEYS:
            if ab_set is not None:
                ab_set(key.encode(), int(env[key]) if key in env else -1)

    # clock settle (bench.py's --settle-ms): the first ~20 ms of load run at
    # ramping clocks, which a short sweep's first rounds would otherwise measure
    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        codec.encode(objs, n, parity=stripes[:, k:], data=data)
        second()
        torch.cuda.synchronize()

    for rnd in range(args.rounds):
        for name, env in variants:
            apply(env)
            if args.full_stripe:
                stripes[:, :k].zero_()
            codec.encode(objs, n, parity=stripes[:, k:], data=data)
            second()
            if args.alt:
                # bench.py's step: encode, decode, encode, ... each kernel
                # timed by events around it (each pays for the other's
                # dirty Infinity-Cache lines, as in the bench)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3 * args.reps)]
                torch.cuda.synchronize()
                for i in range(args.reps):
                    ev[3 * i].record()
                    codec.encode(objs, n, parity=stripes[:, k:], data=data)
                    ev[3 * i + 1].record()
                    second()
                    ev[3 * i + 2].record()
                    if flush is not None:
                        flush.sum()
                torch.cuda.synchronize()
                times[name]["enc"].append(statistics.mean(
                    ev[3 * i].elapsed_time(ev[3 * i + 1]) for i in range(args.reps)) * 1e3)
                times[name]["dec"].append(statistics.mean(
                    ev[3 * i + 1].elapsed_time(ev[3 * i + 2]) for i in range(args.reps)) * 1e3)
            else:
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                torch.cuda.synchronize()
                ev[0].record()
                for _ in range(args.reps):
                    codec.encode(objs, n, parity=stripes[:, k:], data=data)
                ev[1].record()
                for _ in range(args.reps):
                    second()
                ev[2].record()
                torch.cuda.synchronize()
                times[name]["enc"].append(ev[0].elapsed_time(ev[1]) / args.reps * 1e3)
                times[name]["dec"].append(ev[1].elapsed_time(ev[2]) / args.reps * 1e3)
            if rnd == 0 and "NOCOMP" not in name:  # NOCOMP probes compute nothing
                assert torch.equal(stripes, ref_stripes), f"{name}: stripes differ"
                if args.reconstruct:
                    idx = torch.tensor(dests, device=dev)
                    want = stripes[torch.arange(B, device=dev), idx, :80 + bs]
                    assert torch.equal(rec[:, :80 + bs], want), f"{name}: reconstruct differs"
                    rec.zero_()
                else:
                    assert torch.equal(out[:, :n], objs[:, :n]), f"{name}: decode differs"
                out.zero_()
    apply({})

    print(f"{args.ec_type} k={k} m={m} {B} x {n} B, {args.rounds} rounds x {args.reps} launches, "
          f"{'alternating encode/decode' if args.alt else 'back to back'}"
          f"{', inline_crc32' if args.crc else ''}"
          f"{f', {args.flush_mb} MiB clean read sweep before each encode' if flush is not None else ''}")
    print(f"{'variant':<48} {'enc med us':>10} {'min':>8} {'GB/s':>8} "
          f"{'dec med us':>10} {'min':>8} {'GB/s':>8}")
    for name, _ in variants:
        e, d = times[name]["enc"], times[name]["dec"]
        em, dm = statistics.median(e), statistics.median(d)
        print(f"{name:<48} {em:10.1f} {min(e):8.1f} {enc_bytes / em / 1e3:8.1f} "
              f"{dm:10.1f} {min(d):8.1f} {dec_bytes / dm / 1e3:8.1f}")


if __name__ == "__main__":
    main()
