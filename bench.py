#!/usr/bin/env python3
"""Headline benchmark: device-resident rs_vand encode + decode on MI355X.

Metric (BASELINE.json): "device-resident encode+decode GiB/s, k=10 m=4,
4 MiB objects, 1/2/4/8 GPU".  Workload = BASELINE configs[1] + configs[2]:
a batch of 256 objects x 4 MiB per GPU (PCG64 seed 20261015 bytes), k=10,
m=4, and for decode 4 random fragment erasures per object (same seed).

One step = encode the batch (objects -> 4 parity fragments with headers,
ecamd_encode_batch) + decode the batch (first 10 of the surviving fragments
-> objects, ecamd_decode_batch).  Inputs are resident in HBM before timing.
value = (bytes encoded + bytes decoded, all ranks) / step time, in GiB/s
(2^30, user object bytes, like pyeclib's own bench: src/pyeclib/cli/bench.py
:68-99).  Objects are independent, so N GPUs each take their own batch of
256 (weak scaling, no collective on the data path).

Other BASELINE configs run through flags, each printing its own line:
`--ec-type isa_l_rs_cauchy --k 12 --m 4 --obj-bytes 16777216 --global-batch 1024
--second reconstruct` is configs[3] (GF(2^8) Cauchy encode + reconstruct of one
random fragment per object, 1024 objects sharded over the GPUs).

`roofline` covers the kernel that dominates a step (achieved = algorithmic
bytes per launch / mean launch time from HIP events on the launch stream);
`cpu_baseline` times the scalar C oracle (tests-only restatement of
liberasurecode_rs_vand) on rank 0, single thread, over one full step's work.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident encode+decode GiB/s, k=10 m=4, 4 MiB objects, 1/2/4/8 GPU"
FIELD_BITS = {"amd_rs_vand": 16, "liberasurecode_rs_vand": 16, "isa_l_rs_vand": 8,
              "isa_l_rs_cauchy": 8}
SEED = 20261015
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="objects per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="shard this many objects over the GPUs instead (strong scaling)")
    ap.add_argument("--obj-bytes", type=int, default=4 * 1024 * 1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--erasures", type=int, default=4)
    ap.add_argument("--ec-type", default="amd_rs_vand", choices=sorted(FIELD_BITS))
    ap.add_argument("--second", default="decode", choices=["decode", "reconstruct"],
                    help="second half of a step: decode the batch, or rebuild one "
                         "random fragment per object")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="objects in the CPU baseline sample (default: the full batch)")
    ap.add_argument("--host", action="store_true",
                    help="also time the host-resident (pinned H2D/D2H) encode path")
    ap.add_argument("--verify", action="store_true", help="check one object against the oracle")
    return ap.parse_args()


def erasure_masks(rng, n_obj, k, m, erasures):
    full = (1 << (k + m)) - 1
    masks = []
    for _ in range(n_obj):
        lost = rng.choice(k + m, size=erasures, replace=False)
        masks.append(full & ~int(sum(1 << int(i) for i in lost)))
    return masks


def cpu_baseline_generic(args, host_objs, masks, dests, sample):
    """Scalar C oracle (isal_oracle.c for GF(2^8), rs_vand_oracle.c
    otherwise), one thread: encode + decode or reconstruct per object."""
    from oracle import oracle as O
    k, m, n = args.k, args.m, args.obj_bytes
    if FIELD_BITS[args.ec_type] == 8:
        kind = O.ISAL_CAUCHY if args.ec_type == "isa_l_rs_cauchy" else O.ISAL_VAND
        enc = lambda d: O.isal_encode(kind, k, m, d)  # noqa: E731
        dec = lambda f: O.isal_decode(kind, k, m, f)  # noqa: E731
        rec = lambda f, i: O.isal_reconstruct(kind, k, m, f, i)  # noqa: E731
        src = "isal_oracle.c"
    else:
        enc = lambda d: O.encode(k, m, d)  # noqa: E731
        dec = lambda f: O.decode(k, m, f)  # noqa: E731
        rec = lambda f, i: O.reconstruct(k, m, f, i)  # noqa: E731
        src = "rs_vand_oracle.c"
    t_enc = t_two = 0.0
    for o in range(sample):
        data = host_objs[o, :n].tobytes()
        t0 = time.perf_counter()
        frags = enc(data)
        t_enc += time.perf_counter() - t0
        avail = [f for i, f in enumerate(frags) if masks[o] >> i & 1]
        t0 = time.perf_counter()
        if args.second == "decode":
            assert dec(avail) == data
        else:
            assert rec(avail, dests[o]) == frags[dests[o]]
        t_two += time.perf_counter() - t0
    return {
        "value": round(2 * sample * n / (t_enc + t_two) / 2**30, 4),
        "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{sample} objects x {n} B: encode + {args.second} ({src}, "
                  f"{args.ec_type}), 1 thread",
        "encode_GiBps": round(sample * n / t_enc / 2**30, 4),
        f"{args.second}_GiBps": round(sample * n / t_two / 2**30, 4),
        "seconds": round(t_enc + t_two, 2),
    }


def cpu_baseline(args, host_objs, masks, sample):
    """Scalar C oracle, one thread: encode + decode `sample` objects."""
    import ctypes
    from oracle import oracle as O
    L = O.lib()
    k, m, n = args.k, args.m, args.obj_bytes
    fl = O.fragment_len(k, n)
    out = np.zeros((k + m) * fl, dtype=np.uint8)
    obj = np.zeros(n, dtype=np.uint8)
    t_enc = t_dec = 0.0
    for o in range(sample):
        obj[:] = host_objs[o, :n]
        t0 = time.perf_counter()
        rc = L.orc_encode(k, m, O.CHKSUM_NONE, O.LIBEC_VERSION, obj.ctypes.data, n, out.ctypes.data)
        t_enc += time.perf_counter() - t0
        assert rc == 0
        frags = [out[i * fl:(i + 1) * fl].tobytes() for i in range(k + m) if masks[o] >> i & 1]
        arr = (ctypes.c_char_p * len(frags))(*frags)
        dec = np.zeros(n, dtype=np.uint8)
        olen = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        rc = L.orc_decode(k, m, arr, len(frags), fl, dec.ctypes.data, ctypes.byref(olen))
        t_dec += time.perf_counter() - t0
        assert rc == 0 and olen.value == n
    total = 2 * sample * n
    return {
        "value": round(total / (t_enc + t_dec) / 2**30, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{sample} objects x {n} B: encode + decode with {args.erasures} erasures "
                  f"each (one step's work for that many objects), scalar C oracle "
                  f"(oracle/rs_vand_oracle.c), 1 thread",
        "encode_GiBps": round(sample * n / t_enc / 2**30, 4),
        "decode_GiBps": round(sample * n / t_dec / 2**30, 4),
        "seconds": round(t_enc + t_dec, 2),
    }


def load_pmc(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    from pyeclib_amd import shard
    world, rank, local = shard.init("nccl")
    import torch
    from pyeclib_amd import batch

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    k, m, n = args.k, args.m, args.obj_bytes
    if args.global_batch:
        lo, hi = shard.shard_range(args.global_batch, rank, world)
        B = hi - lo
    else:
        B = args.batch
    w = FIELD_BITS[args.ec_type]
    bs = batch.blocksize(k, n, w)
    fs = batch.frag_stride(bs)
    obj_stride = (n + 255) // 256 * 256

    rng = np.random.Generator(np.random.PCG64(SEED + rank))
    host = np.zeros((B, obj_stride), dtype=np.uint8)
    host[:, :n] = rng.integers(0, 256, size=(B, n), dtype=np.uint8)
    masks = erasure_masks(rng, B, k, m, args.erasures)
    # reconstruct: one random lost fragment per object, rebuilt from the rest
    dests = [int(d) for d in rng.integers(0, k + m, size=B)]
    full = (1 << (k + m)) - 1
    rmasks = [full & ~(1 << d) for d in dests]

    codec = batch.BatchCodec(k, m, ec_type=args.ec_type)
    objs = torch.from_numpy(host).to(dev)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    out = torch.zeros((B, obj_stride), dtype=torch.uint8, device=dev)
    rec = torch.zeros((B, fs), dtype=torch.uint8, device=dev)
    # decode inputs: full stripes (data fragments materialised once, untimed)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    torch.cuda.synchronize()

    if args.verify and rank == 0 and w == 16:
        from oracle import oracle as O
        want = O.encode(k, m, host[0, :n].tobytes())
        got = stripes[0, :, :80 + bs].cpu().numpy()
        assert all(got[i].tobytes() == want[i] for i in range(k + m)), "encode mismatch"
        codec.decode(stripes, n, masks, out)
        torch.cuda.synchronize()
        assert torch.equal(out[:, :n].cpu(), torch.from_numpy(host[:, :n])), "decode mismatch"

    stream = torch.cuda.current_stream()

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        codec.encode(objs, n, parity=stripes[:, k:])
        if ev is not None:
            ev[1].record(stream)
        if args.second == "decode":
            codec.decode(stripes, n, masks, out)
        else:
            codec.reconstruct(stripes, n, rmasks, dests, rec)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    shard.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    shard.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, device=dev)

    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in events]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in events]))
    step_s = elapsed / args.steps
    n_total = args.global_batch or B * world
    total_bytes = 2 * n_total * n
    value = total_bytes / step_s / 2**30

    # algorithmic HBM bytes per launch (DESIGN.md "Roofline"):
    #   encode: read the object (L), write m payloads + m headers
    #   decode: read k payloads, write the object
    #   reconstruct: read k payloads, write one fragment
    enc_bytes = B * (n + m * (bs + 80))
    two = args.second
    two_bytes = B * (k * bs + n) if two == "decode" else B * (k * bs + bs + 80)
    kernels = {
        "encode": {"ms": round(enc_ms, 4), "bytes": enc_bytes,
                   "GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 1)},
        two: {"ms": round(dec_ms, 4), "bytes": two_bytes,
              "GBps": round(two_bytes / (dec_ms * 1e-3) / 1e9, 1)},
    }
    dom = two if dec_ms >= enc_ms else "encode"
    default_workload = (args.ec_type in ("amd_rs_vand", "liberasurecode_rs_vand") and k == 10
                        and m == 4 and n == 4 * 1024 * 1024 and two == "decode")
    pmc = (load_pmc(os.path.join(ROOT, "profiles", "pmc_summary.json")) or {}) \
        if default_workload else {}
    traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch")
    achieved = kernels[dom]["GBps"]
    roofline = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "algorithmic_bytes": kernels[dom]["bytes"]}

    metric = METRIC if default_workload else (
        f"device-resident encode+{two} GiB/s, {args.ec_type} k={k} m={m}, {n} B objects")
    result = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None,
        "dtype": "u16" if w == 16 else "u8",
        "data": f"synthetic: PCG64(seed {SEED}+rank) uniform bytes; {args.erasures} random "
                "erasures per object for decode",
        "config": {"workload": f"{args.ec_type} k={k} m={m} encode + "
                               + (f"decode ({args.erasures} erasures)" if two == "decode"
                                  else "reconstruct (1 fragment)")
                               + f", {n} B objects, batch {B} per GPU, device-resident",
                   "k": k, "m": m, "object_bytes": n, "batch_per_gpu": B,
                   "erasures": args.erasures, "parallelism": f"objects sharded over {world} GPU"},
        "encode_GiBps": round(n_total * n / (enc_ms * 1e-3) / 2**30, 3),
        f"{two}_GiBps": round(n_total * n / (dec_ms * 1e-3) / 2**30, 3),
        "kernels": kernels,
        "roofline": roofline,
    }

    if args.host and rank == 0 and w == 16:
        pinned = torch.from_numpy(host).pin_memory()
        hpar = torch.zeros((B, m, fs), dtype=torch.uint8).pin_memory()
        codec.encode_host(pinned, n, hpar)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            codec.encode_host(pinned, n, hpar)
        th = (time.perf_counter() - t0) / reps
        result["host_resident_encode_GiBps"] = round(B * n / th / 2**30, 3)

    if rank == 0 and not args.no_cpu_baseline:
        sample = args.cpu_sample or B
        if w == 16 and two == "decode":
            result["cpu_baseline"] = cpu_baseline(args, host, masks, min(sample, B))
        else:
            masks2 = masks if two == "decode" else rmasks
            result["cpu_baseline"] = cpu_baseline_generic(args, host, masks2, dests,
                                                          min(sample, B))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
