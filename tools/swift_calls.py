#!/usr/bin/env python3
"""The Swift call shape on one GPU: P worker processes, each calling
ECDriver.encode / decode once per segment, as Swift's object servers do
(pyeclib_c.c:512-565 encode, :770-922 decode; one call per segment from many
worker processes, the GIL held inside each call).

Each worker owns its own ECDriver (k=10, m=4, liberasurecode_rs_vand, so its
own HIP context and instance), makes its segment from its own seed, checks
one encode -> decode round trip (4 data fragments missing, so decode runs the
GPU path, not the concatenation fast path), warms up, waits at a barrier and
then calls the one operation back to back for `seconds`.  The aggregate rate
is the segment bytes of all calls over the span from the first start to the
last finish, in GiB/s of segment data (the unit of pyeclib's own
`pyeclib-backend bench`, src/pyeclib/cli/bench.py:68-99).

    python tools/swift_calls.py [--procs 1,4,16] [--sizes 1048576,4194304] [--seconds 2]

At most 16 processes may hold the GPU at once on the test boxes: a parent
that has already opened the GPU (bench.py) passes --procs up to 15.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, size, op, seconds, k, m, barrier, queue):
    sys.path.insert(0, ROOT)
    try:
        import numpy as np
        from pyeclib_amd import ECDriver
        drv = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand")
        data = np.random.Generator(np.random.PCG64(1000 + rank)).integers(
            0, 256, size, dtype=np.uint8).tobytes()
        frags = drv.encode(data)
        avail = frags[m:m + k]  # the first m data fragments lost: the GPU decode path
        ok = drv.decode(avail) == data
        call = (lambda: drv.encode(data)) if op == "encode" else (lambda: drv.decode(avail))
        for _ in range(3):
            call()
        barrier.wait(timeout=120)
        n = 0
        t0 = time.perf_counter()
        while True:
            call()
            n += 1
            t1 = time.perf_counter()
            if t1 - t0 >= seconds:
                break
        drv.close()
        queue.put({"rank": rank, "calls": n, "t0": t0, "t1": t1, "ok": ok})
    except Exception as exc:  # noqa: BLE001 -- reported by the parent
        queue.put({"rank": rank, "error": repr(exc)})
        try:
            barrier.abort()
        except Exception:  # noqa: BLE001
            pass


def run(procs, size, op, seconds=2.0, k=10, m=4):
    """P processes x one op on `size`-byte segments; returns the aggregate."""
    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(procs)
    queue = ctx.Queue()
    workers = [ctx.Process(target=_worker, args=(r, size, op, seconds, k, m, barrier, queue))
               for r in range(procs)]
    for w in workers:
        w.start()
    res = [queue.get(timeout=300) for _ in workers]
    for w in workers:
        w.join(timeout=60)
    errs = [r["error"] for r in res if "error" in r]
    if errs:
        raise RuntimeError(f"swift_calls worker failed: {errs[0]}")
    calls = sum(r["calls"] for r in res)
    span = max(r["t1"] for r in res) - min(r["t0"] for r in res)
    per_call = [(r["t1"] - r["t0"]) / r["calls"] for r in res]
    return {"procs": procs, "size": size, "op": op, "calls": calls,
            "GiBps": round(calls * size / span / 2**30, 3),
            "us_per_call_median": round(1e6 * sorted(per_call)[len(per_call) // 2], 1),
            "verified": all(r["ok"] for r in res)}


def sweep(procs=(1, 4, 16), sizes=(1 << 20, 4 << 20), seconds=2.0):
    """Every (size, op, P) run; a run whose workers fail is recorded with its
    error (and stops the sweep: a worker's GPU fault is not retried)."""
    rows = []
    for size in sizes:
        for op in ("encode", "decode"):
            for p in procs:
                try:
                    rows.append(run(p, size, op, seconds))
                except Exception as exc:  # noqa: BLE001 -- reported in the rows
                    rows.append({"procs": p, "size": size, "op": op, "error": repr(exc),
                                 "verified": False})
                    return rows
    return rows


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--procs", default="1,4,16")
    ap.add_argument("--sizes", default=f"{1 << 20},{4 << 20}")
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    rows = sweep(tuple(int(x) for x in a.procs.split(",")),
                 tuple(int(x) for x in a.sizes.split(",")), a.seconds)
    for r in rows:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
