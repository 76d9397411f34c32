#!/usr/bin/env python3
"""Single-object ECDriver call latency, DMA staging vs zero-copy pinned staging.

The single-object entry points (liberasurecode_encode / _decode /
_reconstruct_fragment, called per Swift segment) stage through HBM with DMA
copies from pageable memory, or -- for objects up to ECAMD_SINGLE_PINNED_MAX
bytes -- through pinned, device-mapped host memory the kernels read and write
directly.  This times both, interleaved in one process, per object size, and
checks every result against the first variant's.

  python3 tools/single_ab.py [--k 10 --m 4 --reps 30]
"""
import argparse
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--sizes", default="65536,262144,1048576,4194304")
    a = ap.parse_args()
    from pyeclib_amd import ECDriver
    rng = np.random.default_rng(5)
    variants = {"dma": "0", "pinned": str(1 << 40)}
    drivers = {}
    for v, val in variants.items():  # the knob is read when an instance is created
        os.environ["ECAMD_SINGLE_PINNED_MAX"] = val
        drivers[v] = ECDriver(k=a.k, m=a.m, ec_type="liberasurecode_rs_vand")
    os.environ.pop("ECAMD_SINGLE_PINNED_MAX", None)
    print(f"k={a.k} m={a.m}, median of {a.reps} calls, microseconds")
    print(f"{'size':>9} {'variant':>7} {'encode':>9} {'decode':>9} {'reconstruct':>12}")
    for n in [int(x) for x in a.sizes.split(",")]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        t = {v: {"e": [], "d": [], "r": []} for v in variants}
        ref = None
        for _ in range(a.reps):
            for v in variants:
                drv = drivers[v]
                t0 = time.perf_counter()
                frags = drv.encode(data)
                t1 = time.perf_counter()
                dec = drv.decode(frags[a.m:a.m + a.k])
                t2 = time.perf_counter()
                rec = drv.reconstruct(frags[1:a.k + 1], [0])
                t3 = time.perf_counter()
                assert dec == data, f"{v}: decode mismatch at {n}"
                if ref is None:
                    ref = frags
                assert frags == ref and rec[0] == ref[0], f"{v}: fragments differ at {n}"
                t[v]["e"].append(t1 - t0)
                t[v]["d"].append(t2 - t1)
                t[v]["r"].append(t3 - t2)
        for v in variants:
            med = {x: 1e6 * statistics.median(t[v][x]) for x in "edr"}
            print(f"{n:>9} {v:>7} {med['e']:9.1f} {med['d']:9.1f} {med['r']:12.1f}")
    for drv in drivers.values():
        drv.close()


if __name__ == "__main__":
    main()
