#!/usr/bin/env python3
"""Per-dispatch kernel durations of a bench.py run under `rocprofv3
--kernel-trace --output-format csv`, summarised for the bench line's
roofline (bench.py reads the result when its library_id matches the loaded
library):

    python tools/kernel_stats_summary.py TRACE_DIR OUT.json --steps K

For the headline kernels -- the k=10 loader / consumer encode (parity only)
and decode -- it reports the mean and median over every dispatch (what
`rocprofv3 --stats` prints) and over the LAST K dispatches, which are the
bench's K timed steps (the settle and warm-up steps come first, at clocks
still ramping), and lists the slowest dispatches with their index.
"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kernel-name prefixes of the headline launches (ec_kernels_impl.hpp); the
# encode with data fragments (full stripe) has DATA = true in its signature
FAMILIES = {
    "encode": ("encode_dma_kernel<ecamd::(anonymous namespace)::Gf16<2>, 10, 4, 3, true, 4, 1, 12, false",),
    "decode": ("decode_dma_kernel<ecamd::(anonymous namespace)::Gf16<2>, 10, 3, true, 4, 12",),
}


def durations(trace_dir):
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {trace_dir}")
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    out = {fam: [] for fam in FAMILIES}
    for t0, t1, name in rows:
        for fam, prefixes in FAMILIES.items():
            if any(p in name for p in prefixes):
                out[fam].append((t1 - t0) / 1e3)
    return out


def summary(us, steps):
    last = us[-steps:] if steps else us
    slow = sorted(range(len(us)), key=lambda i: -us[i])[:5]
    return {"dispatches": len(us),
            "avg_us": round(statistics.mean(us), 2), "med_us": round(statistics.median(us), 2),
            "timed_steps": len(last),
            "timed_avg_us": round(statistics.mean(last), 2),
            "timed_med_us": round(statistics.median(last), 2),
            "slowest": [{"index": i, "us": round(us[i], 2)} for i in slow]}


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("trace_dir")
    ap.add_argument("out")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lib", default=os.path.join(ROOT, "pyeclib_amd", "libpyeclib_amd.so"))
    a = ap.parse_args()
    import hashlib
    with open(a.lib, "rb") as fh:
        lib_id = hashlib.sha256(fh.read()).hexdigest()[:16]
    res = {"library_id": lib_id, "source": "rocprofv3 --kernel-trace (per dispatch)",
           "note": "avg_us over every dispatch of the run (settle + warm-up + timed steps, as "
                   "rocprofv3 --stats); timed_avg_us over the last `timed_steps` dispatches, "
                   "the bench's timed steps"}
    for fam, us in durations(a.trace_dir).items():
        if us:
            res[fam] = summary(us, a.steps)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
