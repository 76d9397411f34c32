#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of bench.py into profiles/pmc_summary.json.

Usage (two separate passes: FETCH_SIZE and WRITE_SIZE do not fit one pass):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o run -- python3 bench.py ...
  python3 tools/pmc_summary.py OUT/fetch OUT/write profiles/pmc_summary.json

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  A "launch" here is one
bench call (main kernel + its edge kernel), matching bench.py's events.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(path, counter):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    per = defaultdict(lambda: defaultdict(float))  # op -> dispatch -> value
    for f in files:
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            op = "encode" if "encode" in name else "decode" if "decode" in name else None
            if op is None or "ecamd" not in name:
                continue
            per[op][(name, row["Dispatch_Id"])] += float(row["Counter_Value"])
    out = {}
    for op, d in per.items():
        main = sorted(v for (n, _), v in d.items() if "edge" not in n)
        edge = sorted(v for (n, _), v in d.items() if "edge" in n)
        # median per kernel: bench.py's untimed set-up encode (which also
        # writes the data fragments) is one of the dispatches
        out[op] = (main[len(main) // 2] if main else 0.0) + (edge[len(edge) // 2] if edge else 0.0)
    return out


def library_id():
    """Build id of the profiled library (same as pyeclib_amd._native.build_id):
    bench.py quotes these counters only while the library is unchanged."""
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "pyeclib_amd", "libpyeclib_amd.so"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def main():
    fetch_dir, write_dir, dst = sys.argv[1:4]
    fetch = load(fetch_dir, "FETCH_SIZE")
    write = load(write_dir, "WRITE_SIZE")
    summary = {"library_id": library_id()}
    for op in sorted(set(fetch) | set(write)):
        f_kib, w_kib = fetch.get(op, 0.0), write.get(op, 0.0)
        summary[op] = {
            "fetch_size_kib": round(f_kib, 1),
            "write_size_kib": round(w_kib, 1),
            "hbm_bytes_per_launch": int(round((2 * f_kib + w_kib) * 1024)),
            "note": "2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction)",
        }
    with open(dst, "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
