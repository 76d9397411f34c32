#!/usr/bin/env python3
"""Durations of, and gaps between, consecutive dispatches of one kernel in a
`rocprofv3 --kernel-trace [--memory-copy-trace] --output-format csv` run (dev
tool), for slices of the dispatch sequence:

    python tools/timeline_gaps.py TRACE_DIR NAME_REGEX  -48:-32 -16:

Copies (memory-copy trace) that start inside a slice's span are counted."""
import csv
import re
import glob
import os
import statistics
import sys


def rows(trace_dir, pattern):
    out = []
    for f in glob.glob(os.path.join(trace_dir, "**", pattern), recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    d, name = sys.argv[1], sys.argv[2]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in rows(d, "*kernel_trace.csv") if re.search(name, r["Kernel_Name"]))
    cps = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""))
                 for r in rows(d, "*memory_copy_trace.csv"))
    print(f"{len(ks)} dispatches of *{name}*, {len(cps)} copies")
    for sl in sys.argv[3:]:
        a, b = (int(x) if x else None for x in sl.split(":"))
        sel = ks[a:b]
        dur = [(e - s) / 1e3 for s, e in sel]
        gaps = [(sel[i][0] - sel[i - 1][1]) / 1e3 for i in range(1, len(sel))]
        span = (sel[-1][1] - sel[0][0]) / 1e3
        inside = [c for c in cps if sel[0][0] <= c[0] <= sel[-1][1]]
        print(f"[{sl}] n={len(sel)} span/call {span / len(sel):.1f} us  dur med {statistics.median(dur):.1f} "
              f"mean {statistics.mean(dur):.1f}  gap med {statistics.median(gaps):.1f} mean "
              f"{statistics.mean(gaps):.1f} max {max(gaps):.1f}  copies {len(inside)} "
              f"(med {statistics.median([(c[1] - c[0]) / 1e3 for c in inside]) if inside else 0:.1f} us)")
        print("   gaps:", " ".join(f"{g:.0f}" for g in gaps))


if __name__ == "__main__":
    main()
