#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 --kernel-trace --stats run.

rocprofv3 (ROCm 7.2) writes a rocpd SQLite database by default; this prints
(and optionally writes as CSV) the same table as its kernel_stats.csv:
name, calls, total/avg/min/max duration in microseconds, share of GPU time.

  python3 tools/rocpd_stats.py gpurun_out/TAG/prof [out.csv]
"""
import csv
import glob
import os
import sqlite3
import sys


def stats(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    rows = {}
    for db in dbs:
        con = sqlite3.connect(db)
        for name, dur in con.execute("select name, duration from kernels"):
            rows.setdefault(name, []).append(dur / 1000.0)
    total = sum(sum(v) for v in rows.values()) or 1.0
    out = []
    for name, d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        d.sort()
        out.append({"name": name, "calls": len(d), "total_us": round(sum(d), 3),
                    "avg_us": round(sum(d) / len(d), 3), "median_us": round(d[len(d) // 2], 3),
                    "min_us": round(d[0], 3), "max_us": round(d[-1], 3),
                    "percent": round(100.0 * sum(d) / total, 2)})
    return out


def main():
    res = stats(sys.argv[1])
    for r in res:
        print(f"{r['avg_us']:10.2f} us avg {r['median_us']:10.2f} med {r['calls']:5d} calls "
              f"{r['percent']:6.2f}%  {r['name'][:110]}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(res[0]))
            w.writeheader()
            w.writerows(res)


if __name__ == "__main__":
    main()
