#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace run (rocpd SQLite database):
start offset, duration, queue and the idle gap before each launch, so the
per-step time a bench line reports can be split into kernel time and the
gaps between kernels (stream joins, host submission).

  python3 tools/rocpd_timeline.py gpurun_out/TAG/prof [--last N]
"""
import argparse
import glob
import os
import sqlite3


def rows(path):
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) if os.path.isdir(path) else [path]
    out = []
    for db in dbs:
        con = sqlite3.connect(db)
        cols = [c[1] for c in con.execute("pragma table_info(kernels)")]
        q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
        sel = f"select name, start, end{', ' + q if q else ''} from kernels order by start"
        for r in con.execute(sel):
            out.append((r[0], int(r[1]), int(r[2]), r[3] if q else 0))
    out.sort(key=lambda r: r[1])
    return out


def short(name):
    for key in ("encode_edge_kernel", "encode_kernel", "decode_edge_kernel", "decode_kernel",
                "copy_data_kernel", "crc_kernel"):
        if key in name:
            tmpl = name[name.find("<"):name.find(">") + 1] if "<" in name else ""
            return key + tmpl
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=24)
    a = ap.parse_args()
    rs = rows(a.path)[-a.last:]
    if not rs:
        print("no kernels")
        return
    t0 = rs[0][1]
    busy_end = t0
    print(f"{'start_us':>10} {'dur_us':>9} {'gap_us':>8} {'queue':>6}  kernel")
    for name, s, e, q in rs:
        gap = (s - busy_end) / 1000.0
        print(f"{(s - t0) / 1000:10.2f} {(e - s) / 1000:9.2f} {gap:8.2f} {q!s:>6}  {short(name)}")
        busy_end = max(busy_end, e)
    span = (busy_end - t0) / 1000.0
    busy = 0.0
    cur_s, cur_e = rs[0][1], rs[0][2]
    for _, s, e, _ in rs[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"span {span:.2f} us, GPU busy {busy / 1000:.2f} us, idle {span - busy / 1000:.2f} us")


if __name__ == "__main__":
    main()
