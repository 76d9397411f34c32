#!/usr/bin/env python3
"""Print per-kernel mean PMC values from rocprofv3 --pmc csv output dirs.

  python3 tools/pmc_table.py DIR [DIR ...]

Each DIR is searched recursively for *counter_collection.csv; values are
summed per dispatch (over dimensions/instances) and averaged per kernel.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("ecamd::(anonymous namespace)::", "")
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main():
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                per[short(row["Kernel_Name"])][row["Counter_Name"]][row["Dispatch_Id"]] += \
                    float(row["Counter_Value"])
    for kern, ctrs in sorted(per.items()):
        print(kern)
        for c, disp in sorted(ctrs.items()):
            vals = list(disp.values())
            print(f"  {c:28s} {sum(vals) / len(vals):16.1f}  (n={len(vals)})")


if __name__ == "__main__":
    main()
