#!/usr/bin/env python3
"""Scan the kernel-resource-usage remarks of a REMARKS=1 build
(pyeclib_amd/csrc/build/*.remarks) and list every kernel that uses scratch
(spills or private arrays) with its VGPR count and occupancy.  Exit 1 if any.
    make -C pyeclib_amd/csrc REMARKS=1 && python tools/check_scratch.py"""
import glob
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bad, seen = [], 0
for path in sorted(glob.glob(os.path.join(ROOT, "pyeclib_amd", "csrc", "build", "*.remarks"))):
    name = vgpr = occ = None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"VGPRs: (\d+)", line)
        if m:
            vgpr = int(m.group(1))
        m = re.search(r"Occupancy \[waves/SIMD\]: (\d+)", line)
        if m:
            occ = int(m.group(1))
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            seen += 1
            if int(m.group(1)):
                bad.append((os.path.basename(path), name, int(m.group(1)), vgpr))
for f, n, sc, v in bad:
    print(f"{f}: {n}: scratch {sc} B/lane, VGPRs {v}")
print(f"{seen} kernels, {len(bad)} with scratch")
sys.exit(1 if bad else 0)
