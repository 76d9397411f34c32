#!/usr/bin/env python3
"""Find VMEM stores whose data VGPRs are overwritten by the very next VALU
instruction (gfx950 assembly from `hipcc --offload-device-only -S`).

Observed on MI355X (round 2): a `buffer_store_dwordx4 v[30:33], ..., s31 offen`
immediately followed by `v_cndmask_b32 v30, ...` stored a wrong first dword
-- hipcc's hazard recognizer assumes no hazard when soffset is an SGPR.  The
kernels put a wait state after such stores (ec_kernels_impl.hpp, st_fence);
this script checks the generated code for any store left exposed.

    python tools/store_hazard.py file.s [...]
"""
import re
import sys

# data operand: first for buffer stores, second (after the address) for global
STORE = re.compile(r"^\s*(?:buffer_store_dword(?:x2|x3|x4)?\s+|global_store_dword(?:x2|x3|x4)?\s+v\[?\d+(?::\d+)?\]?,\s*)"
                   r"v\[?(\d+)(?::(\d+))?\]?")
VALU_DST = re.compile(r"^\s*v_\w+\s+v\[?(\d+)(?::(\d+))?\]?")
KERNEL = re.compile(r"^(_Z\w+):")


def scan(path):
    bad = []
    kernel = None
    lines = open(path).read().split("\n")
    for i, line in enumerate(lines):
        k = KERNEL.match(line)
        if k:
            kernel = k.group(1)
        m = STORE.match(line)
        if not m:
            continue
        lo = int(m.group(1))
        hi = int(m.group(2)) if m.group(2) else lo
        if hi - lo + 1 <= 2:
            continue  # <= 8 bytes of data: no hazard
        # next real instruction
        j = i + 1
        while j < len(lines) and (not lines[j].strip() or lines[j].strip().startswith((";", ".", "s_waitcnt"))
                                  or lines[j].rstrip().endswith(":")):
            j += 1
        if j >= len(lines):
            continue
        d = VALU_DST.match(lines[j])
        if d:
            dlo = int(d.group(1))
            dhi = int(d.group(2)) if d.group(2) else dlo
            if dlo <= hi and dhi >= lo:
                bad.append((kernel, i + 1, line.strip(), lines[j].strip()))
    return bad


def main():
    total = 0
    for path in sys.argv[1:]:
        for kernel, ln, st, nxt in scan(path):
            total += 1
            print(f"{path}:{ln} {(kernel or '?')[:110]}\n    {st}\n    {nxt}")
    print(f"{total} exposed store(s)")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
