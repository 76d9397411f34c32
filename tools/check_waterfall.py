#!/usr/bin/env python3
"""List the waterfall loops in the built gfx950 kernels (dev tool).

A waterfall loop is what hipcc emits when an operand that must be scalar --
a buffer descriptor or soffset -- sits in a VGPR: v_readfirstlane the value,
s_and_saveexec the lanes that hold it, issue the access, repeat for the rest.
With a wave-uniform value it runs once, but every access it wraps waits for
its own readfirstlane/exec round trip and the loads can no longer be batched.
Round 3 found 10 of them per item in the decode stream and 24 in the fused-CRC
encode (ec_kernels_impl.hpp: to_sgpr).

Reads every build/*.hip.o of pyeclib_amd/csrc, extracts its gfx950 code object
with llvm-objdump --offloading into a temp dir, disassembles it and reports,
per kernel, the backward s_cbranch_execnz loops that contain a readfirstlane,
an s_and_saveexec and a memory instruction.  Exit 1 if any kernel whose name
matches --fail-on (default: the streaming kernels) has one.
    python tools/check_waterfall.py [--all]"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernels(code_object):
    out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", code_object], check=True,
                         capture_output=True, text=True).stdout
    name, body = None, []
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
            continue
        m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-F]+):", line)
        if m and name:
            body.append((int(m.group(2), 16), m.group(1)))
    if name:
        yield name, body


def waterfalls(body):
    found = []
    addr_index = {a: i for i, (a, _) in enumerate(body)}
    for i, (addr, ins) in enumerate(body):
        if not ins.startswith("s_cbranch_execnz"):
            continue
        m = re.match(r"s_cbranch_execnz\s+(-?\d+)", ins)
        if not m:
            continue
        off = int(m.group(1))
        if off > 32767:  # simm16 printed unsigned
            off -= 65536
        target = addr + 4 + 4 * off
        j = addr_index.get(target)
        if j is None or j >= i or i - j > 24:  # a waterfall body is a handful of instructions
            continue
        seg = [x for _, x in body[j:i]]
        if (any(x.startswith("v_readfirstlane") for x in seg)
                and any("saveexec" in x for x in seg)):
            mem = [x.split()[0] for x in seg if x.startswith(("buffer_", "global_", "ds_"))]
            if mem:
                found.append(",".join(mem))
    return found


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--all", action="store_true", help="list kernels without waterfalls too")
    ap.add_argument("--fail-on", default="encode_kernel|encode_crc_kernel|decode_kernel")
    ap.add_argument("objs", nargs="*", help="objects to scan (default: the library build)")
    args = ap.parse_args()
    objs = args.objs or sorted(glob.glob(os.path.join(ROOT, "pyeclib_amd", "csrc", "build", "*.hip.o")))
    if not objs:
        sys.exit("no build/*.hip.o: make -C pyeclib_amd/csrc first")
    bad = total = 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            local = os.path.join(tmp, os.path.basename(obj))
            with open(obj, "rb") as src, open(local, "wb") as dst:
                dst.write(src.read())
            subprocess.run([OBJDUMP, "--offloading", local], check=True, capture_output=True,
                           cwd=tmp)
            for co in glob.glob(local + "*gfx950*"):
                for name, body in kernels(co):
                    total += 1
                    wf = waterfalls(body)
                    if wf or args.all:
                        print(f"{os.path.basename(obj)}: {name}: {len(wf)} waterfall loops {sorted(set(wf))}")
                    if wf and re.search(args.fail_on, name):
                        bad += 1
    print(f"{total} kernels, {bad} streaming kernels with waterfall loops")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
