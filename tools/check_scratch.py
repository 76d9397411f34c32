#!/usr/bin/env python3
"""List every kernel of the built library that uses scratch (spills or
private arrays) with its VGPR count.  Exit 1 if any.

Reads the code objects inside the library itself (its .hip_fatbin section:
one offload bundle per translation unit) and their AMDGPU metadata notes, so
it needs no special build:

    python tools/check_scratch.py [--lib pyeclib_amd/libpyeclib_amd.so] [--grep dma]
"""
import argparse
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(lib):
    """The gfx950 code objects of every offload bundle in the library."""
    fat = subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, "/dev/stdout"],
                         check=True, capture_output=True).stdout
    pos = fat.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", fat, pos + 24)[0]
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple and size:
                yield fat[pos + off:pos + off + size]
        pos = fat.find(MAGIC, pos + 32)


def kernels(co):
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        notes = subprocess.run([READELF, "--notes", f.name], check=True, capture_output=True,
                               text=True).stdout
    cur = {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_count|agpr_count):\s+(\S+)", line)
        if not m:
            continue
        cur[m.group(1)] = m.group(2)
        if m.group(1) == "vgpr_count":  # last of the four keys (sorted) per kernel
            yield cur
            cur = {}


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--lib", default=os.path.join(ROOT, "pyeclib_amd", "libpyeclib_amd.so"))
    ap.add_argument("--grep", default="", help="also print VGPRs of kernels whose name contains this")
    a = ap.parse_args()
    seen, bad = 0, []
    for co in code_objects(a.lib):
        for k in kernels(co):
            seen += 1
            if int(k.get("private_segment_fixed_size", 0)):
                bad.append(k)
            if a.grep and a.grep in k.get("name", ""):
                print(f"{k['name']}: VGPRs {k['vgpr_count']} AGPRs {k.get('agpr_count', '?')}")
    for k in bad:
        print(f"{k['name']}: scratch {k['private_segment_fixed_size']} B/lane, VGPRs {k['vgpr_count']}")
    print(f"{seen} kernels, {len(bad)} with scratch")
    sys.exit(1 if bad or not seen else 0)


if __name__ == "__main__":
    main()
