#!/usr/bin/env python3
"""Where the time of one ECDriver.encode / decode call goes (developer tool).

For each object size: the median call time through the Python API (pageable
bytes in and out, as Swift calls it), the library's own host-side phase
times of that call (ecamd_call_phases: staging copy in, launch, host work
beside the kernel, wait for the kernel, copy out, headers), and the Python
part (allocating the output bytes objects).  With --threads the probe
re-runs itself in a child process per ECAMD_COPY_THREADS value (the copy
pool is sized once per process); --pinned does the same for
ECAMD_SINGLE_PINNED_MAX (objects up to it stage through pinned memory, larger
ones through DMA copies), both read when the process / instance starts.

    python tools/single_probe.py [--sizes 1048576,4194304] [--threads 0,4,8]
                                 [--pinned 1048576,1073741824] [--reps 30]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["copy_in", "launch", "beside_kernel", "kernel_wait", "copy_out", "headers"]


def probe(sizes, reps, k=10, m=4):
    import numpy as np
    from pyeclib_amd import ECDriver, _native
    drv = ECDriver(k=k, m=m, ec_type="liberasurecode_rs_vand")
    desc = drv.ec_lib_reference.handle.desc
    buf = (ctypes.c_double * 6)()
    rows = []
    for n in sizes:
        data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
        frags = drv.encode(data)
        avail = frags[m:m + k]
        assert drv.decode(avail) == data
        fl = len(frags[0])
        for op in ("encode", "decode"):
            call = (lambda: drv.encode(data)) if op == "encode" else (lambda: drv.decode(avail))
            for _ in range(3):
                call()
            total, phases = [], {p: [] for p in PHASES}
            for _ in range(reps):
                t0 = time.perf_counter()
                call()
                total.append(1e6 * (time.perf_counter() - t0))
                _native.lib.ecamd_call_phases(desc, buf, 6)
                for i, p in enumerate(PHASES):
                    phases[p].append(buf[i])
            alloc = []
            for _ in range(reps):
                t0 = time.perf_counter()
                if op == "encode":
                    [_native._new_bytes(None, fl) for _ in range(k + m)]
                else:
                    _native._new_bytes(None, n)
                alloc.append(1e6 * (time.perf_counter() - t0))
            rows.append({"size": n, "op": op,
                         "call_us": round(statistics.median(total), 1),
                         "phases_us": {p: round(statistics.median(v), 1) for p, v in phases.items()},
                         "alloc_outputs_us": round(statistics.median(alloc), 1)})
    drv.close()
    try:
        rows.append(register_cost(sizes, reps))
    except Exception as exc:  # noqa: BLE001 -- a probe, not a check
        rows.append({"op": "host_register", "error": repr(exc)})
    return rows


def register_cost(sizes, reps):
    """What pinning the caller's own buffer would cost instead of copying it:
    hipHostRegister (mapped) + hipHostGetDevicePointer + hipHostUnregister on
    a fresh bytes object of each size (median of `reps`)."""
    import numpy as np
    hip = ctypes.CDLL(None)  # the HIP runtime the library was loaded against (RTLD_GLOBAL)
    out = {"op": "host_register"}
    for n in sizes:
        ts = []
        for i in range(reps):
            b = np.random.default_rng(i).integers(0, 256, n, dtype=np.uint8).tobytes()
            ptr = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)
            dptr = ctypes.c_void_p()
            t0 = time.perf_counter()
            rc1 = hip.hipHostRegister(ptr, ctypes.c_size_t(n), ctypes.c_uint(2))  # mapped
            rc2 = hip.hipHostGetDevicePointer(ctypes.byref(dptr), ptr, ctypes.c_uint(0))
            t1 = time.perf_counter()
            rc3 = hip.hipHostUnregister(ptr)
            t2 = time.perf_counter()
            if rc1 or rc2 or rc3:
                out[f"{n}_error"] = [rc1, rc2, rc3]
                break
            ts.append((1e6 * (t1 - t0), 1e6 * (t2 - t1)))
        if ts:
            out[f"{n}_register_us"] = round(statistics.median(t[0] for t in ts), 1)
            out[f"{n}_unregister_us"] = round(statistics.median(t[1] for t in ts), 1)
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--sizes", default=f"{1 << 20},{4 << 20}")
    ap.add_argument("--threads", default="")
    ap.add_argument("--pinned", default="")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--direct", default="",
                    help="comma list of ECAMD_REGISTER_CALLER values, one child process each "
                         "(1: the callers' whole pages used in place)")
    a = ap.parse_args()
    sizes = [int(x) for x in a.sizes.split(",")]
    if a.direct:
        for d in a.direct.split(","):
            env = dict(os.environ, ECAMD_REGISTER_CALLER=d)
            subprocess.run([sys.executable, __file__, "--sizes", a.sizes, "--reps", str(a.reps)],
                           env=env, check=True)
        return
    if not a.threads and not a.pinned:
        for r in probe(sizes, a.reps):
            r["copy_threads"] = os.environ.get("ECAMD_COPY_THREADS", "default")
            r["pinned_max"] = os.environ.get("ECAMD_SINGLE_PINNED_MAX", "default")
            r["register_caller"] = os.environ.get("ECAMD_REGISTER_CALLER", "default")
            print(json.dumps(r), flush=True)
        return
    for t in (a.threads or "4").split(","):
        for pm in (a.pinned or "default").split(","):
            env = dict(os.environ, ECAMD_COPY_THREADS=t)
            if pm != "default":
                env["ECAMD_SINGLE_PINNED_MAX"] = pm
            subprocess.run([sys.executable, __file__, "--sizes", a.sizes, "--reps", str(a.reps)],
                           env=env, check=True)


if __name__ == "__main__":
    main()
