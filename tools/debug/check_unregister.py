"""Diagnostic: does hipHostUnregister of a registered Python bytes buffer
(unaligned start, as CallerPin registers them) leave HIP tracking the range?
For each case: register (mapped), device pointer, unregister, then
hipPointerGetAttributes on the start, middle and last byte."""
import ctypes, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
from pyeclib_amd import _native  # loads the HIP runtime the library uses
hip = ctypes.CDLL(None)

class Attr(ctypes.Structure):  # hipPointerAttribute_t (leading fields)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int),
                ("allocationFlags", ctypes.c_uint), ("pad", ctypes.c_byte * 64)]

def attr(p):
    a = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    hip.hipGetLastError()
    return rc, a.type

torch.zeros(1, device="cuda")
bad = 0
keep = []
for i, n in enumerate([65536, 1 << 20, (1 << 20) + 13, 4 << 20, 3 * 1048576 + 17, 999999, 229392, 4194304 + 7]):
    for rep in range(3):
        b = np.random.default_rng(i * 10 + rep).integers(0, 256, n, dtype=np.uint8).tobytes()
        p = ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value
        r1 = hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t((n + 15) // 16 * 16), ctypes.c_uint(2))
        d = ctypes.c_void_p()
        r2 = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(p), ctypes.c_uint(0))
        before = attr(p)
        r3 = hip.hipHostUnregister(ctypes.c_void_p(p))
        after = [attr(p), attr(p + n // 2), attr(p + n - 1)]
        ok = r1 == 0 and r2 == 0 and r3 == 0 and all(a[0] != 0 or a[1] not in (1,) for a in after)
        print(f"n={n} rep={rep} p%4096={p % 4096} reg={r1} devptr={r2} unreg={r3} before={before} after={after}", flush=True)
        # a pageable torch copy from a fresh array at (likely) the same place
        del b
        arr = np.random.default_rng(99).integers(0, 256, n, dtype=np.uint8)
        t = torch.from_numpy(arr).to("cuda")
        torch.cuda.synchronize()
        assert int(t[-1].item()) == int(arr[-1])
        keep.append(None)
print("done")
