import sys, random
sys.path.insert(0, '.')
import numpy as np
from oracle import oracle as O
from pyeclib_amd import ECDriver
k, m = 4, 2
drv = ECDriver(k=k, m=m, ec_type="amd_rs_vand")
for n in (77, 4099, 300001, 100000, 16384*4+100):
    data = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()
    frags = O.encode(k, m, data)
    for lost in ([0], [1], [0, 1], [4], [2, 5]):
        avail = [f for i, f in enumerate(frags) if i not in lost]
        got = drv.decode(avail)
        if got != data:
            a = np.frombuffer(got, dtype=np.uint8); b = np.frombuffer(data, dtype=np.uint8)
            bad = np.nonzero(a != b)[0]
            bs = O.blocksize(k, n)
            print("n", n, "lost", lost, "bs", bs, "nbad", len(bad), "first", bad[:8], "last", bad[-4:], "frag of first", bad[0] // bs, "pos", bad[0] % bs)
        else:
            print("n", n, "lost", lost, "ok")
