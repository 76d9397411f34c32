#!/usr/bin/env python3
"""Regenerate tests/golden/rs_vand_golden.json from the CPU oracle.

What the vectors pin: the GPU path against the oracle (tests/test_gpu_parity.py
and tests/test_golden.py) and the oracle against regressions.  They do NOT pin
byte-equality with a real liberasurecode build -- none exists in this
container and the reference's own tests hold no parity vectors (DESIGN.md,
"Oracle").  The fixture input storer-storagess06.pdf is a data file from the
reference's test suite (test/test_files/), used by its
test/ec_pyeclib_file_test.sh round trips.

Usage: python tests/golden/make_golden.py   (from the repo root)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

SEED = 20261015


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    out = {"generator": {}, "small": [], "sha": [], "gf_mul": [], "decode": []}
    for k, m in [(4, 2), (10, 4), (12, 2), (11, 2), (10, 2), (8, 4), (12, 4), (3, 5)]:
        out["generator"][f"{k},{m}"] = O.generator(k, m)[k:]
    rng = np.random.Generator(np.random.PCG64(SEED))
    for k, m in [(4, 2), (10, 4), (8, 4)]:
        for n in [1, 9, 1000, 4099]:
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            frags = O.encode(k, m, data)
            out["small"].append({"k": k, "m": m, "data": data.hex(),
                                 "fragments": [f.hex() for f in frags]})
    for k, m, n in [(10, 4, 4 * 1024 * 1024), (4, 2, 1024 * 1024)]:
        data = np.random.Generator(np.random.PCG64(SEED + n)).integers(
            0, 256, n, dtype=np.uint8).tobytes()
        frags = O.encode(k, m, data)
        out["sha"].append({"k": k, "m": m, "source": f"pcg64:{SEED + n}:{n}",
                           "data_sha256": sha(data), "fragments_sha256": [sha(f) for f in frags]})
    pdf = open(os.path.join(HERE, "storer-storagess06.pdf"), "rb").read()
    for k, m in [(10, 4), (4, 2), (12, 3)]:
        frags = O.encode(k, m, pdf)
        out["sha"].append({"k": k, "m": m, "source": "file:storer-storagess06.pdf",
                           "data_sha256": sha(pdf), "fragments_sha256": [sha(f) for f in frags]})
        # fixed erasure sets: decode must give the file back, reconstruct the fragment
        for lost in ([0, 1, 2, 3][:m], [k - 1, k][:m], list(range(k, k + m))):
            avail = [f for i, f in enumerate(frags) if i not in lost]
            assert O.decode(k, m, avail) == pdf
            rebuilt = [sha(O.reconstruct(k, m, avail, i)) for i in lost]
            out["decode"].append({"k": k, "m": m, "lost": lost, "rebuilt_sha256": rebuilt})
    for a, b in [(2, 0x8000), (0x1234, 0x5678), (0xFFFF, 0xFFFF), (3, 7), (0x8000, 0x8000)]:
        out["gf_mul"].append([a, b, O.gf_mul(a, b)])
    with open(os.path.join(HERE, "rs_vand_golden.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
