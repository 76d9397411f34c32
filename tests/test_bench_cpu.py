"""bench.py's CPU-side legs, without a GPU: the rank launcher behind
`--gpus N` (torch.distributed.run started as a child, gloo process group in
--dry-run), the oracle pass that verifies the timed batch object by object,
and the N-process CPU baseline."""
import argparse
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(*argv, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_dry_run_single_rank():
    assert _run("--dry-run")["n_gpus"] == 1


def test_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` (no torchrun around it) starts two ranks itself."""
    out = _run("--gpus", "2", "--dry-run")
    assert out["n_gpus"] == 2 and out["requested_gpus"] == 2 and out["max_rank"] == 1.0


def _args(ec_type, k, m, n, second):
    return argparse.Namespace(ec_type=ec_type, k=k, m=m, obj_bytes=n, second=second)


@pytest.mark.parametrize("ec_type,second", [("amd_rs_vand", "decode"),
                                            ("amd_rs_vand", "reconstruct"),
                                            ("isa_l_rs_cauchy", "reconstruct"),
                                            ("isa_l_rs_vand", "decode")])
def test_oracle_pass_verifies_and_flags(oracle, ec_type, second):
    k, m, n, B = 4, 2, 20000 + 3, 5
    args = _args(ec_type, k, m, n, second)
    rng = np.random.Generator(np.random.PCG64(3))
    host = np.zeros((B, (n + 255) // 256 * 256), dtype=np.uint8)
    host[:, :n] = rng.integers(0, 256, (B, n), dtype=np.uint8)
    masks = bench.erasure_masks(rng, B, k, m, 2)
    dests = [int(d) for d in rng.integers(0, k + m, B)]
    full = (1 << (k + m)) - 1
    if second == "reconstruct":
        masks = [full & ~(1 << d) for d in dests]
    # expected outputs from the oracle's own Python API
    if bench.FIELD_BITS[ec_type] == 8:
        kind = oracle.ISAL_CAUCHY if ec_type == "isa_l_rs_cauchy" else oracle.ISAL_VAND
        frags = [oracle.isal_encode(kind, k, m, host[o, :n].tobytes()) for o in range(B)]
    else:
        frags = [oracle.encode(k, m, host[o, :n].tobytes()) for o in range(B)]
    fl = len(frags[0][0])
    gf = np.stack([np.frombuffer(b"".join(f), np.uint8).reshape(k + m, fl) for f in frags])
    if second == "decode":
        g2 = host.copy()
    else:
        g2 = np.stack([np.frombuffer(frags[o][dests[o]], np.uint8) for o in range(B)])
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=B)
    assert bad == []
    gf[2, k, 100] ^= 1          # a flipped parity byte
    g2[4, 7] ^= 0x80            # a flipped output byte
    _, _, bad, _ = bench.oracle_pass(args, host, masks, dests, gf, g2, sample=B)
    assert (2, "encode") in bad and (4, second) in bad and len(bad) == 2


def test_cpu_parallel_baseline(oracle):
    k, m, n, B = 4, 2, 65536, 6
    args = _args("amd_rs_vand", k, m, n, "decode")
    rng = np.random.Generator(np.random.PCG64(5))
    host = rng.integers(0, 256, (B, n), dtype=np.uint8)
    masks = bench.erasure_masks(rng, B, k, m, 2)
    t = bench.cpu_parallel(args, host, masks, [0] * B, B, 2)
    assert 0 < t < 60
