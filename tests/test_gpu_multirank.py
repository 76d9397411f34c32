"""The N-rank path with the HIP library loaded, on the one leased GPU: two
ranks under torch.distributed.run, both on cuda:0 (--same-device), gloo
bookkeeping (no RCCL), each rank encoding / decoding its own batch and
verifying it (bench.py against the CPU oracle, swift_mix.py against the
device-resident path and the original objects).  SURVEY §8(e); the driver's
8-GPU scaling run takes the same code with one GPU per rank."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(script, *argv, timeout=240):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, script), *argv],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_same_device():
    out = _run("bench.py", "--gpus", "2", "--same-device", "--batch", "8", "--steps", "2",
               "--warmup", "1", "--no-host", "--cpu-sample", "8", "--fresh-steps", "2")
    assert out["n_gpus"] == 2 and out["same_device"] is True
    assert out["verified"] is True and out["verified_objects"] == 16
    assert out["value"] > 0 and out["decode_fresh_ms"] > 0
    assert "cpu_baseline" not in out  # N > 1: the CPU baseline is N = 1 only


def test_swift_mix_two_ranks_same_device():
    out = _run("tools/swift_mix.py", "--gpus", "2", "--same-device", "--group-mib", "4",
               "--schemes", "10:4,6:2", "--sizes", "65536,1048576", "--passes", "1")
    assert out["n_gpus"] == 2 and out["verified"] is True
