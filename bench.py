#!/usr/bin/env python3
"""Headline benchmark: device-resident rs_vand encode + decode on MI355X.

Metric (BASELINE.json): "device-resident encode+decode GiB/s, k=10 m=4,
4 MiB objects, 1/2/4/8 GPU".  Workload = BASELINE configs[1] + configs[2]:
a batch of 256 objects x 4 MiB per GPU (PCG64 seed 20261015 + rank bytes),
k=10, m=4, and for decode 4 random fragment erasures per object (same seed).

One step = encode the batch (objects -> 4 parity fragments with headers,
ecamd_encode_batch) + decode the batch (first 10 of the surviving fragments
-> objects, ecamd_decode_batch).  Inputs are resident in HBM before timing.
value = (bytes encoded + bytes decoded, all ranks) / step time, in GiB/s
(2^30, user object bytes, like pyeclib's own bench: src/pyeclib/cli/bench.py
:68-99, which also times encode + decode of the same segment per iteration).
Objects are independent, so N GPUs each take their own batch of 256 (weak
scaling, no collective on the data path; `--global-batch` shards one batch
instead, strong scaling).

`--gpus N` runs N ranks, one process per GPU: launched by the driver under
torch.distributed.run, or -- when started directly -- bench.py starts
torch.distributed.run itself as a child process (before anything touches the
GPU) and exits with its status.  `--dry-run` exercises the rank launch and
the process group on CPU (gloo) without touching a GPU.

After the timed steps every object of the timed batch is checked: all k+m
fragments (headers included) against the CPU oracle's encode, and the decoded
(or reconstructed) output against the object (or the oracle's fragment).
Any mismatch exits non-zero; the JSON line carries "verified": true.

Other BASELINE configs run through flags, each printing its own line:
`--ec-type isa_l_rs_cauchy --k 12 --m 4 --obj-bytes 16777216 --global-batch 1024
--second reconstruct` is configs[3] (GF(2^8) Cauchy encode + reconstruct of one
random fragment per object, 1024 objects sharded over the GPUs).

`roofline` covers the kernel that dominates a step (achieved = algorithmic
bytes per launch / mean launch time from HIP events on the launch stream) and
lists the encode fraction beside it; `traffic` is the PMC-measured HBM bytes
of that launch from profiles/pmc_summary.json, quoted only when that file was
recorded on this exact library build.  `cpu_baseline` times the scalar C
oracle (tests-only restatement of liberasurecode_rs_vand) on rank 0, over
the same objects, in N worker processes (the reference's own scaling model:
one single-threaded call per process, pyeclib_c.c:1245-1251) with the
1-process figure beside it.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import statistics
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident encode+decode GiB/s, k=10 m=4, 4 MiB objects, 1/2/4/8 GPU"
FIELD_BITS = {"amd_rs_vand": 16, "liberasurecode_rs_vand": 16, "isa_l_rs_vand": 8,
              "isa_l_rs_cauchy": 8}
SEED = 20261015
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
CPU_WORKERS_PER_GPU = 16  # the GPU box's CPU share per GPU


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="objects per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="shard this many objects over the GPUs instead (strong scaling)")
    ap.add_argument("--obj-bytes", type=int, default=4 * 1024 * 1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--erasures", type=int, default=4)
    ap.add_argument("--ec-type", default="amd_rs_vand", choices=sorted(FIELD_BITS))
    ap.add_argument("--second", default="decode", choices=["decode", "reconstruct"],
                    help="second half of a step: decode the batch, or rebuild one "
                         "random fragment per object")
    ap.add_argument("--inline-crc32", action="store_true",
                    help="chksum_type inline_crc32: every fragment header carries the zlib "
                         "CRC-32 of its payload (core.py:59-63)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="objects in the CPU baseline sample (default: the full batch)")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip checking the timed batch against the oracle (profiling runs)")
    ap.add_argument("--no-host", action="store_true",
                    help="skip the host-resident (pinned H2D/D2H) encode/decode timing")
    ap.add_argument("--host", action="store_true", help=argparse.SUPPRESS)  # always on now
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="before the --warmup steps, run untimed steps for this long so the "
                         "GPU reaches its steady clocks (the kernel times fall by up to 25 %% "
                         "over the first ~20 ms of load: profiles/r03q_bench_*.json step_ms); "
                         "0 = off.  Reported as `settle` in the JSON line")
    ap.add_argument("--events", choices=("nofence", "torch"), default="nofence",
                    help="timing events of the timed steps: HIP events without the system-scope "
                         "fence (default) or torch.cuda.Event")
    ap.add_argument("--fresh-steps", type=int, default=8,
                    help="decode steps whose erasure masks are new every step (drawn from "
                         "the seed outside the clock, handed over inside it): timed apart "
                         "from the headline step, which replays one batch of masks")
    ap.add_argument("--crc-steps", type=int, default=10,
                    help="launches per run of the inline_crc32 encode leg (0: skip it)")
    ap.add_argument("--full-stripe-steps", type=int, default=10,
                    help="launches of the full-stripe encode (k data + m parity fragments, "
                         "headers included: liberasurecode_encode's output) timed after the "
                         "headline steps; 0 = skip")
    ap.add_argument("--swift-procs", default="1,4,15",
                    help="process counts of the Swift call-shape leg (tools/swift_calls.py: "
                         "P processes calling ECDriver.encode / decode per segment); '' = skip")
    ap.add_argument("--swift-seconds", type=float, default=1.0)
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (exercises the N-rank path on one GPU)")
    ap.add_argument("--no-numa", action="store_true",
                    help="do not bind each rank's CPUs to its GPU's NUMA node")
    ap.add_argument("--cpu-baseline-all", action="store_true",
                    help="also run the CPU baseline when N > 1 (default: N = 1 only)")
    ap.add_argument("--config0", action="store_true",
                    help="BASELINE configs[0]: time tools/pyeclib_encode.py / "
                         "pyeclib_decode.py (k=4 m=2, one 1 MiB file) and the oracle")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks and the process group (gloo) without a GPU")
    return ap.parse_args(argv)


# ---------------- rank launch ----------------

def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch_ranks(args) -> int:
    """Start `torch.distributed.run` with one rank per GPU as a CHILD process
    (never exec: nothing here has touched the GPU, and the ranks initialise
    their own devices) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def erasure_masks(rng, n_obj, k, m, erasures):
    full = (1 << (k + m)) - 1
    masks = []
    for _ in range(n_obj):
        lost = rng.choice(k + m, size=erasures, replace=False)
        masks.append(full & ~int(sum(1 << int(i) for i in lost)))
    return masks


def first_k(mask, k, n):
    return [i for i in range(n) if mask >> i & 1][:k]


# ---------------- CPU oracle (checker + baseline) ----------------

class OracleCodec:
    """Raw-pointer view of the scalar C oracle for one (ec_type, k, m, L):
    each call returns the seconds spent inside the C function only."""

    def __init__(self, ec_type, k, m, n, crc=False):
        from oracle import oracle as O
        self.O, self.k, self.m, self.n = O, k, m, n
        self.ct = O.CHKSUM_CRC32 if crc else O.CHKSUM_NONE
        self.w8 = FIELD_BITS[ec_type] == 8
        if self.w8:
            self.kind = O.ISAL_CAUCHY if ec_type == "isa_l_rs_cauchy" else O.ISAL_VAND
            self.L = O.lib8()
            self.fl = O.isal_blocksize(k, n) + O.HDR
            self.src = "isal_oracle.c"
        else:
            self.L = O.lib()
            self.fl = O.fragment_len(k, n)
            self.src = "rs_vand_oracle.c"
        self.frags = np.zeros((k + m, self.fl), dtype=np.uint8)
        self.obj = np.zeros(max(n, 1), dtype=np.uint8)
        self.dec = np.zeros(max(n, 1), dtype=np.uint8)
        self.rec = np.zeros(self.fl, dtype=np.uint8)

    def encode(self, data) -> float:
        self.obj[:self.n] = data
        O, L = self.O, self.L
        t0 = time.perf_counter()
        if self.w8:
            rc = L.o8_encode(self.kind, self.k, self.m, self.ct, O.LIBEC_VERSION,
                             self.obj.ctypes.data, self.n, self.frags.ctypes.data)
        else:
            rc = L.orc_encode(self.k, self.m, self.ct, O.LIBEC_VERSION,
                              self.obj.ctypes.data, self.n, self.frags.ctypes.data)
        dt = time.perf_counter() - t0
        assert rc == 0, f"oracle encode rc={rc}"
        return dt

    def _avail(self, mask):
        idx = [i for i in range(self.k + self.m) if mask >> i & 1]
        ptrs = (ctypes.c_void_p * len(idx))(*[self.frags[i].ctypes.data for i in idx])
        return ctypes.cast(ptrs, ctypes.POINTER(ctypes.c_char_p)), len(idx)

    def decode(self, mask) -> float:
        arr, cnt = self._avail(mask)
        olen = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        if self.w8:
            rc = self.L.o8_decode(self.kind, self.k, self.m, arr, cnt, self.dec.ctypes.data,
                                  ctypes.byref(olen))
        else:
            rc = self.L.orc_decode(self.k, self.m, arr, cnt, self.fl, self.dec.ctypes.data,
                                   ctypes.byref(olen))
        dt = time.perf_counter() - t0
        assert rc == 0 and olen.value == self.n, f"oracle decode rc={rc}"
        return dt

    def reconstruct(self, mask, dest) -> float:
        arr, cnt = self._avail(mask)
        O = self.O
        t0 = time.perf_counter()
        if self.w8:
            rc = self.L.o8_reconstruct(self.kind, self.k, self.m, self.ct, O.LIBEC_VERSION,
                                       arr, cnt, self.fl, dest, self.rec.ctypes.data)
        else:
            rc = self.L.orc_reconstruct(self.k, self.m, self.ct, O.LIBEC_VERSION, arr,
                                        cnt, self.fl, dest, self.rec.ctypes.data)
        dt = time.perf_counter() - t0
        assert rc == 0, f"oracle reconstruct rc={rc}"
        return dt


def oracle_pass(args, host, masks, dests, gpu_frags=None, gpu_second=None, sample=None):
    """Run the oracle over objects [0, sample): time it, and -- when GPU
    outputs are given -- compare every fragment (header included) and every
    decoded object / rebuilt fragment with it.  Returns (t_enc, t_two, bad)."""
    k, m, n = args.k, args.m, args.obj_bytes
    oc = OracleCodec(args.ec_type, k, m, n, crc=getattr(args, "inline_crc32", False))
    fl = oc.fl
    t_enc = t_two = 0.0
    bad = []
    for o in range(sample):
        t_enc += oc.encode(host[o, :n])
        if gpu_frags is not None and not np.array_equal(gpu_frags[o, :, :fl], oc.frags):
            bad.append((o, "encode"))
        if args.second == "decode":
            t_two += oc.decode(masks[o])
            if not np.array_equal(oc.dec[:n], host[o, :n]):
                bad.append((o, "oracle decode"))
            if gpu_second is not None and not np.array_equal(gpu_second[o, :n], host[o, :n]):
                bad.append((o, "decode"))
        else:
            t_two += oc.reconstruct(masks[o], dests[o])
            if not np.array_equal(oc.rec, oc.frags[dests[o]]):
                bad.append((o, "oracle reconstruct"))
            if gpu_second is not None and not np.array_equal(gpu_second[o, :fl], oc.rec):
                bad.append((o, "reconstruct"))
    return t_enc, t_two, bad, oc.src


def _cpu_worker(path, shape, lo, hi, args_dict, masks, dests, barrier, q, repeat=1):
    """One CPU-baseline process: encode + decode/reconstruct objects [lo, hi)
    with the scalar oracle, `repeat` times, after every worker is ready (one
    untimed warm-up pass over its first object: tables built, pages in)."""
    host = np.memmap(path, dtype=np.uint8, mode="r", shape=shape)
    a = argparse.Namespace(**args_dict)
    oc = OracleCodec(a.ec_type, a.k, a.m, a.obj_bytes, crc=getattr(a, "inline_crc32", False))
    np.asarray(host[lo:hi]).sum()  # page the slice in before the clock starts

    def one(o):
        oc.encode(host[o, :a.obj_bytes])
        if a.second == "decode":
            oc.decode(masks[o])
        else:
            oc.reconstruct(masks[o], dests[o])
    if hi > lo:
        one(lo)
    barrier.wait()
    t0 = time.perf_counter()
    for _ in range(repeat):
        for o in range(lo, hi):
            one(o)
    q.put(time.perf_counter() - t0)


def cpu_parallel(args, host, masks, dests, sample, workers, repeat=1):
    """The oracle over objects [0, sample) in `workers` spawned processes
    (fresh interpreters that never touch the GPU; objects shared through a
    memory-mapped temporary file), each worker's share `repeat` times.
    Returns the seconds of the slowest worker."""
    import multiprocessing as mp
    import tempfile
    shape = (sample, host.shape[1])
    fd, path = tempfile.mkstemp(prefix="ecamd_cpu_", suffix=".bin")
    os.close(fd)
    procs = []
    try:
        mm = np.memmap(path, dtype=np.uint8, mode="w+", shape=shape)
        mm[:] = host[:sample]
        mm.flush()
        del mm
        ctx = mp.get_context("spawn")
        barrier, q = ctx.Barrier(workers), ctx.Queue()
        keys = ("ec_type", "k", "m", "obj_bytes", "second", "inline_crc32")
        ad = {key: getattr(args, key, False) for key in keys}
        for w in range(workers):
            lo, hi = sample * w // workers, sample * (w + 1) // workers
            p = ctx.Process(target=_cpu_worker,
                            args=(path, shape, lo, hi, ad, masks, dests, barrier, q, repeat))
            p.start()
            procs.append(p)
        times = []
        deadline = time.time() + 600
        while len(times) < workers:
            try:
                times.append(q.get(timeout=2))
            except Exception:  # queue.Empty
                if time.time() > deadline or any(p.exitcode not in (None, 0) for p in procs):
                    raise RuntimeError("CPU baseline worker failed")
        for p in procs:
            p.join(timeout=60)
        return max(times)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
        os.unlink(path)


def cgroup_cpus():
    """CPUs the process's cgroup (v2 cpu.max) grants, or None when unlimited
    or unreadable."""
    try:
        with open("/proc/self/cgroup") as fh:
            rel = next(line.split(":", 2)[2].strip() for line in fh if line.startswith("0::"))
        with open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")) as fh:
            quota, period = fh.read().split()[:2]
        return None if quota == "max" else round(int(quota) / int(period), 2)
    except (OSError, ValueError, StopIteration):
        return None


def _cgroup_dir():
    try:
        with open("/proc/self/cgroup") as fh:
            rel = next(line.split(":", 2)[2].strip() for line in fh if line.startswith("0::"))
        return os.path.join("/sys/fs/cgroup", rel.lstrip("/"))
    except (OSError, StopIteration):
        return None


def cgroup_cpu_stat():
    """The cgroup v2 cpu.stat counters (usage / throttling), or {}."""
    d = _cgroup_dir()
    try:
        with open(os.path.join(d, "cpu.stat")) as fh:
            return {k: int(v) for k, v in (line.split() for line in fh if line.strip())}
    except (OSError, TypeError, ValueError):
        return {}


def cpu_env():
    """What bounds the CPU baseline on this box: the affinity, its physical
    cores (SMT siblings folded), the cgroup's cpu.max / cpu.weight and the
    cgroup v1 CFS quota when those files exist."""
    aff = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in aff:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as fh:
                cores.add(fh.read().strip())
        except OSError:
            cores.add(str(c))
    env = {"affinity_cpus": len(aff), "physical_cores_in_affinity": len(cores)}
    d = _cgroup_dir()
    for name in ("cpu.max", "cpu.weight", "cpuset.cpus.effective"):
        try:
            with open(os.path.join(d, name)) as fh:
                env[name] = fh.read().strip()
        except (OSError, TypeError):
            pass
    for name in ("cpu.cfs_quota_us", "cpu.cfs_period_us"):
        try:
            with open(os.path.join("/sys/fs/cgroup/cpu", name)) as fh:
                env[name] = fh.read().strip()
        except OSError:
            pass
    return env


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class HipEvent:
    """A HIP timing event without the system-scope fence
    (hipEventDisableSystemFence), recorded on the launch stream by handle:
    torch.cuda.Event's record writes back the caches between the two kernels
    it separates, a cost the timed steps would otherwise carry twice per step
    (round 5).  Same interface as torch.cuda.Event for record/elapsed_time."""
    _hip = None

    def __init__(self):
        if HipEvent._hip is None:
            HipEvent._hip = ctypes.CDLL("libamdhip64.so")
        self.h = ctypes.c_void_p()
        rc = HipEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(0x20000000))
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: {rc}")

    def record(self, stream):
        rc = HipEvent._hip.hipEventRecord(self.h, ctypes.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: {rc}")

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        rc = HipEvent._hip.hipEventElapsedTime(ctypes.byref(ms), self.h, end.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime: {rc}")
        return ms.value

    def __del__(self):
        if HipEvent._hip is not None and self.h:
            HipEvent._hip.hipEventDestroy(self.h)


def load_pmc(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


# ---------------- host-resident (pinned H2D / D2H) ----------------

def host_resident(args, codec, host, stripes, masks, fs, bs, reps=3):
    """Host-resident encode and decode rates of the same batch (BASELINE
    north_star: the path starts and ends in host memory).  Inputs and outputs
    in pinned host memory; outputs checked against the device-resident ones."""
    import torch
    k, m, n = args.k, args.m, args.obj_bytes
    B = host.shape[0]
    out = {}
    pinned = torch.from_numpy(host).pin_memory()
    # the link itself: pinned H2D and D2H of the object batch (torch copies)
    dev_buf = torch.empty(pinned.shape, dtype=torch.uint8, device=stripes.device)
    for name, (dst, src) in (("h2d", (dev_buf, pinned)), ("d2h", (pinned, dev_buf))):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        out[f"pcie_{name}_GiBps"] = round(pinned.numel() * reps / (time.perf_counter() - t0) / 2**30, 3)
    del dev_buf
    hpar = torch.zeros((B, m, fs), dtype=torch.uint8).pin_memory()
    codec.encode_host(pinned, n, hpar)
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.encode_host(pinned, n, hpar)
    te = (time.perf_counter() - t0) / reps
    ok = torch.equal(hpar[:, :, :80 + bs], stripes[:, k:, :80 + bs].cpu())
    out["host_resident_encode_GiBps"] = round(B * n / te / 2**30, 3)
    if args.second == "decode":
        # the k fragments each object's decode reads, as Swift would hand them over
        idx = torch.tensor([first_k(mk, k, k + m) for mk in masks], dtype=torch.long,
                           device=stripes.device)
        sel = stripes[torch.arange(B, device=stripes.device)[:, None], idx]
        hfr = torch.empty((B, k, fs), dtype=torch.uint8).pin_memory()
        hfr.copy_(sel)
        del sel
        hout = torch.zeros((B, host.shape[1]), dtype=torch.uint8).pin_memory()
        codec.decode_host(hfr, n, masks, hout)
        t0 = time.perf_counter()
        for _ in range(reps):
            codec.decode_host(hfr, n, masks, hout)
        td = (time.perf_counter() - t0) / reps
        ok = ok and torch.equal(hout[:, :n], pinned[:, :n])
        out["host_resident_decode_GiBps"] = round(B * n / td / 2**30, 3)
    # the copy-engine pipeline for the record: inputs H2D in chunks on 3
    # streams, kernels writing the host outputs (staged) or HBM + D2H copies
    # (staged_out)
    for tag, env in (("staged", {"ECAMD_HOST_STAGED": "1"}),
                     ("staged_out", {"ECAMD_HOST_STAGED": "1", "ECAMD_HOST_STAGED_OUT": "1"})):
        os.environ.update(env)
        try:
            # the knobs are read when an instance is created
            from pyeclib_amd import batch
            c2 = batch.BatchCodec(k, m, ec_type=args.ec_type, inline_crc32=args.inline_crc32)
            hpar2 = torch.zeros_like(hpar).pin_memory()
            c2.encode_host(pinned, n, hpar2)
            t0 = time.perf_counter()
            for _ in range(reps):
                c2.encode_host(pinned, n, hpar2)
            out[f"host_{tag}_encode_GiBps"] = round(B * n / ((time.perf_counter() - t0) / reps) / 2**30, 3)
            ok = ok and torch.equal(hpar2[:, :, :80 + bs], hpar[:, :, :80 + bs])
            if args.second == "decode":
                hout.zero_()
                c2.decode_host(hfr, n, masks, hout)
                t0 = time.perf_counter()
                for _ in range(reps):
                    c2.decode_host(hfr, n, masks, hout)
                out[f"host_{tag}_decode_GiBps"] = round(B * n / ((time.perf_counter() - t0) / reps) / 2**30, 3)
                ok = ok and torch.equal(hout[:, :n], pinned[:, :n])
        finally:
            for key in env:
                del os.environ[key]
    out["host_resident_verified"] = bool(ok)
    out["host_resident_note"] = (f"pinned host in/out, {reps} reps of the batch; kernels read "
                                 "and write the mapped host arrays over PCIe (staged: inputs "
                                 "H2D by the copy engine in chunks on 3 streams; staged_out: "
                                 "outputs too, through HBM + D2H copies)")
    return out


# ---------------- single-object calls (the ECDriver path Swift uses) ----------------

def single_object_calls(args, sizes=(64 << 10, 1 << 20, 4 << 20), reps=20):
    """Per-call latency of ECDriver.encode / decode (one object, pageable Python
    bytes in and out: pyeclib_c.c:512-565 / :770-922 through the C ABI) and of
    the scalar oracle on the same object, median of `reps` calls.  Decode drops
    the first `erasures` data fragments, so it runs the GPU path, not the
    concatenation fast path."""
    from pyeclib_amd import ECDriver
    k, m = args.k, args.m
    ec_type = "liberasurecode_rs_vand" if args.ec_type == "amd_rs_vand" else args.ec_type
    drv = ECDriver(k=k, m=m, ec_type=ec_type)
    rng = np.random.Generator(np.random.PCG64(SEED + 7))
    res = {}
    for n in sizes:
        data = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        frags = drv.encode(data)
        lost = min(args.erasures, m)
        avail = frags[lost:lost + k]
        assert drv.decode(avail) == data, "single-object decode mismatch"
        te, td = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            drv.encode(data)
            t1 = time.perf_counter()
            drv.decode(avail)
            t2 = time.perf_counter()
            te.append(t1 - t0)
            td.append(t2 - t1)
        oc = OracleCodec(args.ec_type, k, m, n)
        arr = np.frombuffer(data, dtype=np.uint8)
        mask = ((1 << (k + m)) - 1) & ~((1 << lost) - 1)
        for _ in range(2):  # warm: page in the buffers and the tables
            oc.encode(arr)
            oc.decode(mask)
        ce = [oc.encode(arr) for _ in range(reps)]
        cd = [oc.decode(mask) for _ in range(reps)]
        res[f"{n >> 10}KiB"] = {
            "gpu_encode_us": round(1e6 * float(np.median(te)), 1),
            "gpu_decode_us": round(1e6 * float(np.median(td)), 1),
            "oracle_encode_us": round(1e6 * float(np.median(ce)), 1),
            "oracle_decode_us": round(1e6 * float(np.median(cd)), 1),
        }
    drv.close()
    return {"single_object_calls": res,
            "single_object_note": f"ECDriver({k},{m},{ec_type}) per-call latency, pageable bytes "
                                  f"in/out, median of {reps}; decode with {min(args.erasures, m)} "
                                  "data fragments missing; oracle = scalar C restatement, 1 core, "
                                  f"2 warm-up calls then the median of {reps}"}


# ---------------- main ----------------

def dry_run(args):
    from pyeclib_amd import placement, shard
    world, rank, local = shard.init("gloo")
    numa = placement.bind_to_gpu_numa(shard.device_index(local, args.same_device),
                                      apply=False)
    t = shard.max_over_ranks(float(rank))
    ok = shard.min_over_ranks(1)
    shard.barrier()
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "requested_gpus": args.gpus,
                          "max_rank": t, "all_ok": ok, "numa": numa}), flush=True)
    shard.finish()


# ---------------- the reference's own benchmark: `pyeclib-backend bench` ----------------

def reference_cli_bench(iterations=200, oracle_iterations=20):
    """pyeclib's own benchmark tool at its defaults (src/pyeclib/cli/
    __init__.py:74-96: k=10, m=5, 1 MiB segments, 2 unavailable data
    fragments; cli/bench.py:36-99: 200 iterations, MB/s = iterations x
    segment / 2^20 over wall time, one ECDriver call per segment, a fresh
    slice of the data per encode, a random fragment choice per decode), run
    through this package's CLI (`python -m pyeclib_amd.cli bench`) for the
    GPU ec_types, beside the scalar C oracle on one core doing the same
    calls (`oracle_iterations` of them)."""
    import random
    import re
    import subprocess
    from oracle import oracle as O
    out = {}
    cmd = [sys.executable, "-m", "pyeclib_amd.cli", "bench", "--ec-type", "amd_rs_vand",
           "--ec-type", "liberasurecode_rs_vand", "--iterations", str(iterations)]
    text = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300).stdout
    for name, op, rate in re.findall(r"^(\S+) \((encode|decode)\): ([0-9.]+)MB/s", text, re.M):
        out.setdefault(name, {})[f"{op}_MBps"] = float(rate)
    k, m, seg, u = 10, 5, 1 << 20, 2
    data = os.urandom(seg + oracle_iterations)
    frags = O.encode(k, m, data[:seg])
    t0 = time.perf_counter()
    for i in range(oracle_iterations):
        O.encode(k, m, data[i:i + seg])
    enc = oracle_iterations * seg / 2**20 / (time.perf_counter() - t0)
    rng = random.Random(5)
    t0 = time.perf_counter()
    for _ in range(oracle_iterations):
        O.decode(k, m, rng.sample(frags[:k], k - u) + rng.sample(frags[k:], u))
    dec = oracle_iterations * seg / 2**20 / (time.perf_counter() - t0)
    out["oracle_1core"] = {"encode_MBps": round(enc, 1), "decode_MBps": round(dec, 1)}
    out["note"] = (f"`python -m pyeclib_amd.cli bench` at the reference tool's defaults (k=10 "
                   f"m=5, 1 MiB segments, 2 unavailable, {iterations} iterations; "
                   "src/pyeclib/cli/bench.py), beside the scalar C oracle on one core making the "
                   f"same calls ({oracle_iterations} of each)")
    return {"reference_cli_bench": out}


# ---------------- first calls of a fresh process ----------------

_FIRST_CALL = r"""
import json, os, time
t0 = time.perf_counter()
import pyeclib_amd
t1 = time.perf_counter()
d = pyeclib_amd.ECDriver(k=10, m=4, ec_type="liberasurecode_rs_vand")
t2 = time.perf_counter()
data = os.urandom(1 << 20)
r = {"import_ms": t1 - t0, "driver_ms": t2 - t1}
for i in (1, 2):
    t = time.perf_counter(); frags = d.encode(data); r[f"encode_{i}_ms"] = time.perf_counter() - t
for i in (1, 2):
    t = time.perf_counter(); back = d.decode(frags[4:]); r[f"decode_{i}_ms"] = time.perf_counter() - t
assert back == data
print(json.dumps({k: round(v * 1e3, 2) for k, v in r.items()}))
"""


def first_call():
    """What a fresh process pays before its first results (round 5, verdict
    item 6): import, ECDriver construction (HIP initialisation, device
    tables), then the first and second 1 MiB encode and decode (the first
    launch of each kernel loads its code object).  A child interpreter, so
    nothing of this process's warm state counts."""
    text = subprocess.run([sys.executable, "-c", _FIRST_CALL], cwd=ROOT, capture_output=True,
                          text=True, timeout=300, check=True).stdout
    out = json.loads(text.strip().splitlines()[-1])
    out["note"] = ("fresh interpreter: import pyeclib_amd, ECDriver(10, 4) construction, then the "
                   "first and second 1 MiB encode and decode (4 data fragments missing), wall ms")
    return {"first_call": out}


# ---------------- configs[0]: the file CLI on k=4 m=2 ----------------

def config0_cli(args, size=1 << 20, reps=5):
    """BASELINE configs[0]: one 1 MiB file through tools/pyeclib_encode.py and
    tools/pyeclib_decode.py (the reference's positional CLI,
    tools/pyeclib_encode.py:27-37 there), k=4 m=2, GPU ec_type, with m random
    fragments dropped before the decode (test/ec_pyeclib_file_test.sh's
    recipe).  Reports the CLI wall time (a fresh interpreter per call, as a
    user runs it) and the in-process ECDriver time for the same bytes, plus
    the scalar oracle (1 core) on the same file."""
    import random
    import tempfile
    from pyeclib_amd import ECDriver
    k, m = 4, 2
    ec_type = "liberasurecode_rs_vand"
    rng = np.random.Generator(np.random.PCG64(SEED + 11))
    data = rng.integers(0, 256, size=size, dtype=np.uint8).tobytes()
    pick = random.Random(SEED)
    out = {}
    with tempfile.TemporaryDirectory(prefix="ecamd_cfg0_") as d:
        src = os.path.join(d, "file.bin")
        with open(src, "wb") as fh:
            fh.write(data)
        fdir = os.path.join(d, "frags")
        os.makedirs(fdir)
        enc = [sys.executable, os.path.join(ROOT, "tools", "pyeclib_encode.py"), str(k), str(m),
               "0", ec_type, d, "file.bin", fdir]
        t_enc, t_dec = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            subprocess.run(enc, check=True, stdout=subprocess.DEVNULL)
            t_enc.append(time.perf_counter() - t0)
            keep = sorted(pick.sample(range(k + m), k))
            dec = [sys.executable, os.path.join(ROOT, "tools", "pyeclib_decode.py"), str(k), str(m),
                   "0", ec_type] + [os.path.join(fdir, f"file.bin.{i}") for i in keep] + \
                  [os.path.join(d, "out")]
            t0 = time.perf_counter()
            subprocess.run(dec, check=True, stdout=subprocess.DEVNULL)
            t_dec.append(time.perf_counter() - t0)
            with open(os.path.join(d, "out.decoded"), "rb") as fh:
                if fh.read() != data:
                    raise SystemExit("configs[0]: decoded file differs from the input")
    mib = size / 2**20
    out["cli_encode_s"] = round(float(np.median(t_enc)), 4)
    out["cli_decode_s"] = round(float(np.median(t_dec)), 4)
    out["cli_encode_MiBps"] = round(mib / out["cli_encode_s"], 2)
    out["cli_decode_MiBps"] = round(mib / out["cli_decode_s"], 2)
    # in process: the ECDriver calls the CLI makes, without interpreter start-up
    drv = ECDriver(k=k, m=m, ec_type=ec_type)
    frags = drv.encode(data)
    te, td = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        frags = drv.encode(data)
        te.append(time.perf_counter() - t0)
        keep = sorted(pick.sample(range(k + m), k))
        t0 = time.perf_counter()
        got = drv.decode([frags[i] for i in keep])
        td.append(time.perf_counter() - t0)
        if got != data:
            raise SystemExit("configs[0]: in-process decode differs from the input")
    drv.close()
    out["inproc_encode_us"] = round(1e6 * float(np.median(te)), 1)
    out["inproc_decode_us"] = round(1e6 * float(np.median(td)), 1)
    out["inproc_encode_MiBps"] = round(mib / float(np.median(te)), 1)
    out["inproc_decode_MiBps"] = round(mib / float(np.median(td)), 1)
    # the scalar oracle on the same file (CPU baseline leg: 1 core)
    oc = OracleCodec(ec_type, k, m, size)
    arr = np.frombuffer(data, dtype=np.uint8)
    mask = ((1 << (k + m)) - 1) & ~0b11  # data fragments 0 and 1 lost: the GF path
    for _ in range(2):
        oc.encode(arr)
        oc.decode(mask)
    ce = [oc.encode(arr) for _ in range(20)]
    cd = [oc.decode(mask) for _ in range(20)]
    out["oracle_encode_us"] = round(1e6 * float(np.median(ce)), 1)
    out["oracle_decode_us"] = round(1e6 * float(np.median(cd)), 1)
    out["note"] = (f"k={k} m={m} {ec_type}, one {size} B file; CLI = fresh interpreter per "
                   f"call, median of {reps}, decode from {k} of {k + m} fragment files "
                   "(m random dropped); in-process = ECDriver calls, median of 20; oracle = "
                   "scalar C restatement, 1 core, median of 20")
    return {"config0": out}


# ---------------- decode with erasures that change every step ----------------

def fresh_decode_steady(args, codec, stripes, objs, out, stream, B, rank, head_masks):
    """Decode with erasures drawn anew for every call, back to back: the
    masks of all `--fresh-steps` calls are drawn first (outside the clock),
    then the calls are made with no synchronisation between them, so call
    i+1's host work (first-k choice, decode rows and tables of new patterns,
    descriptors and their copy -- what the reference redoes in every decode,
    pyeclib_c.c:878) overlaps call i's kernel, as a server streaming decodes
    would run.  Reported per call: GPU event span / calls, and host wall /
    calls.  Every call decodes the same objects, so the last call's output is
    compared with them; each call's output is also checked, against the
    objects, by the idle-GPU variant (fresh_decode).  A third pass makes the
    same calls with the headline's masks every time (the control: the same
    back-to-back shape, no new masks)."""
    import torch
    k, m, n = args.k, args.m, args.obj_bytes
    steps = max(2, args.fresh_steps)

    def run(first, fixed=None):  # `steps` calls, masks new for every call (or `fixed`)
        all_masks = []
        for i in range(first, first + steps):
            rng = np.random.Generator(np.random.PCG64(SEED + rank + 7919 * (i + 1)))
            all_masks.append(erasure_masks(rng, B, k, m, args.erasures) if fixed is None
                             else fixed)
        out.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        # one extra call ahead of the clock: the span then starts with the
        # pipeline full (call i+1's host work under call i's kernel), not
        # with the GPU idle through the first call's host work
        codec.decode(stripes, n, fixed if fixed is not None else erasure_masks(
            np.random.Generator(np.random.PCG64(SEED + rank + 104729 + first)), B, k, m,
            args.erasures), out)
        e0.record(stream)
        t0 = time.perf_counter()
        for masks in all_masks:
            codec.decode(stripes, n, masks, out)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return e0.elapsed_time(e1) / steps, 1e3 * wall / steps, bool(torch.equal(out[:, :n], objs[:, :n]))

    # first pass: the device's table pool meets most of the batch's erasure
    # patterns for the first time (decode rows and tables built on the host);
    # second pass: new masks again, their patterns mostly cached
    cold_ms, cold_wall, ok0 = run(0)
    ms, wall_ms, ok1 = run(steps)
    rep_ms, rep_wall, ok2 = run(0, head_masks)
    return {"decode_fresh_ms": round(ms, 4),
            "decode_repeat_ms": round(rep_ms, 4),
            "decode_repeat_wall_ms": round(rep_wall, 4),
            "decode_fresh_vs_repeat": round(ms / rep_ms, 4),
            "decode_fresh_wall_ms": round(wall_ms, 4),
            "decode_fresh_cold_ms": round(cold_ms, 4),
            "decode_fresh_cold_wall_ms": round(cold_wall, 4),
            "decode_fresh_steps": steps,
            "decode_fresh_note": "steady state: new erasure masks for every call (PCG64 seed + "
                                 "rank + 7919*call, drawn before the clock), calls back to back "
                                 "with no sync between them, so each call's host descriptor/table "
                                 "build and upload overlap the previous call's kernel; per call = "
                                 "event span / calls, the span opened behind one untimed call of "
                                 "the same kind (pipeline full); decode_fresh_cold_ms = the first "
                                 "such pass, "
                                 "whose patterns are mostly new to the device's table pool, "
                                 "decode_fresh_ms = the next pass (new masks, patterns mostly "
                                 "cached); both passes' last outputs compared with the objects; "
                                 "decode_repeat_ms = the same back-to-back pass with the "
                                 "headline's masks in every call (the control)"}, \
        ok0 and ok1 and ok2


def fresh_decode(args, codec, stripes, objs, out, stream, B, rank):
    """`--fresh-steps` decode steps whose masks are drawn anew each step (seed
    + rank + step, outside the clock) and handed to the call inside it, so
    the per-call work the reference does in every decode (pyeclib_c.c:878:
    first-k choice, inverse, tables, descriptors, their H2D) is timed.  The
    GPU is idle when each step starts, so the event span covers the host
    work before the launch too.  Every step's output is compared with the
    objects (on the GPU, untimed); returns the timing dict and all-ok."""
    import torch
    k, m, n = args.k, args.m, args.obj_bytes
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.fresh_steps)]
    gpu_ms, wall_ms, ok = [], [], True
    for i in range(args.fresh_steps):
        rng = np.random.Generator(np.random.PCG64(SEED + rank + 1000 * (i + 1)))
        masks = erasure_masks(rng, B, k, m, args.erasures)
        out.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[i][0].record(stream)
        codec.decode(stripes, n, masks, out)
        ev[i][1].record(stream)
        torch.cuda.synchronize()
        wall_ms.append(1e3 * (time.perf_counter() - t0))
        gpu_ms.append(ev[i][0].elapsed_time(ev[i][1]))
        ok = ok and bool(torch.equal(out[:, :n], objs[:, :n]))
    return {"decode_fresh_idle_ms": round(float(np.mean(gpu_ms)), 4),
            "decode_fresh_idle_first_ms": round(gpu_ms[0], 4),
            "decode_fresh_idle_wall_ms": round(float(np.mean(wall_ms)), 4),
            "decode_fresh_idle_note": "new erasure masks every step (PCG64 seed + rank + "
                                      "1000*step), each from an idle GPU (sync before): event "
                                      "span = host descriptor build + H2D + kernel + clock ramp; "
                                      "every step's objects compared with the originals"}, ok


def crc_encode_leg(args, codec, objs, n, k, m, bs, B, stream):
    """Per-launch time of the parity encode with and without inline_crc32
    (CRC kernels + finishing pass), same buffers, back to back."""
    import zlib
    import torch
    from pyeclib_amd import batch
    crc_codec = batch.BatchCodec(k, m, ec_type=args.ec_type, inline_crc32=True)
    dev = objs.device
    st_plain = batch.stripe_buffer(B, k, m, bs, device=dev)
    st_crc = batch.stripe_buffer(B, k, m, bs, device=dev)
    steps = args.crc_steps
    ms = {}
    for name, c, st in (("plain", codec, st_plain), ("crc", crc_codec, st_crc), ("plain2", codec, st_plain),
                        ("crc2", crc_codec, st_crc)):
        c.encode(objs, n, parity=st[:, k:])
        torch.cuda.synchronize()
        # an event pair around every call: the device time of its launches
        # (the CRC encode's finishing pass included), not the host's pace
        mk = HipEvent if args.events == "nofence" else (lambda: torch.cuda.Event(enable_timing=True))
        ev = [(mk(), mk()) for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            c.encode(objs, n, parity=st[:, k:])
            b.record(stream)
        torch.cuda.synchronize()
        ms[name] = statistics.median([a.elapsed_time(b) for a, b in ev])
    # payloads equal, and chksum[0] (header bytes 21..24) = crc32 of the payload
    ok = bool(torch.equal(st_plain[:, k:, 80:80 + bs], st_crc[:, k:, 80:80 + bs]))
    for o in sorted({0, B // 3, B // 2, B - 1}):
        for q in range(m):
            frag = st_crc[o, k + q, :80 + bs].cpu().numpy().tobytes()
            ok = ok and int.from_bytes(frag[21:25], "little") == zlib.crc32(frag[80:80 + bs])
    plain, crc = min(ms["plain"], ms["plain2"]), min(ms["crc"], ms["crc2"])
    del st_plain, st_crc, crc_codec
    return {"ms": round(crc, 4), "plain_ms": round(plain, 4), "vs_plain": round(crc / plain, 3),
            "launches": 2 * steps, "verified_sample": ok,
            "note": "parity-only encode with chksum_type inline_crc32 (chunk CRCs on the matrix cores "
                    "+ the finishing pass) against the plain parity encode, on this box: an event pair "
                    "(the headline's kind) around every call (device time), the median of `launches`/2 "
                    "calls, the faster of two runs each; "
                    "headers of 4 objects checked against zlib.crc32"}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_ranks(args))
    if args.dry_run:
        return dry_run(args)
    from pyeclib_amd import placement, shard
    world, rank, local = shard.rank_info()
    dev_idx = shard.device_index(local, args.same_device)
    # CPUs first, before anything starts the HIP runtime (its threads inherit
    # the mask), then the pinned buffers are first touched on that node
    numa = {"bound": False, "reason": "--no-numa"} if args.no_numa else \
        placement.bind_to_gpu_numa(dev_idx)
    import torch
    from pyeclib_amd import _native, batch
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    shard.init("gloo")  # bookkeeping only: no RCCL communicator
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks; "
              f"reporting n_gpus={world}", file=sys.stderr)
    k, m, n = args.k, args.m, args.obj_bytes
    if args.global_batch:
        lo, hi = shard.shard_range(args.global_batch, rank, world)
        B = hi - lo
    else:
        B = args.batch
    w = FIELD_BITS[args.ec_type]
    bs = batch.blocksize(k, n, w)
    fs = batch.frag_stride(bs)
    fl = 80 + bs
    obj_stride = (n + 255) // 256 * 256

    rng = np.random.Generator(np.random.PCG64(SEED + rank))
    host = np.zeros((B, obj_stride), dtype=np.uint8)
    host[:, :n] = rng.integers(0, 256, size=(B, n), dtype=np.uint8)
    masks = erasure_masks(rng, B, k, m, args.erasures)
    # reconstruct: one random lost fragment per object, rebuilt from the rest
    dests = [int(d) for d in rng.integers(0, k + m, size=B)]
    full = (1 << (k + m)) - 1
    rmasks = [full & ~(1 << d) for d in dests]
    two = args.second
    two_masks = masks if two == "decode" else rmasks

    codec = batch.BatchCodec(k, m, ec_type=args.ec_type, inline_crc32=args.inline_crc32)
    objs = torch.from_numpy(host).to(dev)
    stripes = batch.stripe_buffer(B, k, m, bs, device=dev)
    out = torch.zeros((B, obj_stride), dtype=torch.uint8, device=dev)
    rec = torch.zeros((B, fs), dtype=torch.uint8, device=dev)
    # decode inputs: full stripes (data fragments materialised once, untimed)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    p_parity = stripes[:, k:]

    # Kernel timing: HIP events on the launch stream, two per step -- before
    # the encode and before the decode; a decode ends at the next step's first
    # event (or the closing one).  (Each event record costs the stream ~5 us
    # of GPU time between kernels: profiles/r02n_timeline.txt.)
    def step(ev_enc=None, ev_dec=None):
        if ev_enc is not None:
            ev_enc.record(stream)
        codec.encode(objs, n, parity=p_parity)
        if ev_dec is not None:
            ev_dec.record(stream)
        if two == "decode":
            codec.decode(stripes, n, masks, out)
        else:
            codec.reconstruct(stripes, n, rmasks, dests, rec)

    # Clock settle, then the W warmup steps.  A fresh box starts the step
    # below its steady clocks and the kernels speed up over the first ~20 ms
    # of sustained load (r03q, --inline-crc32: encode 528 us in the first
    # timed step after 5 warmup steps, 360 us twenty steps later; 373 -> 340
    # after 30 warmup steps), so the timed steps would measure the ramp, not
    # the path.  The settle steps are the same untimed work as the warmup
    # steps, bounded by time, and reported.
    settle_steps, t_settle = 0, time.perf_counter()
    while args.settle_ms > 0 and (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        step()
        settle_steps += 1
        if settle_steps % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    settle_ms = (time.perf_counter() - t_settle) * 1e3 if settle_steps else 0.0
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    events = [HipEvent() if args.events == "nofence" else torch.cuda.Event(enable_timing=True)
              for _ in range(2 * args.steps + 1)]
    shard.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[2 * i], events[2 * i + 1])
    events[-1].record(stream)
    torch.cuda.synchronize()
    shard.barrier()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0)

    enc_ms = float(np.mean([events[2 * i].elapsed_time(events[2 * i + 1])
                            for i in range(args.steps)]))
    dec_ms = float(np.mean([events[2 * i + 1].elapsed_time(events[2 * i + 2])
                            for i in range(args.steps)]))
    step_s = elapsed / args.steps
    n_total = args.global_batch or B * world
    total_bytes = 2 * n_total * n
    value = total_bytes / step_s / 2**30

    # algorithmic HBM bytes per launch:
    #   encode: read the object (L), write m payloads + m headers
    #   decode: read k payloads, write the object
    #   reconstruct: read k payloads, write one fragment
    enc_read = B * n
    two_read = B * k * bs
    enc_bytes = enc_read + B * m * (bs + 80)
    two_bytes = two_read + (B * n if two == "decode" else B * (bs + 80))
    kernels = {
        "encode": {"ms": round(enc_ms, 4), "bytes": enc_bytes, "read_bytes": enc_read,
                   "GBps": round(enc_bytes / (enc_ms * 1e-3) / 1e9, 1)},
        two: {"ms": round(dec_ms, 4), "bytes": two_bytes, "read_bytes": two_read,
              "GBps": round(two_bytes / (dec_ms * 1e-3) / 1e9, 1)},
    }
    dom = two if dec_ms >= enc_ms else "encode"
    default_workload = (args.ec_type in ("amd_rs_vand", "liberasurecode_rs_vand") and k == 10
                        and m == 4 and n == 4 * 1024 * 1024 and two == "decode"
                        and B == 256 and not args.inline_crc32)
    pmc = (load_pmc(os.path.join(ROOT, "profiles", "pmc_summary.json")) or {}) \
        if default_workload else {}
    lib_id = _native.build_id()
    pmc_ok = pmc.get("library_id") == lib_id
    # rocprof per-dispatch kernel times of this same library (profiles/
    # kernel_stats.json, tools/kernel_stats_summary.py), beside the events
    kst = (load_pmc(os.path.join(ROOT, "profiles", "kernel_stats.json")) or {}) \
        if default_workload else {}
    kst_ok = kst.get("library_id") == lib_id
    traffic = pmc.get(dom, {}).get("hbm_bytes_per_launch") if pmc_ok else None
    achieved = kernels[dom]["GBps"]

    def read_frac(kk):
        v = kernels[kk]
        return round(v["read_bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)

    roofline = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "algorithmic_bytes": kernels[dom]["bytes"],
                "read_frac": read_frac(dom),
                "frac_by_kernel": {kk: round(v["GBps"] / HBM_PEAK_GBPS, 4)
                                   for kk, v in kernels.items()},
                "read_frac_by_kernel": {kk: read_frac(kk) for kk in kernels},
                "traffic_by_kernel": ({kk: pmc.get(kk, {}).get("hbm_bytes_per_launch")
                                       for kk in kernels} if pmc_ok else None),
                "library_id": lib_id}
    if kst_ok and dom in kst:
        # the same algorithmic bytes over rocprof's kernel time: every
        # dispatch of the profiled run (rocprofv3 --stats) and its timed steps
        def frac_us(us, kk):
            return round(kernels[kk]["bytes"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
        roofline["frac_rocprof"] = frac_us(kst[dom]["avg_us"], dom)
        roofline["frac_rocprof_timed"] = frac_us(kst[dom]["timed_avg_us"], dom)
        roofline["rocprof_us"] = {kk: {"avg": kst[kk]["avg_us"], "timed_avg": kst[kk]["timed_avg_us"],
                                       "frac": frac_us(kst[kk]["avg_us"], kk),
                                       "frac_timed": frac_us(kst[kk]["timed_avg_us"], kk)}
                                  for kk in kernels if kk in kst}
        roofline["rocprof_source"] = "profiles/kernel_stats.json (tools/kernel_stats_summary.py)"

    metric = METRIC if default_workload else (
        f"device-resident encode+{two} GiB/s, {args.ec_type} k={k} m={m}, {n} B objects"
        + (", inline_crc32" if args.inline_crc32 else ""))
    result = {
        "metric": metric,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch else "weak",
        "vs_baseline": None,
        "dtype": "u16" if w == 16 else "u8",
        "data": f"synthetic: PCG64(seed {SEED}+rank) uniform bytes; {args.erasures} random "
                "erasures per object for decode",
        "config": {"workload": f"{args.ec_type} k={k} m={m} encode + "
                               + (f"decode ({args.erasures} erasures)" if two == "decode"
                                  else "reconstruct (1 fragment)")
                               + f", {n} B objects, batch {B} per GPU, device-resident",
                   "k": k, "m": m, "object_bytes": n, "batch_per_gpu": B,
                   "erasures": args.erasures, "parallelism": f"objects sharded over {world} GPU"
                   + (" (all ranks on cuda:0)" if args.same_device and world > 1 else "")},
        "encode_GiBps": round(n_total * n / (enc_ms * 1e-3) / 2**30, 3),
        f"{two}_GiBps": round(n_total * n / (dec_ms * 1e-3) / 2**30, 3),
        "kernels": kernels,
        "roofline": roofline,
        "timing_events": args.events,
        "settle": {"ms": round(settle_ms, 1), "steps": settle_steps,
                   "note": "untimed steps before the warmup steps, until the GPU's clocks "
                           "settle (--settle-ms)"},
        "step_ms": {"encode": [round(events[2 * i].elapsed_time(events[2 * i + 1]), 4)
                               for i in range(args.steps)],
                    two: [round(events[2 * i + 1].elapsed_time(events[2 * i + 2]), 4)
                          for i in range(args.steps)]},
    }
    if args.same_device and world > 1:
        result["same_device"] = True

    # ---- erasures that change every step (untimed by the headline) ----
    fresh_ok = True
    if two == "decode" and args.fresh_steps > 0:
        fresh, fresh_ok = fresh_decode(args, codec, stripes, objs, out, stream, B, rank)
        result.update(fresh)
        steady, steady_ok = fresh_decode_steady(args, codec, stripes, objs, out, stream, B, rank,
                                                masks)
        result.update(steady)
        fresh_ok = fresh_ok and steady_ok
        # the headline batch is decoded again so the oracle check below sees it
        codec.decode(stripes, n, masks, out)
        torch.cuda.synchronize()

    # ---- full-stripe encode: liberasurecode_encode's whole output (k data +
    # m parity fragments, headers included) in one launch per batch; the
    # verification below then checks the stripes this leg wrote ----
    if args.full_stripe_steps > 0:
        ev_fs = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        par_ref = p_parity.clone()  # the headline (parity-only) encode's output
        stripes[:, :k].zero_()
        codec.encode(objs, n, parity=p_parity, data=stripes[:, :k])
        torch.cuda.synchronize()
        ev_fs[0].record(stream)
        for _ in range(args.full_stripe_steps):
            codec.encode(objs, n, parity=p_parity, data=stripes[:, :k])
        ev_fs[1].record(stream)
        torch.cuda.synchronize()
        fs_ms = ev_fs[0].elapsed_time(ev_fs[1]) / args.full_stripe_steps
        parity_same = bool(torch.equal(p_parity, par_ref))
        del par_ref
        fs_bytes = B * n + B * (k + m) * (bs + 80)
        result["encode_full_stripe_ms"] = round(fs_ms, 4)
        result["encode_full_stripe"] = {
            "bytes": fs_bytes, "GBps": round(fs_bytes / (fs_ms * 1e-3) / 1e9, 1),
            "frac": round(fs_bytes / (fs_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "launches": args.full_stripe_steps,
            "note": "k data + m parity fragments with headers per object in one launch, back "
                    "to back; these stripes are the ones the oracle check below compares"}

    # ---- inline_crc32 encode beside the plain one (round 6: the chunk CRCs on
    # the matrix cores): the same batch, parity only,
    # both back to back on this box, so the ratio is the CRC's cost; a
    # sample of headers checked against zlib's crc32 of their payloads.  An
    # auxiliary leg: recorded, never fatal to the headline ----
    if args.crc_steps > 0 and not args.inline_crc32 and args.ec_type in ("amd_rs_vand", "liberasurecode_rs_vand"):
        try:
            result["encode_inline_crc32"] = crc_encode_leg(args, codec, objs, n, k, m, bs, B, stream)
        except Exception as exc:  # noqa: BLE001
            result["encode_inline_crc32"] = {"error": repr(exc)[:300]}

    # ---- verification of the timed batch (every object), and the CPU baseline ----
    bad = []
    t_enc = t_two = None
    src = ""
    if not args.no_verify:
        gpu_frags = stripes[:, :, :fl].cpu().numpy()
        gpu_second = (out[:, :n] if two == "decode" else rec[:, :fl]).cpu().numpy()
        t_enc, t_two, bad, src = oracle_pass(args, host, two_masks, dests, gpu_frags,
                                             gpu_second, sample=B)
        del gpu_frags, gpu_second
    if not fresh_ok:
        bad.append((-1, "fresh-erasure decode"))
    if args.full_stripe_steps > 0 and not parity_same:
        bad.append((-1, "headline parity differs from the full-stripe encode's"))
    verified = bool(shard.min_over_ranks(0 if bad else 1)) and not args.no_verify
    result["verified"] = verified
    if not args.no_verify:
        result["verified_objects"] = n_total
    if bad:
        print(f"rank {rank}: {len(bad)} mismatches vs the oracle, first: {bad[:5]}",
              file=sys.stderr, flush=True)

    numa_all = numa
    if rank == 0:
        result["placement"] = {"rank0": numa, "cpu_affinity": len(os.sched_getaffinity(0))}
        from pyeclib_amd import system_liberasurecode
        result["system_liberasurecode"] = {
            "found": system_liberasurecode.probe(),
            "note": "ctypes.util.find_library('erasurecode') on this box (SURVEY 8(c) upgrade path); "
                    "when found, tests/test_system_liberasurecode.py pins the oracle and the GPU "
                    "path to its bytes"}

    if rank == 0 and not args.no_host and w == 16:
        result.update(host_resident(args, codec, host, stripes, masks, fs, bs))
        result.update(single_object_calls(args))
    if rank == 0 and args.config0:
        result.update(config0_cli(args))
    if rank == 0 and world == 1 and not args.no_host and w == 16:
        try:
            result.update(reference_cli_bench())
        except Exception as exc:  # noqa: BLE001 -- an auxiliary leg: recorded, not fatal
            result["reference_cli_bench"] = {"error": repr(exc)}
        try:
            result.update(first_call())
        except Exception as exc:  # noqa: BLE001 -- an auxiliary leg: recorded, not fatal
            result["first_call"] = {"error": repr(exc)}
    if rank == 0 and world == 1 and args.swift_procs and not args.no_host and w == 16:
        # the Swift call shape: P processes, one ECDriver call per segment
        # (this process holds the GPU too: at most 15 workers beside it)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import swift_calls
        procs = tuple(min(15, int(x)) for x in args.swift_procs.split(",") if x)
        rows = swift_calls.sweep(procs, (1 << 20, 4 << 20), args.swift_seconds)
        result["swift_calls"] = {
            f"{r['op']}_{r['size'] >> 20}MiB_P{r['procs']}":
                ({"error": r["error"]} if "error" in r else
                 {"GiBps": r["GiBps"], "us_per_call": r["us_per_call_median"]}) for r in rows}
        result["swift_calls_verified"] = all(r["verified"] for r in rows)
        result["swift_calls_note"] = (
            "P worker processes on this GPU, each its own ECDriver(10, 4, liberasurecode_rs_vand) "
            "calling encode (or decode, 4 data fragments missing) on its own pageable segment "
            f"back to back for {args.swift_seconds} s; aggregate segment GiB/s over the span from "
            "the first start to the last finish; us_per_call = median over processes; the "
            "callers' buffers staged through pinned memory (ECAMD_REGISTER_CALLER=1 uses them in place)")

    if rank == 0 and not args.no_cpu_baseline and (world == 1 or args.cpu_baseline_all):
        sample = min(args.cpu_sample or B, B)
        if t_enc is None or sample != B:
            t_enc, t_two, _, src = oracle_pass(args, host, two_masks, dests, sample=sample)
        # N = every CPU this process may run on (the whole
        # node's share after the NUMA binding), the objects split evenly;
        # the 16-worker figure (the box's CPU share per GPU) beside it
        affinity = len(os.sched_getaffinity(0))
        workers = max(1, min(affinity, sample))
        # each worker's share repeated to >= 16 object passes (~0.2 s at 4 MiB),
        # so start-up jitter across many processes does not set the time
        rep = max(1, -(-16 * workers // sample))
        st0 = cgroup_cpu_stat()
        t_par = cpu_parallel(args, host, two_masks, dests, sample, workers, rep)
        st1 = cgroup_cpu_stat()
        w16 = max(1, min(affinity, CPU_WORKERS_PER_GPU * world, sample))
        rep16 = max(1, -(-16 * w16 // sample))
        t_16 = cpu_parallel(args, host, two_masks, dests, sample, w16, rep16)
        st2 = cgroup_cpu_stat()

        def stat_delta(a, b, wall):
            # cgroup CPU time consumed (in CPUs) and throttling during a run
            d = {k: b[k] - a[k] for k in b if k in a}
            out = {"cpus_used": round(d["usage_usec"] / 1e6 / wall, 2)} if "usage_usec" in d else {}
            for k in ("nr_throttled", "throttled_usec", "nr_periods"):
                if k in d:
                    out[k] = d[k]
            return out
        one = 2 * sample * n / (t_enc + t_two) / 2**30
        v_all = 2 * sample * n * rep / t_par / 2**30
        v_16 = 2 * sample * n * rep16 / t_16 / 2**30
        # the better of the two is the baseline: on a box whose cgroup grants
        # fewer CPUs than the affinity mask lists, every-CPU runs throttle
        best_all = v_all >= v_16
        quota = cgroup_cpus()
        result["cpu_baseline"] = {
            "value": round(max(v_all, v_16), 4),
            "unit": "GiB/s", "cores": workers if best_all else w16, "kind": "port",
            "sample": f"{sample} objects x {n} B: encode + {two} ({src}, {args.ec_type}), "
                      f"the faster of {workers} single-threaded worker processes (every CPU "
                      f"of the process's affinity, each share {rep}x) and {w16} (each share "
                      f"{rep16}x); objects split evenly",
            "cpu_model": cpu_model(),
            "affinity_cpus": affinity,
            "cgroup_cpus": quota,
            "numa_node": numa_all.get("numa_node"),
            "value_all_affinity": round(v_all, 4),
            "value_16_workers": round(v_16, 4),
            "single_core_value": round(one, 4),
            "single_core_encode_GiBps": round(sample * n / t_enc / 2**30, 4),
            f"single_core_{two}_GiBps": round(sample * n / t_two / 2**30, 4),
            "single_core_seconds": round(t_enc + t_two, 2),
            "parallel_seconds": round(t_par, 3),
            "parallel_seconds_16_workers": round(t_16, 3),
            "cpu_env": cpu_env(),
            "cgroup_during_all_affinity_run": stat_delta(st0, st1, t_par),
            "cgroup_during_16_worker_run": stat_delta(st1, st2, t_16),
        }
    if rank == 0:
        print(json.dumps(result), flush=True)
    shard.finish()
    if not args.no_verify and not verified:
        sys.exit(3)


if __name__ == "__main__":
    main()
