"""Concurrent instances and streams, on the GPU through the C ABI.

pyeclib creates and drives instances from several threads at once
(test/test_pyeclib_api.py:192-218; the GIL is released on free-threaded
builds, src/pyeclib_c/pyeclib_c.c:1245-1251), and ctypes releases the GIL
around every call into libpyeclib_amd.so.  The runtime therefore never waits
for the whole device: a buffer an instance rewrites (its decode table pool,
its cached descriptors) is ordered after the launches of THAT instance, on the
streams they were queued on (ec_runtime.cpp Instance::order_after_streams).
These tests run two instances on two threads and streams at once -- one with a
5-slot table pool, so every call recycles it several times -- and the staged
host pipeline, whose chunks are dealt over three streams and reuse table sets
staged by another stream's chunk.  Every output is checked.
"""
import os
import random
import sys
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _objects(B, n, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    host = np.zeros((B, (n + 255) // 256 * 256), dtype=np.uint8)
    host[:, :n] = rng.integers(0, 256, size=(B, n), dtype=np.uint8)
    return host


def _worker(codec, k, m, n, host, calls, seed, stream, errors, label, oracle):
    import torch
    from pyeclib_amd import batch
    try:
        rng = random.Random(seed)
        B = host.shape[0]
        full = (1 << (k + m)) - 1
        with torch.cuda.stream(stream):
            bs = codec.blocksize(n)
            objs = torch.from_numpy(host).to(stream.device, non_blocking=False)
            stripes = batch.stripe_buffer(B, k, m, bs, device=stream.device)
            codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
            stream.synchronize()
            want0 = oracle.encode(k, m, host[0, :n].tobytes())
            got0 = stripes[0, :, :80 + bs].cpu().numpy()
            if any(got0[i].tobytes() != want0[i] for i in range(k + m)):
                errors.append(f"{label}: encode differs from the oracle")
                return
            ref = stripes.clone()
            for call in range(calls):
                masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), m))
                         for _ in range(B)]
                out = torch.zeros_like(objs)
                codec.decode(stripes, n, masks, out)
                dest = [rng.randrange(k + m) for _ in range(B)]
                rmasks = [full & ~(1 << d) & ~(1 << ((d + 1 + o) % (k + m)))
                          for o, d in enumerate(dest)]
                rec = torch.zeros((B, stripes.shape[2]), dtype=torch.uint8, device=stream.device)
                codec.reconstruct(stripes, n, rmasks, dest, rec)
                stream.synchronize()
                if not torch.equal(out[:, :n], objs[:, :n]):
                    errors.append(f"{label}: decode differs in call {call}")
                    return
                for o in range(B):
                    if not torch.equal(rec[o, :80 + bs], ref[o, dest[o], :80 + bs]):
                        errors.append(f"{label}: reconstruct differs in call {call}, object {o}")
                        return
    except Exception as exc:  # noqa: BLE001 -- reported by the test
        errors.append(f"{label}: {exc!r}")


def test_two_instances_two_threads_one_recycling(gpu, oracle, monkeypatch):
    """Instance A (k=28 m=4, pool forced to 5 table-set slots: C(32,4) patterns,
    so each call recycles the pool several times) and instance B (k=10 m=4,
    default pool) decode and reconstruct batches with erasures drawn anew every
    call, concurrently, from two threads on two streams."""
    import torch
    from pyeclib_amd import batch
    monkeypatch.setenv("ECAMD_POOL_SLOTS", "5")
    codec_a = batch.BatchCodec(28, 4)
    monkeypatch.delenv("ECAMD_POOL_SLOTS")
    codec_b = batch.BatchCodec(10, 4)
    na, nb = 28 * 2 * 3000 + 6, (1 << 20) + 10
    host_a, host_b = _objects(23, na, 1), _objects(40, nb, 2)
    sa, sb = torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)
    errors = []
    ta = threading.Thread(target=_worker, args=(codec_a, 28, 4, na, host_a, 6, 11, sa, errors,
                                                "A(k=28, 5 slots)", oracle))
    tb = threading.Thread(target=_worker, args=(codec_b, 10, 4, nb, host_b, 6, 12, sb, errors,
                                                "B(k=10)", oracle))
    ta.start()
    tb.start()
    ta.join(timeout=240)
    tb.join(timeout=240)
    assert not ta.is_alive() and not tb.is_alive(), "worker hung"
    assert errors == []


def test_one_instance_two_threads_shared_pool(gpu, oracle):
    """One instance driven from two threads on two streams: the calls are
    serialised by the instance, but their launches interleave on the GPU, and
    each call's table copies and cached descriptors must be ordered after the
    other stream's launches that still read the old ones."""
    import torch
    from pyeclib_amd import batch
    codec = batch.BatchCodec(10, 4)
    n = (256 << 10) + 6
    host1, host2 = _objects(64, n, 3), _objects(64, n, 4)
    s1, s2 = torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)
    errors = []
    t1 = threading.Thread(target=_worker, args=(codec, 10, 4, n, host1, 8, 21, s1, errors, "t1",
                                                oracle))
    t2 = threading.Thread(target=_worker, args=(codec, 10, 4, n, host2, 8, 22, s2, errors, "t2",
                                                oracle))
    t1.start()
    t2.start()
    t1.join(timeout=240)
    t2.join(timeout=240)
    assert not t1.is_alive() and not t2.is_alive(), "worker hung"
    assert errors == []


@pytest.mark.parametrize("second", ["decode", "reconstruct"])
def test_staged_pipeline_reuses_patterns_across_streams(gpu, oracle, monkeypatch, second):
    """The staged host pipeline (ECAMD_HOST_STAGED=1) deals chunks of 3
    objects over 3 streams.  Chunk c's first object brings a new erasure
    pattern, its second reuses the pattern chunk c-1 brought (staged by a copy
    on another stream) and its third chunk c-2's -- the case where a launch
    could read a table slot before another stream's copy of it has landed."""
    import torch
    from pyeclib_amd import batch
    monkeypatch.setenv("ECAMD_HOST_STAGED", "1")
    monkeypatch.setenv("ECAMD_HOST_CHUNK_MB", "1")
    k, m, n, B = 10, 4, 256 << 10, 27
    codec = batch.BatchCodec(k, m)
    bs = codec.blocksize(n)
    fs = batch.frag_stride(bs)
    fl = 80 + bs
    assert (1 << 20) // (k * fs) == 3  # 3 objects per chunk
    host = _objects(B, n, 5)
    rng = random.Random(9)
    full = (1 << (k + m)) - 1
    frags = [oracle.encode(k, m, host[o, :n].tobytes()) for o in range(B)]
    seen = set()
    for rep in range(3):  # new patterns every repetition: every chunk stages tables again
        fresh = []
        while len(fresh) < B // 3:
            mk = full & ~sum(1 << i for i in rng.sample(range(k + m), m))
            if mk not in seen:
                seen.add(mk)
                fresh.append(mk)
        masks = []
        for c in range(B // 3):
            masks += [fresh[c], fresh[max(c - 1, 0)], fresh[max(c - 2, 0)]]
        hfr = torch.zeros((B, k, fs), dtype=torch.uint8).pin_memory()
        for o in range(B):
            idx = [i for i in range(k + m) if masks[o] >> i & 1][:k]
            for c, i in enumerate(idx):
                hfr[o, c, :fl] = torch.frombuffer(bytearray(frags[o][i]), dtype=torch.uint8)
        if second == "decode":
            out = torch.zeros((B, host.shape[1]), dtype=torch.uint8).pin_memory()
            codec.decode_host(hfr, n, masks, out)
            assert torch.equal(out[:, :n], torch.from_numpy(host[:, :n])), rep
        else:
            dest = [next(i for i in range(k + m) if not masks[o] >> i & 1) for o in range(B)]
            rec = torch.zeros((B, fs), dtype=torch.uint8).pin_memory()
            codec.reconstruct_host(hfr, n, masks, dest, rec)
            for o in range(B):
                assert rec[o, :fl].numpy().tobytes() == frags[o][dest[o]], (rep, o)


def test_destroyed_caller_streams(gpu, oracle, monkeypatch):
    """A caller may destroy its stream once a call on it has returned (round-4
    advice): calls on a stream created and destroyed per call, on one
    instance with a 5-slot table pool -- so later calls recycle the pool
    (and rewrite cached descriptors) after launches queued on streams that
    no longer exist -- never touch those handles, and every output is right."""
    import ctypes
    import torch
    from pyeclib_amd import batch
    monkeypatch.setenv("ECAMD_POOL_SLOTS", "5")
    import importlib.util
    lib = os.path.join(importlib.util.find_spec("torch").submodule_search_locations[0], "lib",
                       "libamdhip64.so")
    hip = ctypes.CDLL(lib if os.path.exists(lib) else "libamdhip64.so")  # the loaded runtime
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    k, m, n, B = 10, 4, (64 << 10) + 10, 12
    codec = batch.BatchCodec(k, m)
    host = _objects(B, n, 7)
    objs = torch.from_numpy(host).to(gpu)
    stripes = batch.stripe_buffer(B, k, m, codec.blocksize(n), device=gpu)
    codec.encode(objs, n, parity=stripes[:, k:], data=stripes[:, :k])
    torch.cuda.synchronize()
    rng = random.Random(11)
    full = (1 << (k + m)) - 1
    for call in range(40):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        masks = [full & ~sum(1 << i for i in rng.sample(range(k + m), m)) for _ in range(B)]
        if call % 3 == 0:  # the same masks twice in a row: the cached descriptor path
            masks = prev if call else masks
        prev = masks
        out = torch.zeros_like(objs)
        torch.cuda.synchronize()
        codec.decode(stripes, n, masks, out, stream=s.value)
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        assert torch.equal(out[:, :n].cpu(), torch.from_numpy(host[:, :n])), call


def test_stream_marks_stay_bounded(gpu, oracle):
    """Round-5 advice: an encode-only caller that takes a new stream per call
    (header cache resident, no pool recycle) once grew the instance's stream
    end marks by one event per call.  300 encodes, each on a stream created
    and destroyed around the call: the marks stay bounded
    (ecamd_instance_stats) and every parity row matches the oracle's."""
    import ctypes
    import torch
    from pyeclib_amd import _native, batch
    import importlib.util
    lib = os.path.join(importlib.util.find_spec("torch").submodule_search_locations[0], "lib",
                       "libamdhip64.so")
    hip = ctypes.CDLL(lib if os.path.exists(lib) else "libamdhip64.so")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    k, m, n, B = 10, 4, (64 << 10) + 10, 4
    codec = batch.BatchCodec(k, m)
    host = _objects(B, n, 9)
    objs = torch.from_numpy(host).to(gpu)
    stripes = batch.stripe_buffer(B, k, m, codec.blocksize(n), device=gpu)
    torch.cuda.synchronize()
    peak = 0
    for call in range(300):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        codec.encode(objs, n, parity=stripes[:, k:], stream=s.value)
        assert hip.hipStreamSynchronize(s) == 0
        assert hip.hipStreamDestroy(s) == 0
        peak = max(peak, _native.instance_stats(codec.handle)["marks"])
    assert peak <= 20, peak
    want = oracle.encode(k, m, host[0, :n].tobytes())
    got = stripes[0].cpu().numpy()
    fl = 80 + codec.blocksize(n)
    for i in range(k, k + m):
        assert got[i, :fl].tobytes() == want[i], i
