"""The N>1 path on CPU: world_size-2 gloo process group, objects sharded by
pyeclib_amd.shard, each rank encoding its own range (with the CPU oracle as
the stand-in codec -- no GPU here), digests gathered and compared with a
single-process encode of the whole batch; plus the MAX time reduction that
bench.py uses (MAX time, MIN verified flag, on CPU tensors: no RCCL)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from pyeclib_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _objects(n, size):
    rng = np.random.Generator(np.random.PCG64(7))
    return [rng.integers(0, 256, size, dtype=np.uint8).tobytes() for _ in range(n)]


def _digest(frags):
    return hashlib.sha256(b"".join(frags)).hexdigest()


def _worker(rank, world, port, n_obj, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    from oracle import oracle as O
    w, r, _ = shard.init("gloo")
    assert (w, r) == (world, rank)
    a, b = shard.shard_range(n_obj, r, w)
    objs = _objects(n_obj, 3000)
    mine = {i: _digest(O.encode(4, 2, objs[i])) for i in range(a, b)}
    gathered = [None] * w
    dist.all_gather_object(gathered, mine)
    t = shard.max_over_ranks(float(rank + 1))
    ok = shard.min_over_ranks(0 if rank == 1 else 1)
    total = shard.sum_over_ranks(b - a)
    shard.barrier()
    if rank == 0:
        merged = {}
        for part in gathered:
            merged.update(part)
        q.put((merged, t, ok, total))
    shard.finish()


def test_shard_range_partitions():
    for n in (0, 1, 7, 256, 1024):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)


def test_two_rank_gloo_sharded_encode():
    from oracle import oracle as O
    n_obj, world = 9, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_obj, q)) for r in range(world)]
    for p in procs:
        p.start()
    merged, tmax, ok, total = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    objs = _objects(n_obj, 3000)
    assert merged == {i: _digest(O.encode(4, 2, objs[i])) for i in range(n_obj)}
    assert tmax == 2.0 and ok == 0 and total == n_obj
