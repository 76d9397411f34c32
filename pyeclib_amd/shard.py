"""Object sharding across GPUs (one process per GPU, torch.distributed).

Objects are independent, so a batch is partitioned into contiguous per-rank
ranges and every rank encodes / decodes its own range on its own device with
no collective on the data path.  The only collectives are bookkeeping: a
barrier around timed regions and a MAX reduction of the elapsed time
(bench.py), both tiny.
"""
from __future__ import annotations

import os


def rank_info() -> tuple[int, int, int]:
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Balanced contiguous partition: ranks get floor or ceil of n/world."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_items, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def init(backend: str | None = None) -> tuple[int, int, int]:
    """Join the process group when launched with more than one rank."""
    world, rank, local = rank_info()
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend or "nccl", rank=rank, world_size=world)
    return world, rank, local


def barrier() -> None:
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a scalar over all ranks (identity when not distributed)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
