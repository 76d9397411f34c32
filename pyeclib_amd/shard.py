"""Object sharding across GPUs (one process per GPU, torch.distributed).

Objects are independent, so a batch is partitioned into contiguous per-rank
ranges and every rank encodes / decodes its own range on its own device with
no collective on the data path (BASELINE north_star: "no RCCL collective
required").  The only collectives are bookkeeping -- a barrier around timed
regions, a MAX of the elapsed time and a MIN of the verification flag -- and
they run on a gloo group with CPU tensors, so no RCCL communicator is ever
created: the N-rank path works with any GPU mapping, including every rank on
one device (`device_for(..., same_device=True)`, for exercising the N-rank
code on a single leased GPU).
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


def device_index(local_rank: int, same_device: bool = False) -> int:
    """GPU ordinal of a rank: its local rank, or 0 for every rank when
    `same_device` (N ranks sharing one leased GPU)."""
    return 0 if same_device else local_rank


def init(backend: str = "gloo") -> tuple[int, int, int]:
    """Join the (bookkeeping) process group when launched with more than one
    rank.  gloo by default: the group carries three scalars per run."""
    world, rank, local = rank_info()
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group(backend, rank=rank, world_size=world)
    return world, rank, local


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def barrier() -> None:
    dist = _dist()
    if dist is not None:
        dist.barrier()


def _reduce(value, op_name: str, dtype):
    import torch
    dist = _dist()
    if dist is None:
        return value
    t = torch.tensor([value], dtype=dtype)  # CPU tensor: gloo
    dist.all_reduce(t, op=getattr(dist.ReduceOp, op_name))
    return t.item()


def max_over_ranks(value: float, device=None) -> float:
    """MAX of a scalar over all ranks (identity when not distributed).
    `device` is accepted for old callers and ignored: the reduction runs on
    CPU tensors."""
    return float(_reduce(float(value), "MAX", _float64()))


def min_over_ranks(value: int) -> int:
    """MIN of an integer over all ranks (e.g. an all-verified flag)."""
    return int(_reduce(int(value), "MIN", _int64()))


def sum_over_ranks(value: int) -> int:
    return int(_reduce(int(value), "SUM", _int64()))


def _float64():
    import torch
    return torch.float64


def _int64():
    import torch
    return torch.int64


def finish() -> None:
    dist = _dist()
    if dist is not None:
        dist.destroy_process_group()
