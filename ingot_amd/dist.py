"""Multi-GPU plumbing for the parse path: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on ROCm; "gloo" in CPU tests).

Packets are independent (ingot's parse is a pure per-packet function), so a
batch shards by contiguous index ranges with no data-path collective.  The only
exchange is config 5's per-flow histogram, summed across ranks; timing is the
max over ranks.
"""
from __future__ import annotations


def shard(rank: int, world: int, n_per_rank: int) -> tuple[int, int]:
    """Weak scaling: rank r owns frames [r*n, (r+1)*n) of the global stream."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return rank * n_per_rank, n_per_rank


def split(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Strong scaling: contiguous near-equal split of n_total frames."""
    base, extra = divmod(n_total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def _active():
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _gloo() -> bool:
    import torch.distributed as dist

    return dist.get_backend() == "gloo"


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    if not _active():
        return float(value)
    dev = None if _gloo() else device
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_histogram(hist):
    """In-place SUM of a per-rank flow histogram across ranks (RCCL all-reduce
    over xGMI on GPUs: 65,536 x u32 = 256 KiB, one ring pass).  torch has no
    uint32 collectives, so the buffer is reduced as int32: counts per launch are
    far below 2^31 and two's-complement addition is the same bit pattern."""
    import torch
    import torch.distributed as dist

    if not _active():
        return hist
    view = hist.view(torch.int32) if hist.dtype != torch.int32 else hist
    if _gloo() and view.is_cuda:  # rehearsal backend: reduce through host memory
        host = view.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM)
        view.copy_(host)
    else:
        dist.all_reduce(view, op=dist.ReduceOp.SUM)
    return hist


class _Done:
    def wait(self):
        return None


def reduce_histogram_async(hist):
    """As reduce_histogram, without making the caller's stream wait: returns
    a handle whose wait() orders the caller's current stream after the
    all-reduce (RCCL: the collective runs on its own stream, so the next
    batch's kernels overlap it).  The gloo rehearsal path completes at once."""
    import torch
    import torch.distributed as dist

    if not _active():
        return _Done()
    view = hist.view(torch.int32) if hist.dtype != torch.int32 else hist
    if _gloo():
        reduce_histogram(hist)
        return _Done()
    return dist.all_reduce(view, op=dist.ReduceOp.SUM, async_op=True)
