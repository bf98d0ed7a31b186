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


def gather_over_ranks(value: float, device=None) -> list:
    """Every rank's `value`, in rank order (all-gather; [value] at world 1)."""
    import torch
    import torch.distributed as dist

    if not _active():
        return [float(value)]
    dev = None if _gloo() else device
    t = torch.tensor([float(value)], dtype=torch.float64, device=dev)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def sum_over_ranks(t):
    """In-place SUM of an int64 tensor across ranks (through host memory on
    gloo); returns it.  World 1: unchanged."""
    import torch.distributed as dist

    if not _active():
        return t
    if _gloo() and t.is_cuda:
        host = t.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM)
        t.copy_(host)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def world_info() -> dict:
    """What the process group itself reports (not what the launcher asked
    for): world size and backend; world 1 without a process group."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
                "process_group": True}
    return {"world_size": 1, "backend": None, "process_group": False}


def flow_hist_check(hist, flow_ids, ok_l3_local: int, bins: int) -> dict:
    """Config 5's reduce, checked after the timed region on the buffers of one
    step: `hist` holds that step's histogram after the all-reduce, `flow_ids`
    this rank's per-packet bins of the same step (-1 = not counted).  Checks
    (1) the reduced histogram equals the all-reduce of every rank's bincount
    of its flow ids, bin for bin, and (2) its total equals the all-reduced
    count of Ok packets with an L3 layer (the packets the flow kernel counts,
    from this rank's parse records)."""
    import torch

    fid = flow_ids.to(torch.int64)
    counted = fid[fid >= 0]
    ref = torch.bincount(counted, minlength=bins)[:bins].to(torch.int64)
    sum_over_ranks(ref)
    exp = torch.tensor([int(ok_l3_local), int(counted.numel())], dtype=torch.int64,
                       device=ref.device)
    sum_over_ranks(exp)
    got = hist.view(torch.int32).to(torch.int64)
    total = int(got.sum().item())
    bins_equal = bool(torch.equal(got, ref))
    ok_l3, counted_all = (int(x) for x in exp.tolist())
    return {"hist_total": total, "ok_l3_packets_all_ranks": ok_l3,
            "flow_ids_counted_all_ranks": counted_all,
            "bins_equal_allreduced_bincount": bins_equal,
            "ok": bins_equal and total == ok_l3 == counted_all}


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


def product_comm(ctx):
    """The communicator of config 5's reduce, over the same ranks as the
    torch.distributed group.  A group over RCCL lends its own communicator
    (ingot_gpu_comm_wrap): one RCCL communicator per process, never two
    (DESIGN.md §6).  A gloo group carries rank 0's 128-byte id to every rank
    for the library's own (ingot_gpu_comm_create).  World 1 (no group): a
    one-rank communicator, so the reduce is the same RCCL call at every N."""
    import torch.distributed as dist

    import ingot_amd

    with _stdout_to_stderr():  # RCCL prints its version banner on stdout
        if _active() and not _gloo():
            return ingot_amd.Comm.from_process_group(ctx)
        if _active():
            obj = [ingot_amd.comm_unique_id() if dist.get_rank() == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            return ingot_amd.Comm(ctx, dist.get_world_size(), dist.get_rank(), obj[0])
        return ingot_amd.Comm(ctx, 1, 0, ingot_amd.comm_unique_id())


class _stdout_to_stderr:
    """File descriptor 1 pointed at fd 2 for the block: what native code
    prints there (RCCL's init banner) stays out of bench.py's one-line
    stdout."""

    def __enter__(self):
        import os
        import sys

        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        import os
        import sys

        sys.stdout.flush()
        os.dup2(self._saved, 1)
        os.close(self._saved)
        return False


class _StreamDone:
    """Completion of a reduce enqueued on the current stream: wait() orders
    the caller's current stream after it (an event, no host wait)."""

    def __init__(self, torch):
        self._torch = torch
        self.ev = torch.cuda.Event()
        self.ev.record()

    def wait(self):
        self._torch.cuda.current_stream().wait_event(self.ev)


def product_reduce(comm):
    """reduce_fn for the config-5 runner: ingot_gpu_flow_hist_allreduce of the
    step's histogram, enqueued on the step's stream after its flow kernels (the
    next steps' kernels on the other streams overlap it)."""
    import torch

    def reduce(hist):
        comm.allreduce_hist(hist)
        return _StreamDone(torch)

    return reduce
