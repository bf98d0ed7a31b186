"""The N>1 path on CPU: world_size-2 `gloo` process groups exercising the
sharding, the max-over-ranks timing and the per-flow histogram all-reduce that
bench.py runs over RCCL on GPUs (ingot_amd/dist.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from ingot_amd import REC_DTYPE, Chain, dist as idist
from tests.frames import build_frames, pack

N_PER_RANK = 1500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = build_frames(N_PER_RANK * world, seed=123)
        first, n = idist.shard(rank, world, N_PER_RANK)
        arena, off, lens = pack(frames[first:first + n])
        hist, _ = oracle.flow_hist(arena, off, lens, Chain.VlanUlp, bins=4096)
        t = torch.from_numpy(hist.astype(np.uint32).view(np.int32).copy())
        t2 = t.clone()
        idist.reduce_histogram(t)
        # the overlapped form bench.py uses: a handle, then wait()
        idist.reduce_histogram_async(t2).wait()
        assert torch.equal(t, t2)
        slowest = idist.max_over_ranks(0.5 + rank)
        if rank == 0:
            q.put((t.numpy().view(np.uint32).copy(), slowest))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_and_split():
    assert idist.shard(0, 4, 100) == (0, 100)
    assert idist.shard(3, 4, 100) == (300, 100)
    parts = [idist.split(1003, r, 4) for r in range(4)]
    assert sum(n for _, n in parts) == 1003
    assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(3))
    with pytest.raises(ValueError):
        idist.shard(4, 4, 1)


@pytest.mark.parametrize("world", [2, 4])
def test_histogram_allreduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    hist, slowest = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames = build_frames(N_PER_RANK * world, seed=123)
    arena, off, lens = pack(frames)
    want, _ = oracle.flow_hist(arena, off, lens, Chain.VlanUlp, bins=4096)
    assert (hist == want).all()
    assert slowest == 0.5 + (world - 1)


def _check_worker(rank, world, port, q):
    """bench.py's C5 checks at world 2: the per-rank region times, the
    process group's own world size / backend, and the reduced histogram
    against every rank's flow ids and Ok-with-L3 count."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        frames = build_frames(N_PER_RANK * world, seed=321)
        first, n = idist.shard(rank, world, N_PER_RANK)
        arena, off, lens = pack(frames[first:first + n])
        bins = 4096
        hist, _ = oracle.flow_hist(arena, off, lens, Chain.VlanUlp, bins=bins)
        fids = torch.from_numpy(oracle.flow_hist.last_flows.view(np.int32).copy())
        recs = oracle.parse_batch(arena, off, lens, Chain.VlanUlp).view(REC_DTYPE)
        ok_l3 = int(((recs["status"] == 0) & (recs["l3_kind"] != 0)).sum())
        h = torch.from_numpy(hist.astype(np.uint32).view(np.int32).copy())
        idist.reduce_histogram(h)
        good = idist.flow_hist_check(h, fids, ok_l3, bins)
        bad_h = h.clone()
        bad_h[7] += 1
        bad = idist.flow_hist_check(bad_h, fids, ok_l3, bins)
        times = idist.gather_over_ranks(1.0 + 0.25 * rank)
        info = idist.world_info()
        if rank == 0:
            q.put((good, bad, times, info))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_flow_hist_check_and_rank_report_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    good, bad, times, info = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert good["ok"] and good["bins_equal_allreduced_bincount"]
    assert good["hist_total"] == good["ok_l3_packets_all_ranks"] == \
        good["flow_ids_counted_all_ranks"] > 0
    assert not bad["ok"] and not bad["bins_equal_allreduced_bincount"]
    assert times == [1.0, 1.25]
    assert info == {"world_size": 2, "backend": "gloo", "process_group": True}


def test_rank_report_world_one():
    assert idist.gather_over_ranks(3.5) == [3.5]
    assert idist.world_info()["world_size"] == 1
    h = torch.tensor([2, 0, 1], dtype=torch.int32)
    f = torch.tensor([0, -1, 0, 2], dtype=torch.int32)
    r = idist.flow_hist_check(h, f, 3, 3)
    assert r["ok"] and r["hist_total"] == 3


class _CpuTorch:
    """torch for bench.FlowRunner / bench._timed on CPU: streams and events
    are no-ops; the histograms are real CPU tensors reduced over gloo."""

    class cuda:  # noqa: N801
        class Event:
            def __init__(self, enable_timing=False):
                pass

            def record(self, s=None):
                pass

            def elapsed_time(self, other):
                return 1.0

        @staticmethod
        def synchronize():
            pass

        class stream:  # noqa: N801
            def __init__(self, s):
                pass

            def __enter__(self):
                return self

            def __exit__(self, *a):
                return False

    uint8 = torch.uint8
    empty = staticmethod(torch.empty)


class _CpuStream:
    cuda_stream = 0

    def wait_event(self, ev):
        pass


class _Ptr:
    def __init__(self, i):
        self.i = i

    def data_ptr(self):
        return self.i


def _c5_subline_worker(rank, world, port, q):
    """The C5 sub-line's distributed plumbing at world 4 over gloo: the
    rank's shard (bench.frames_for_rank), the gate policy RCCL would get,
    bench.FlowRunner with the real async all-reduce (ingot_amd.dist) — the
    flows kernel stood in for by the oracle's flow ids over the first frames
    of the rank's own shard (the host generator, same bytes) — and the
    line's flow_hist_check, world info and max-over-ranks time."""
    import bench
    from ingot_amd import GenProfile
    from ingot_amd.hostgen import gen_frames_host

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, n, total = bench.frames_for_rank("c5", "weak", rank, world)
        policy = bench.gate_policy(True, world, "nccl", False)
        m, bins = 4096, bench.FLOW_BINS
        arena, off, lens = gen_frames_host(GenProfile.FLOWS, m, first=first)
        hist_np, _ = oracle.flow_hist(arena, off, lens, Chain.VlanUlp, bins=bins)
        fids = torch.from_numpy(oracle.flow_hist.last_flows.view(np.int32).copy())
        recs = oracle.parse_batch(arena, off, lens, Chain.VlanUlp).view(REC_DTYPE)
        ok_l3 = int(((recs["status"] == 0) & (recs["l3_kind"] != 0)).sum())
        reps = 4
        hists = [torch.zeros(bins, dtype=torch.int32) for _ in range(reps)]
        by_ptr = {h.data_ptr(): h for h in hists}
        log = []

        class _Lib:  # the flows kernel: this rank's histogram into `hist`
            def ingot_gpu_flow_hist_workspace_size(self, n, bins):
                return 0

            def ingot_gpu_flow_hist_ws(self, h, arena, optr, lptr, stride, n, c, key, nbins,
                                       flow, hashes, hist, work, wbytes, stream):
                log.append("kernel")
                if hist:
                    by_ptr[hist].copy_(torch.from_numpy(hist_np.view(np.int32)))
                return 0

        class _Ctx:
            _h = None

        class _Gate:
            def arm(self, streams):
                log.append("arm")

            def open(self):
                log.append("open")

        def reduce_fn(h):
            log.append("reduce")
            return idist.reduce_histogram_async(h)

        r = bench.FlowRunner(_CpuTorch, _Lib(), _Ctx(), Chain.VlanUlp, m,
                             [_Ptr(i + 1) for i in range(reps)], _Ptr(0), _Ptr(0), hists,
                             [_Ptr(0)] * reps, [_CpuStream(), _CpuStream()], reduce_fn,
                             open_before_collective=policy == "until_collective")
        steps = 6
        r.run(steps, gate=_Gate())
        # the last step's histogram, all-reduced, against every rank's flow ids
        check = idist.flow_hist_check(hists[(steps - 1) % reps], fids, ok_l3, bins)
        first_reduce = log.index("reduce")
        res = {"rank": rank, "first": first, "n": n, "total": total, "policy": policy,
               "open_before_first_reduce": "open" in log[:first_reduce],
               "reduces": log.count("reduce"), "check": check, "info": idist.world_info(),
               "slowest": idist.max_over_ranks(0.1 * (rank + 1))}
        out = [None] * world
        dist.all_gather_object(out, res)
        if rank == 0:
            q.put(out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_c5_subline_plumbing_world4_gloo():
    """before SCALE runs, the N>1 C5 path on the CPU side
    at world 4 — equal 8,388,608-frame shards, the until_collective gate
    opened before any all-reduce is enqueued, flow_hist_check ok on the
    all-reduced histogram, world size 4 in the line's distributed block."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 4
    procs = [ctx.Process(target=_c5_subline_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o["n"] for o in out] == [8_388_608] * world
    assert [o["first"] for o in out] == [r * 8_388_608 for r in range(world)]
    assert all(o["total"] == 8_388_608 * world for o in out)
    assert all(o["policy"] == "until_collective" for o in out)
    assert all(o["open_before_first_reduce"] and o["reduces"] == 6 for o in out)
    assert all(o["check"]["ok"] and o["check"]["bins_equal_allreduced_bincount"] for o in out)
    assert out[0]["check"]["hist_total"] == out[0]["check"]["ok_l3_packets_all_ranks"] > 0
    assert all(o["info"] == {"world_size": 4, "backend": "gloo", "process_group": True}
               for o in out)
    assert all(o["slowest"] == pytest.approx(0.4) for o in out)


def _comm_id_worker(rank, world, port, q):
    """idist.product_comm at world > 1 without a GPU: the library's
    communicator calls are replaced by recorders, so what is checked is the
    plumbing around them — rank 0 alone makes the id, every rank creates its
    communicator with that id, the group's size and its own rank, and fd 1
    is restored after the stdout redirect around RCCL's init."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ingot_amd

        made = []

        def fake_id():
            made.append(rank)
            return bytes([rank + 1]) * ingot_amd.COMM_ID_BYTES

        class FakeComm:
            def __init__(self, ctx, nranks, r, uid):
                self.args = (ctx, nranks, r, uid)

        ingot_amd.comm_unique_id = fake_id
        ingot_amd.Comm = FakeComm
        before = os.fstat(1)
        c = idist.product_comm("ctx")
        after = os.fstat(1)
        fd1 = (before.st_dev, before.st_ino) == (after.st_dev, after.st_ino)
        out = [None] * world
        dist.all_gather_object(out, (made, c.args[1:], fd1))
        if rank == 0:
            q.put(out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_product_comm_id_exchange_gloo():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_id_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    uid0 = bytes([1]) * 128
    for r, (made, (nranks, rank, uid), fd1) in enumerate(out):
        assert made == ([0] if r == 0 else [])  # only rank 0 makes the id
        assert (nranks, rank, uid) == (world, r, uid0)
        assert fd1


def test_product_comm_borrows_an_rccl_groups_communicator(monkeypatch):
    """A torch group over RCCL lends its communicator (Comm.from_process_group
    -> ingot_gpu_comm_wrap): no id is made and no second communicator is
    created.  The group's state is faked; the GPU side is
    tests/test_comm.py::test_borrowed_process_group_communicator."""
    import ingot_amd

    calls = []

    class FakeComm:
        def __init__(self, *a):
            calls.append(("create", a))

        @classmethod
        def from_process_group(cls, ctx, group=None):
            calls.append(("borrow", ctx))
            return "borrowed"

    monkeypatch.setattr(idist, "_active", lambda: True)
    monkeypatch.setattr(idist, "_gloo", lambda: False)
    monkeypatch.setattr(ingot_amd, "Comm", FakeComm)
    monkeypatch.setattr(ingot_amd, "comm_unique_id",
                        lambda: calls.append(("id",)) or b"\0" * 128)
    assert idist.product_comm("ctx") == "borrowed"
    assert calls == [("borrow", "ctx")]

