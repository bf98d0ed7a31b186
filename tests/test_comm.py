"""Config 5's histogram reduce behind the C ABI (ingot_gpu_comm_*,
ingot_gpu_flow_hist_allreduce: RCCL all-reduce, sum over uint32).

The reference has no collective; the reduce is the GPU
design's only exchange.  The argument checks run on the CPU.  On the GPU: a
one-rank communicator (the box has one GPU; RCCL refuses two ranks on one
device) reduces a histogram the flow kernel filled, and the result equals the
oracle's histogram; then bench.py's config-5 runner runs with the product
reduce under gate_policy "until_collective" and every reduce is issued only
after the region's doorbell has been rung."""
import ctypes

import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd import _lib


def test_comm_argument_errors():
    lib = _lib.load()
    out = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * ingot_amd.COMM_ID_BYTES)()
    assert lib.ingot_gpu_comm_unique_id(None) == -1
    assert lib.ingot_gpu_comm_create(None, 1, 0, uid, ctypes.byref(out)) == -1
    assert lib.ingot_gpu_flow_hist_allreduce(None, None, 1 << 16, None) == -1
    assert lib.ingot_gpu_comm_size(None) == -1 and lib.ingot_gpu_comm_rank(None) == -1
    assert lib.ingot_gpu_comm_destroy(None) == -1 and lib.ingot_gpu_comm_abort(None) == -1
    assert lib.ingot_gpu_comm_wrap(None, None, ctypes.byref(out)) == -1
    assert lib.ingot_gpu_strerror(-6) == b"collective (RCCL) call failed"
    with pytest.raises(ValueError):
        ingot_amd.Comm(None, 1, 0, b"short")


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


@pytest.fixture(scope="module")
def comm(ctx):
    c = ingot_amd.Comm(ctx, 1, 0, ingot_amd.comm_unique_id())
    yield c
    c.close()


@pytest.mark.gpu
def test_one_rank_allreduce_equals_the_oracle(torch, ctx, comm):
    assert (comm.size, comm.rank) == (1, 0)
    n, bins = 200_003, 1 << 16
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=77)
    hist = torch.zeros(bins, dtype=torch.int32, device="cuda")
    ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n,
                  workspace=ctx.flow_hist_workspace(n, bins))
    comm.allreduce_hist(hist)
    torch.cuda.synchronize()
    w_hist, _ = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                                 Chain.VlanUlp, n=n, bins=bins)
    got = hist.cpu().numpy().view(np.uint32)
    assert got.sum() > 0 and (got == w_hist).all()
    # enqueued on a side stream, ordered after the work already there
    s = torch.cuda.Stream()
    h2 = torch.zeros(bins, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(s):
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=h2, n=n)
        comm.allreduce_hist(h2)
    torch.cuda.synchronize()
    assert (h2.cpu().numpy().view(np.uint32) == w_hist).all()


@pytest.mark.gpu
def test_allreduce_argument_errors(torch, comm):
    lib = _lib.load()
    h = torch.zeros(1000, dtype=torch.int32, device="cuda")
    assert lib.ingot_gpu_flow_hist_allreduce(comm._h, h.data_ptr(), 1000, None) == -5
    assert lib.ingot_gpu_flow_hist_allreduce(comm._h, None, 1024, None) == -1
    assert lib.ingot_gpu_flow_hist_allreduce(comm._h, h.data_ptr(), 1 << 25, None) == -5
    assert lib.ingot_gpu_flow_hist_allreduce(comm._h, h.data_ptr(), 0, None) == -5
    big = torch.ones(1 << 24, dtype=torch.int32, device="cuda")  # the largest table
    comm.allreduce_hist(big)
    torch.cuda.synchronize()
    assert int(big.sum()) == 1 << 24
    with pytest.raises(ValueError):
        comm.allreduce_hist(torch.zeros(1024, dtype=torch.int64, device="cuda"))


@pytest.mark.gpu
def test_comm_create_argument_errors(torch, ctx):
    import ctypes

    lib = _lib.load()
    a, b = ingot_amd.comm_unique_id(), ingot_amd.comm_unique_id()
    assert a != b  # a fresh id per call
    buf = (ctypes.c_uint8 * ingot_amd.COMM_ID_BYTES).from_buffer_copy(a)
    out = ctypes.c_void_p()
    for nranks, rank in ((0, 0), (1, 1), (2, -1), (2, 2)):
        assert lib.ingot_gpu_comm_create(ctx._h, nranks, rank, buf, ctypes.byref(out)) == -1
        assert not out.value
    assert lib.ingot_gpu_comm_create(ctx._h, 1, 0, None, ctypes.byref(out)) == -1
    assert lib.ingot_gpu_comm_create(ctx._h, 1, 0, buf, None) == -1
    # abort releases a one-rank communicator at once
    c = ingot_amd.Comm(ctx, 1, 0, b)
    c.abort()
    c.abort()  # the handle is gone: a no-op


@pytest.mark.gpu
def test_flow_runner_until_collective_with_the_product_reduce(torch, ctx, comm):
    """bench.py's config-5 step (flow kernel, histogram pass, then the reduce
    through ingot_gpu_flow_hist_allreduce) under gate_policy
    "until_collective": no reduce is enqueued while the region's doorbell is
    unrung, and the last step's reduced histogram passes flow_hist_check."""
    import bench
    from ingot_amd import dist as idist

    assert bench.gate_policy(True, 1, "nccl", False) == "until_collective"
    lib = _lib.load()
    n, reps, steps = 131_072, 4, 12
    bins = bench.FLOW_BINS
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=3)
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    hists = [torch.zeros(bins, dtype=torch.int32, device="cuda") for _ in range(reps)]
    flows = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(reps)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    gate = bench.Gate(ingot_amd, ctx)
    rung = []
    open_ = gate.open

    def opened():
        rung.append(gate.seq)
        open_()

    gate.open = opened
    red = idist.product_reduce(comm)
    issued_after_ring = []

    def reduce_fn(h):
        issued_after_ring.append(bool(rung) and rung[-1] == gate.seq)
        return red(h)

    runner = bench.FlowRunner(torch, lib, ctx, Chain.VlanUlp, n, arenas, off, lens, hists, flows,
                              streams, reduce_fn, open_before_collective=True)
    runner.run(4)  # warm-up, ungated
    issued_after_ring.clear()
    ms, _ = runner.run(steps, gate)
    torch.cuda.synchronize()
    assert ms > 0 and len(issued_after_ring) == steps and all(issued_after_ring)
    recs = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, Chain.VlanUlp))
    ok_l3 = int(((recs["status"] == 0) & (recs["l3_kind"] != 0)).sum())
    last = (steps - 1) % reps
    chk = idist.flow_hist_check(hists[last], flows[last], ok_l3, bins)
    assert chk["ok"], chk
    w_hist, _ = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                                 Chain.VlanUlp, n=n, bins=bins)
    assert (hists[last].cpu().numpy().view(np.uint32) == w_hist).all()


@pytest.mark.gpu
def test_borrowed_process_group_communicator(torch, ctx):
    """ingot_gpu_comm_wrap: the reduce over the communicator of torch's own
    RCCL group (one communicator per process).  Releasing the
    handle leaves the group's communicator working."""
    import torch.distributed as dist

    from ingot_amd import dist as idist

    lib = _lib.load()
    out = ctypes.c_void_p()
    assert lib.ingot_gpu_comm_wrap(ctx._h, None, ctypes.byref(out)) == -1
    assert not dist.is_initialized()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        c = ingot_amd.Comm.from_process_group(ctx)
        assert (c.size, c.rank) == (1, 0)
        ptr = dist.group.WORLD._get_backend(torch.device("cuda:0"))._comm_ptr()
        assert lib.ingot_gpu_comm_wrap(ctx._h, ctypes.c_void_p(ptr), None) == -1
        n, bins = 100_000, 1 << 16
        arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=5)
        hist = torch.zeros(bins, dtype=torch.int32, device="cuda")
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n)
        c.allreduce_hist(hist)
        torch.cuda.synchronize()
        w_hist, _ = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(),
                                     lens.cpu().numpy(), Chain.VlanUlp, n=n, bins=bins)
        assert (hist.cpu().numpy().view(np.uint32) == w_hist).all()
        c.close()  # the handle only
        c.close()
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)  # the group's communicator still works
        torch.cuda.synchronize()
        assert t.tolist() == [1.0] * 4
        # bench's product_comm at world 1 with a group: its own one-rank
        # communicator (a group of one is not "active")
        c1 = idist.product_comm(ctx)
        assert (c1.size, c1.rank) == (1, 0)
        c1.close()
    finally:
        dist.destroy_process_group()
