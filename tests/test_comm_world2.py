"""Config 5's product reduce at world 2 with real RCCL kernels, on the one GPU
of the test box.

RCCL refuses two ranks on one device ("Duplicate GPU"), judged by host
identity and bus id; NCCL_HOSTID gives each rank its own host identity, and
with P2P, SHM and InfiniBand off the two ranks talk over the loopback socket
transport.  Both ranks' RCCL kernels then run on the same GPU.  The rates are
meaningless; what runs is the N > 1 product path the driver's SCALE run
takes: rank 0's id carried to rank 1 (idist.product_comm over a gloo group),
ingot_gpu_comm_create at world 2, ingot_gpu_flow_hist_allreduce of each
rank's flow-kernel histogram (its contiguous shard of the C5 stream), and
bench.py's C5 FlowRunner under gate_policy "until_collective" — every reduce
issued after the region's doorbell, no rank left waiting.  The reduced
histogram equals the oracle's histogram of both shards, bin for bin.

INGOT_WORLD2_PG=nccl runs the torch group over RCCL instead, and
product_comm then borrows its communicator (ingot_gpu_comm_wrap): one RCCL
communicator per process either way (DESIGN.md §6 has why)."""
import os
import socket

import numpy as np
import pytest

N = 65_536
BINS = 1 << 16


def _rank_env():
    import bench

    return bench.REHEARSAL_ENV


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import faulthandler

    faulthandler.dump_traceback_later(40, repeat=True)  # a stalled rank shows where
    os.environ.update(_rank_env())
    os.environ["NCCL_HOSTID"] = f"ingot-rehearsal-rank{rank}"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import bench
    import ingot_amd
    from ingot_amd import Chain, GenProfile
    from ingot_amd import dist as idist

    # INGOT_WORLD2_PG=nccl: the torch group over RCCL, whose communicator
    # product_comm borrows (ingot_gpu_comm_wrap, still one per process);
    # default gloo
    backend = os.environ.get("INGOT_WORLD2_PG", "gloo")
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda:0"))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {"rank": rank}
    try:
        ctx = ingot_amd.Context(0)
        comm = idist.product_comm(ctx)
        res["comm"] = (comm.size, comm.rank)
        arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, N, first=rank * N)
        hist = torch.zeros(BINS, dtype=torch.int32, device="cuda")
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=N,
                      workspace=ctx.flow_hist_workspace(N, BINS))
        comm.allreduce_hist(hist)
        torch.cuda.synchronize()
        res["hist"] = hist.cpu().numpy().view(np.uint32).copy()

        # bench's C5 step at world 2: the product reduce under "until_collective"
        reps, steps = 4, 8
        arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
        hists = [torch.zeros(BINS, dtype=torch.int32, device="cuda") for _ in range(reps)]
        flows = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(reps)]
        streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
        gate = bench.Gate(ingot_amd, ctx)
        rung = []
        open_ = gate.open

        def opened():
            rung.append(gate.seq)
            open_()

        gate.open = opened
        red = idist.product_reduce(comm)
        after_ring = []

        def reduce_fn(h):
            after_ring.append(bool(rung) and rung[-1] == gate.seq)
            return red(h)

        policy = bench.gate_policy(True, world, "nccl", False)
        runner = bench.FlowRunner(torch, ingot_amd.load_library(), ctx, Chain.VlanUlp, N, arenas,
                                  off, lens, hists, flows, streams, reduce_fn,
                                  open_before_collective=policy == "until_collective")
        runner.run(2)
        after_ring.clear()
        ms, _ = runner.run(steps, gate)
        torch.cuda.synchronize()
        recs = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, Chain.VlanUlp))
        ok_l3 = int(((recs["status"] == 0) & (recs["l3_kind"] != 0)).sum())
        last = (steps - 1) % reps
        res["runner"] = {"policy": policy, "ms": ms, "reduces": len(after_ring),
                         "all_after_ring": all(after_ring),
                         "check": idist.flow_hist_check(hists[last], flows[last], ok_l3, BINS),
                         "hist": hists[last].cpu().numpy().view(np.uint32).copy()}
        comm.close()
        res["closed"] = True
    except Exception as e:  # reported to the test, which fails on it
        res["error"] = repr(e)
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_product_reduce_world2_on_one_gpu():
    import torch
    import torch.multiprocessing as mp

    import oracle
    from ingot_amd import Chain, GenProfile
    from ingot_amd.hostgen import gen_frames_host

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = q.get(timeout=100)
        for p in procs:
            p.join(timeout=30)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not any("error" in o for o in out), [o.get("error") for o in out]
    want = np.zeros(BINS, np.uint32)
    for r in range(world):
        a, o, ln = gen_frames_host(GenProfile.FLOWS, N, first=r * N)
        oracle.flow_hist(a, o, ln, Chain.VlanUlp, bins=BINS, hist=want)
    assert want.sum() > 0
    for r, o in enumerate(out):
        assert o["comm"] == (world, r)
        assert (o["hist"] == want).all()  # both shards, summed by RCCL
        ru = o["runner"]
        assert ru["policy"] == "until_collective"
        assert ru["reduces"] == 8 and ru["all_after_ring"]
        assert ru["check"]["ok"], ru["check"]
        assert (ru["hist"] == want).all()
