"""The persistent ring consumer (ingot_gpu_parse_ring): one launch over up to
64 batches of fixed slots returns, for every batch, exactly the records of
ingot_gpu_parse_strided over that batch and of the oracle — for every chain,
record width, grid (INGOT_TUNE_RING_GRID), depth (INGOT_TUNE_PIPE_DEPTH) and
cache policy, ragged batch sizes, and BASELINE configs[1]'s full batches as
bench.py times them (20 x 1 M frames over the rotated arena copies).  The
in-kernel doorbell: batches published one by one by a host thread are parsed
correctly, and a batch never published makes the waves give up after the
timeout (status bit set, its records untouched) instead of hanging.
Needs an MI355X."""
import threading
import time

import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd.abi import TUNE_CACHE_POLICY, TUNE_PIPE_DEPTH, TUNE_RING_GRID, TUNE_RING_GROUPS

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _batches(torch, prof, n, stride, k, seed=7):
    return [ingot_amd.gen_frames(prof, n, seed=seed + b, stride=stride)[0] for b in range(k)]


def _want(arena, chain, stride, n):
    return oracle.parse_batch(arena.cpu().numpy(), None, None, chain, stride=stride, n=n,
                              nthreads=8)


@pytest.mark.parametrize("grid,depth,pol,groups", [
    (0, 0, 0, 0), (1, 0, 0, 0), (4, 0, 0, 0), (8, 0, 0, 0), (0, 3, 0, 0), (0, 4, 0, 0),
    (2, 3, 1, 0), (0, 0, 4, 0), (0, 0, 3, 0), (3, 4, 75, 0), (0, 0, 0, 2), (4, 0, 0, 4),
    (3, 3, 0, 2), (1, 0, 0, 4)])
@pytest.mark.parametrize("n", [1, 63, 65, 4097, 100_003])
def test_ring_bit_exact(torch, grid, depth, pol, groups, n):
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_RING_GRID, grid)
    ctx.set_tuning(TUNE_RING_GROUPS, groups)
    ctx.set_tuning(TUNE_PIPE_DEPTH, depth)
    ctx.set_tuning(TUNE_CACHE_POLICY, pol)
    for prof, stride, k in ((GenProfile.V4UDP64, 64, 5), (GenProfile.ADVERSARIAL, 64, 3),
                            (GenProfile.MIXED, 128, 2)):
        arenas = _batches(torch, prof, n, stride, k, seed=n + grid)
        for chain in (Chain.UdpParser, Chain.GenericUlp, Chain.VlanUlp):
            outs = [torch.full((n, 16), 0xAB, dtype=torch.uint8, device="cuda") for _ in arenas]
            outs8 = [torch.full((n, 8), 0xAB, dtype=torch.uint8, device="cuda") for _ in arenas]
            ctx.parse_ring(arenas, stride, n, chain, outs)
            ctx.parse_ring(arenas, stride, n, chain, outs8, record_bytes=8)
            torch.cuda.synchronize()
            for a, o, o8 in zip(arenas, outs, outs8):
                want = _want(a, chain, stride, n)
                assert o.cpu().numpy().tobytes() == want.tobytes(), (prof, chain)
                assert o8.cpu().numpy().tobytes() == ingot_amd.rec16_to_rec8(want).tobytes()


def test_ring_equals_per_batch_launches_and_aliased_batches(torch):
    """A batch list may name the same arena twice (the bench rotates copies);
    every batch's records equal a single-batch parse of its arena."""
    ctx = ingot_amd.Context(0)
    n = 50_000
    arenas = _batches(torch, GenProfile.ADVERSARIAL, n, 64, 3, seed=99)
    seq = [arenas[b % 3] for b in range(64)]
    outs = [torch.zeros((n, 16), dtype=torch.uint8, device="cuda") for _ in seq]
    ctx.parse_ring(seq, 64, n, Chain.GenericUlp, outs)
    singles = [ctx.parse_strided(a, 64, n, Chain.GenericUlp) for a in arenas]
    torch.cuda.synchronize()
    for b, o in enumerate(outs):
        assert torch.equal(o, singles[b % 3]), b


def test_ring_full_bench_workload(torch):
    """BASELINE configs[1] as bench.py's ring mode times it: 20 batches of
    1,048,576 x 64-B Eth/IPv4/UDP frames over 8 rotated arena copies, every
    batch's records against the oracle."""
    ctx = ingot_amd.Context(0)
    n = 1 << 20
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    copies = [arena] + [arena.clone() for _ in range(7)]
    outs = [torch.zeros((n, 16), dtype=torch.uint8, device="cuda") for _ in range(20)]
    ctx.parse_ring([copies[b % 8] for b in range(20)], 64, n, Chain.UdpParser, outs)
    torch.cuda.synchronize()
    want = _want(arena, Chain.UdpParser, 64, n).tobytes()
    for b, o in enumerate(outs):
        assert o.cpu().numpy().tobytes() == want, b


def test_ring_rejects_bad_arguments(torch):
    ctx = ingot_amd.Context(0)
    a = torch.zeros(64 * 128, dtype=torch.uint8, device="cuda")
    o = torch.zeros((128, 16), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        ctx.parse_ring([a] * 65, 64, 128, Chain.UdpParser, [o] * 65)
    with pytest.raises(RuntimeError):  # slots < 64 B
        ctx.parse_ring([a], 32, 128, Chain.UdpParser, [o])
    with pytest.raises(RuntimeError):  # the tunnel chain has no ring kernel
        ctx.parse_ring([a], 64, 128, Chain.GeneveOverV6Tunnel, [o])
    with pytest.raises(RuntimeError):  # 8-B records need 8-B outputs; 12 is no width
        ctx.parse_ring([a], 64, 128, Chain.UdpParser, [o], record_bytes=12)
    db = ingot_amd.Doorbell(ctx)
    with pytest.raises(RuntimeError):  # a doorbell needs a bounded wait
        ctx.parse_ring([a], 64, 128, Chain.UdpParser, [o], doorbell=db, timeout_ms=0)
    db.close()
    ctx.parse_ring([], 64, 128, Chain.UdpParser, [])  # nothing to do


def test_ring_doorbell_publishes_batches_one_by_one(torch):
    """The launch starts before any batch is published; a host thread
    publishes batch b (copying its frames in first) every few ms.  Every
    batch's records are right and the launch ends after the last ring."""
    ctx = ingot_amd.Context(0)
    n, k = 200_000, 6
    src = _batches(torch, GenProfile.ADVERSARIAL, n, 64, k, seed=5)
    dst = [torch.zeros_like(a) for a in src]  # filled only after the launch started
    outs = [torch.zeros((n, 16), dtype=torch.uint8, device="cuda") for _ in range(k)]
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    db = ingot_amd.Doorbell(ctx)
    torch.cuda.synchronize()
    ring_s = torch.cuda.Stream()
    copy_s = torch.cuda.Stream()
    first = 100
    rung = []

    def producer():
        for b in range(k):
            time.sleep(0.005)
            with torch.cuda.stream(copy_s):
                dst[b].copy_(src[b])
            copy_s.synchronize()
            db.ring(first + b)
            rung.append(time.perf_counter())

    end = torch.cuda.Event()
    try:
        ctx.parse_ring(dst, 64, n, Chain.GenericUlp, outs, doorbell=db, db_first=first,
                       timeout_ms=20_000, status=status, stream=ring_s)
        end.record(ring_s)
        time.sleep(0.05)
        assert not end.query(), "the ring launch finished before any batch was published"
        t = threading.Thread(target=producer)
        t.start()
        t.join()
    finally:
        db.ring(first + k)
    ring_s.synchronize()
    assert int(status.item()) == 0
    for a, o in zip(src, outs):
        assert o.cpu().numpy().tobytes() == _want(a, Chain.GenericUlp, 64, n).tobytes()
    db.close()


def test_ring_doorbell_timeout_ends_the_launch(torch):
    """Two batches published, the third never: the waves that reach it give
    up after timeout_ms, set the status bit, and leave its records as they
    were; the published batches are parsed."""
    ctx = ingot_amd.Context(0)
    n = 100_000
    arenas = _batches(torch, GenProfile.V4UDP64, n, 64, 3, seed=11)
    outs = [torch.full((n, 16), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(3)]
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    db = ingot_amd.Doorbell(ctx)
    db.ring(2)  # batches 0 and 1 (db_first 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.parse_ring(arenas, 64, n, Chain.UdpParser, outs, doorbell=db, db_first=1,
                   timeout_ms=200, status=status)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    assert 0.15 < el < 10.0, el
    assert int(status.item()) == 1
    for b in (0, 1):
        assert outs[b].cpu().numpy().tobytes() == _want(arenas[b], Chain.UdpParser, 64, n).tobytes()
    assert bool((outs[2] == 0xAB).all())
    db.close()


def test_ring_doorbell_argument_checks(torch):
    """db_first + nbatches must fit the kernel's 32-bit comparison (ERANGE);
    nothing is launched."""
    ctx = ingot_amd.Context(0)
    n = 4096
    arenas = _batches(torch, GenProfile.V4UDP64, n, 64, 2, seed=5)
    outs = [torch.full((n, 16), 0xAB, dtype=torch.uint8, device="cuda") for _ in range(2)]
    db = ingot_amd.Doorbell(ctx)
    with pytest.raises(RuntimeError, match=r"\(-?\d+\)"):
        ctx.parse_ring(arenas, 64, n, Chain.UdpParser, outs, doorbell=db,
                       db_first=0xFFFFFFFF, timeout_ms=100)
    torch.cuda.synchronize()
    assert all(bool((o == 0xAB).all()) for o in outs)
    # the exact boundary: the last batch's value db_first + 1 == 0x1_0000_0000
    # wraps (ERANGE); db_first + 1 == 0xFFFFFFFF does not
    with pytest.raises(RuntimeError, match=r"\(-?\d+\)"):
        ctx.parse_ring(arenas, 64, n, Chain.UdpParser, outs, doorbell=db,
                       db_first=0xFFFFFFFF, timeout_ms=100)
    db.ring(0xFFFFFFFF)  # publishes both batches from db_first 0xFFFFFFFE
    torch.cuda.synchronize()
    ctx.parse_ring(arenas, 64, n, Chain.UdpParser, outs, doorbell=db, db_first=0xFFFFFFFE,
                   timeout_ms=2000)
    torch.cuda.synchronize()
    for a, o in zip(arenas, outs):
        assert o.cpu().numpy().tobytes() == _want(a, Chain.UdpParser, 64, n).tobytes()
    db.close()


def test_ring_doorbell_other_device_is_einval(torch):
    """A doorbell of another device's context is EINVAL (needs two GPUs)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: the cross-device EINVAL path needs a second context device")
    ctx0, ctx1 = ingot_amd.Context(0), ingot_amd.Context(1)
    n = 4096
    arenas = _batches(torch, GenProfile.V4UDP64, n, 64, 1, seed=6)
    outs = [torch.zeros((n, 16), dtype=torch.uint8, device="cuda")]
    db = ingot_amd.Doorbell(ctx1)
    with pytest.raises(RuntimeError, match="EINVAL|invalid"):
        ctx0.parse_ring(arenas, 64, n, Chain.UdpParser, outs, doorbell=db, timeout_ms=100)
    db.close()
