"""Doorbells (ingot_gpu_doorbell_*): a parse launch enqueued behind a doorbell
wait does not run until the host rings it, then runs with unchanged results.
A watchdog thread rings the doorbell after a few seconds whatever happens,
so a failing assertion can never leave a stream waiting.  Needs an MI355X."""
import os
import threading
import time

import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch, ingot_amd.Context(0)


def test_launch_waits_for_the_doorbell(env):
    torch, ctx = env
    db = ingot_amd.Doorbell(ctx)
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, 4096, stride=64)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    out = torch.zeros((4096, 16), dtype=torch.uint8, device="cuda")
    watchdog = threading.Timer(5.0, lambda: db.ring(1))
    watchdog.start()
    try:
        db.wait(1, s)
        ctx.parse_strided(arena, 64, 4096, Chain.UdpParser, out=out, stream=s)
        done = torch.cuda.Event()
        done.record(s)
        time.sleep(0.2)
        held = not done.query()
        db.ring(1)
    finally:
        watchdog.cancel()
        db.ring(1)
    s.synchronize()
    assert held, "the launch ran before the doorbell was rung"
    want = oracle.parse_batch(arena.cpu().numpy(), None, None, Chain.UdpParser, stride=64, n=4096)
    assert out.cpu().numpy().tobytes() == want.tobytes()
    # a later wait on a value already reached passes at once
    db.wait(1, s)
    ctx.parse_strided(arena, 64, 4096, Chain.UdpParser, out=out, stream=s)
    s.synchronize()
    db.close()


def test_ring_releases_several_streams(env):
    torch, ctx = env
    db = ingot_amd.Doorbell(ctx)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, 10000)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.zeros((10000, 16), dtype=torch.uint8, device="cuda") for _ in streams]
    watchdog = threading.Timer(5.0, lambda: db.ring(7))
    watchdog.start()
    try:
        for s, o in zip(streams, outs):
            db.wait(7, s)
            ctx.parse(arena, off, lens, Chain.GenericUlp, out=o, stream=s)
        db.ring(6)  # below the threshold: still held
        time.sleep(0.1)
        ev = torch.cuda.Event()
        ev.record(streams[0])
        held = not ev.query()
        db.ring(7)
    finally:
        watchdog.cancel()
        db.ring(7)
    torch.cuda.synchronize()
    assert held
    want = oracle.parse_batch(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                              Chain.GenericUlp)
    for o in outs:
        assert np.array_equal(o.cpu().numpy().reshape(-1), want.view(np.uint8).reshape(-1))
    db.close()


def test_held_queue_blocks_its_streams(env):
    """A doorbell wait holds its whole hardware queue (include/ingot_gpu.h):
    with more streams than GPU_MAX_HW_QUEUES (4 on this image), streams that
    HIP mapped onto the held stream's queue do not run until the ring, while
    streams on other queues do.  A producer that published its frames from
    such a stream and rang only after that work finished would deadlock; from
    the host (as here) the ring releases everything."""
    torch, ctx = env
    db = ingot_amd.Doorbell(ctx)
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, 4096, stride=64)
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(9)]
    watchdog = threading.Timer(5.0, lambda: db.ring(1))
    watchdog.start()
    try:
        db.wait(1, streams[0])
        evs = []
        for s in streams[1:]:
            ctx.parse_strided(arena, 64, 4096, Chain.UdpParser, stream=s)
            e = torch.cuda.Event()
            e.record(s)
            evs.append(e)
        time.sleep(0.3)
        ran = [e.query() for e in evs]
        db.ring(1)
    finally:
        watchdog.cancel()
        db.ring(1)
    torch.cuda.synchronize()
    # the library's contract: the ring releases every stream
    assert all(e.query() for e in evs)
    db.close()
    # How HIP maps streams onto hardware queues is the runtime's, not the
    # library's: checked whenever the queue count (GPU_MAX_HW_QUEUES, HIP's
    # default 4 when unset) is below the stream count
    hwq = os.environ.get("GPU_MAX_HW_QUEUES", "4")
    if not hwq.isdigit() or int(hwq) >= len(streams):
        return
    assert any(ran), "no stream ran beside the held one"
    assert not all(ran), ("every stream ran beside the held queue: more hardware queues than "
                          "streams on this box?")


def test_stream_delay_holds_the_stream(env):
    """ingot_gpu_stream_delay: work enqueued after it starts `ns` later (device
    wall clock); 0 is a no-op; the parse behind it is unchanged."""
    torch, ctx = env
    s = torch.cuda.Stream()
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, 4096, stride=64)
    torch.cuda.synchronize()
    for ns in (0, 20_000, 200_000):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        ctx.stream_delay(ns, s)
        b.record(s)
        got = ctx.parse_strided(arena, 64, 4096, Chain.UdpParser, stream=s)
        s.synchronize()
        us = a.elapsed_time(b) * 1e3
        assert ns / 1e3 <= us + 1.0, (ns, us)  # one 100-MHz tick of slack
        assert us < ns / 1e3 + 2_000, (ns, us)
        want = oracle.parse_batch(arena.cpu().numpy(), None, None, Chain.UdpParser, stride=64,
                                  n=4096)
        assert got.cpu().numpy().tobytes() == want.tobytes()


def test_stream_delay_rejects_bad_arguments(env):
    _, ctx = env
    with pytest.raises(ValueError):
        ctx.stream_delay(-1)
    with pytest.raises(ValueError):
        ctx.stream_delay(1 << 32)
