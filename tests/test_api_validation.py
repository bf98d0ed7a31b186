"""The Python mirror validates every buffer before its raw pointer crosses the
C ABI (ingot_amd.Context._arg / _frames): a wrong dtype (element size), a
strided view, a short output or too many slots for the arena would be an
out-of-bounds access on the device, so each is a ValueError raised on the
host, before any launch.  Runs on CPU: the checks precede the device check
and the library call."""
import pytest
import torch

import ingot_amd
from ingot_amd import Chain, EditOp, Field


@pytest.fixture()
def ctx():
    c = object.__new__(ingot_amd.Context)  # no device needed: nothing is launched
    c._lib, c._h, c.device = None, None, 0
    return c


def _bufs(n=8):
    arena = torch.zeros(4096, dtype=torch.uint8)
    off = torch.arange(n, dtype=torch.int64) * 64
    lens = torch.full((n,), 60, dtype=torch.int32).to(torch.uint16)
    return arena, off, lens


def test_offsets_must_be_64_bit(ctx):
    arena, off, lens = _bufs()
    with pytest.raises(ValueError, match="off must be int64"):
        ctx.parse(arena, off.to(torch.int32), lens, Chain.UdpParser)


def test_lengths_must_be_16_bit(ctx):
    arena, off, lens = _bufs()
    with pytest.raises(ValueError, match="lens must be uint16"):
        ctx.parse(arena, off, lens.to(torch.int64), Chain.UdpParser)


def test_arena_must_be_bytes(ctx):
    arena, off, lens = _bufs()
    with pytest.raises(ValueError, match="arena must be uint8"):
        ctx.parse(arena.view(torch.int32), off, lens, Chain.UdpParser)


def test_strided_views_are_rejected(ctx):
    arena, off, lens = _bufs(16)
    with pytest.raises(ValueError, match="off must be contiguous"):
        ctx.parse(arena, off[::2], lens[::2], Chain.UdpParser)


def test_output_too_small(ctx):
    arena, off, lens = _bufs()
    out = torch.empty((7, 16), dtype=torch.uint8)
    with pytest.raises(ValueError, match="out holds 112 elements, needs at least 128"):
        ctx.parse(arena, off, lens, Chain.UdpParser, out=out)
    with pytest.raises(ValueError, match="out holds"):
        ctx.fields(arena, off, lens, Chain.UdpParser, out=torch.empty((8, 16), dtype=torch.uint8))


def test_slots_must_fit_the_arena(ctx):
    arena = torch.zeros(64 * 10, dtype=torch.uint8)
    out = torch.empty((11, 16), dtype=torch.uint8)
    with pytest.raises(ValueError, match="11 slots of 64 B exceed the 640-B arena"):
        ctx.parse_strided(arena, 64, 11, Chain.UdpParser, out=out)
    with pytest.raises(ValueError, match="multiple of 16"):
        ctx.parse_strided(arena, 40, 4, Chain.UdpParser, out=out)
    with pytest.raises(ValueError, match="exceed"):
        ctx.parse_modify(arena, None, None, Chain.UdpParser,
                         [(2, Field.UDP_DESTINATION, EditOp.SUB, 1)], stride=64, n=11)


def test_parse_read_tables(ctx):
    arena = torch.zeros(1024, dtype=torch.uint8)
    seg_off = torch.zeros(4, dtype=torch.int64)
    seg_len = torch.zeros(4, dtype=torch.int16)
    pkt_seg = torch.tensor([0, 2, 4], dtype=torch.int32)
    with pytest.raises(ValueError, match="pkt_seg must be int32 or uint32"):
        ctx.parse_read(arena, seg_off, seg_len, pkt_seg.to(torch.int64), Chain.GenericUlp)
    with pytest.raises(ValueError, match="seg_len holds 3 elements"):
        ctx.parse_read(arena, seg_off, seg_len[:3], pkt_seg, Chain.GenericUlp)


def test_flow_buffers(ctx):
    arena, off, lens = _bufs()
    with pytest.raises(ValueError, match="flow holds 4 elements"):
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, flow=torch.empty(4, dtype=torch.int32))
    with pytest.raises(ValueError, match="hist holds 16 elements, needs at least 65536"):
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=torch.zeros(16, dtype=torch.int32),
                      bins=65536, flow=torch.empty(8, dtype=torch.int32))
    with pytest.raises(ValueError, match="40 bytes"):
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, key=b"short",
                      flow=torch.empty(8, dtype=torch.int32))


def test_host_tensors_are_rejected_after_shape_checks(ctx):
    """Well-formed CPU tensors reach the device check (the context's device)."""
    arena, off, lens = _bufs()
    with pytest.raises(ValueError, match="must live on cuda:0"):
        ctx.parse(arena, off, lens, Chain.UdpParser, out=torch.empty((8, 16), dtype=torch.uint8))


def test_check_descriptors_catches_out_of_arena_values():
    """Descriptor values are the caller's contract; check_descriptors tests
    them on demand (CPU tensors here)."""
    import torch

    import ingot_amd

    arena = torch.zeros(1000, dtype=torch.uint8)
    off = torch.tensor([0, 100, 900], dtype=torch.int64)
    lens = torch.tensor([60, 64, 100], dtype=torch.int32).to(torch.uint16)
    ingot_amd.check_descriptors(arena, off=off, lens=lens)
    with pytest.raises(ValueError):
        ingot_amd.check_descriptors(arena, off=off, lens=torch.tensor([60, 64, 101]).to(
            torch.uint16))
    seg_off = torch.tensor([0, 14, 34], dtype=torch.int64)
    seg_len = torch.tensor([14, 20, 30], dtype=torch.int32).to(torch.uint16)
    ps = torch.tensor([0, 2, 3], dtype=torch.int32)
    ingot_amd.check_descriptors(arena, seg_off=seg_off, seg_len=seg_len, pkt_seg=ps)
    with pytest.raises(ValueError):
        ingot_amd.check_descriptors(arena, seg_off=seg_off, seg_len=seg_len,
                                    pkt_seg=torch.tensor([0, 2, 4], dtype=torch.int32))
    with pytest.raises(ValueError):
        ingot_amd.check_descriptors(arena, seg_off=seg_off, seg_len=seg_len,
                                    pkt_seg=torch.tensor([0, 2, 1], dtype=torch.int32))
    dense = (seg_off << 16) | seg_len.to(torch.int64)
    ingot_amd.check_descriptors(arena, seg=dense, pkt_seg=ps)
    with pytest.raises(ValueError):
        ingot_amd.check_descriptors(arena, seg=dense + (1000 << 16), pkt_seg=ps)
