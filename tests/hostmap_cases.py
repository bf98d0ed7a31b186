"""Zero-copy host rings (ingot_gpu_host_map): the kernels read frames straight
from pinned host memory across PCIe and may write records into host memory.
Results must be bit-identical to the device-resident path (which
test_gpu_parity.py pins to the oracle) and to the oracle itself.  Needs an
MI355X.

Run by tests/test_hostmap.py in a child process of its own: these cases
page-lock, map and release host memory (hipHostRegister / hipHostUnregister
on pageable numpy buffers, mapped pinned tensors), and that host-side
mapping state stays out of the process that runs the rest of the GPU suite.
Directly: `pytest tests/hostmap_cases.py`."""
import ctypes

import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


def _page_aligned(a):
    """A copy of numpy array `a` in its own page-aligned, page-padded buffer
    (pageable memory; no two arrays share a page when registered)."""
    raw = np.zeros(a.nbytes + 2 * 4096, np.uint8)
    start = (-raw.ctypes.data) % 4096
    out = raw[start:start + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def _pinned(torch, t):
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h


@pytest.mark.parametrize("profile,chain,stride", [
    ("MIXED", Chain.GenericUlp, None), ("ADVERSARIAL", Chain.VlanUlp, None),
    ("GENEVE_ADVERSARIAL", Chain.GeneveOverV6Tunnel, None),
    ("V4UDP64", Chain.UdpParser, 64), ("VLAN_V6EH", Chain.VlanUlp, 256),
])
def test_parse_from_pinned_host_ring(torch, ctx, profile, chain, stride):
    """Arena (and descriptors) in hipHostMalloc memory, records written into
    pinned host memory: equal to the device-resident records and the oracle."""
    n = 50_001
    lib = _lib.load()
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=21, stride=stride)
    want = (ctx.parse_strided(arena, stride, n, chain, lens=lens) if stride
            else ctx.parse(arena, off, lens, chain))
    torch.cuda.synchronize()
    h_arena = _pinned(torch, arena)
    h_out = torch.zeros((n, 16), dtype=torch.uint8, pin_memory=True)
    d_arena, d_out = ctx.host_map(h_arena), ctx.host_map(h_out)
    if stride:
        h_lens = _pinned(torch, lens) if lens is not None else None
        d_lens = ctx.host_map(h_lens) if h_lens is not None else None
        rc = lib.ingot_gpu_parse_strided(ctx._h, d_arena, stride, d_lens, n, int(chain), d_out,
                                         None)
    else:
        h_off, h_lens = _pinned(torch, off), _pinned(torch, lens)
        rc = lib.ingot_gpu_parse(ctx._h, d_arena, ctx.host_map(h_off), ctx.host_map(h_lens), n,
                                 int(chain), d_out, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert h_out.numpy().tobytes() == want.cpu().numpy().tobytes()
    w = oracle.parse_batch(h_arena.numpy(), None if stride else off.cpu().numpy(),
                           None if lens is None else lens.cpu().numpy(), chain,
                           stride=stride or 0, n=n, nthreads=8)
    assert h_out.numpy().tobytes() == w.tobytes()


def test_parse_from_registered_pageable_memory(torch, ctx):
    """Pageable numpy memory is page-locked and mapped by ingot_gpu_host_map
    (hipHostRegister) and released by ingot_gpu_host_unmap."""
    n = 20_000
    lib = _lib.load()
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=5)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp)
    torch.cuda.synchronize()
    raw = np.zeros(arena.numel() + 8192, dtype=np.uint8)
    a = raw[(-raw.ctypes.data) % 4096:][:arena.numel()]  # page-aligned view
    a[:] = arena.cpu().numpy()
    d_arena = ctx.host_map(a)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    assert lib.ingot_gpu_parse(ctx._h, d_arena, off.data_ptr(), lens.data_ptr(), n,
                               int(Chain.GenericUlp), out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    ctx.host_unmap(a)
    assert out.cpu().numpy().tobytes() == want.cpu().numpy().tobytes()


def test_host_map_rejects_bad_arguments(ctx):
    lib = _lib.load()
    d = ctypes.c_void_p()
    assert lib.ingot_gpu_host_map(ctx._h, None, 64, ctypes.byref(d)) == -1
    buf = np.zeros(64, np.uint8)
    assert lib.ingot_gpu_host_map(ctx._h, buf.ctypes.data, 0, ctypes.byref(d)) == -1
    assert lib.ingot_gpu_host_map(None, buf.ctypes.data, 64, ctypes.byref(d)) == -1
    assert lib.ingot_gpu_host_unmap(ctx._h, None) == -1


def test_parse_read_over_mblk_chains_in_host_memory(torch, ctx):
    """OPTE's real input: packets as chains of chunks (mblk_t) in host
    memory.  The chunk pool and its tables stay in pageable host memory
    (page-locked and mapped by ingot_gpu_host_map), parse_read runs over PCIe,
    records and remainder-chunk indices land in mapped host memory; equal to
    the oracle's parse_read."""
    lib = _lib.load()
    from tests.frames import build_frames

    frames = build_frames(3000, seed=17, vlan=False)
    rng = np.random.default_rng(3)
    packets = []
    for f in frames:  # 1-3 chunks, cut at random points (headers may straddle)
        cuts = sorted(rng.integers(1, max(2, len(f)), rng.integers(0, 3)))
        parts, prev = [], 0
        for c in cuts:
            if c > prev:
                parts.append(f[prev:c])
                prev = c
        parts.append(f[prev:])
        packets.append(parts)
    arena, so, sl, ps = (_page_aligned(x) for x in ingot_amd.chunk_tables(packets))
    n = len(packets)
    recs = _page_aligned(np.zeros((n, 16), np.uint8))
    chunk = _page_aligned(np.zeros(n, np.uint16))
    d = [ctx.host_map(x) for x in (arena, so, sl, ps, recs, chunk)]
    for chain in (Chain.GenericUlp, Chain.UdpParser):
        recs[:] = 0xEE
        assert lib.ingot_gpu_parse_read(ctx._h, d[0], d[1], d[2], d[3], n, int(chain), d[4],
                                        d[5], None) == 0
        torch.cuda.synchronize()
        w_rec, _, w_chunk = oracle.parse_read_batch(arena, so, sl, ps, chain)
        assert recs.tobytes() == np.asarray(w_rec).tobytes(), chain
        assert (chunk == np.asarray(w_chunk).astype(np.uint16)).all(), chain
    for x in (arena, so, sl, ps, recs, chunk):
        ctx.host_unmap(x)


@pytest.mark.parametrize("stride", [None, 64, 128])
def test_parse_modify_in_host_memory(torch, ctx, stride):
    """ingot's setters applied in place to frames that stay in mapped host
    memory (the reference's parse-and-decr-v4 and a multi-field edit list):
    the host bytes afterwards equal the oracle's rewrite."""
    from ingot_amd import EditOp, Field, edits_array

    lib = _lib.load()
    n = 20_003
    prof = GenProfile.V4UDP64 if stride == 64 else GenProfile.MIXED
    arena, off, lens = ingot_amd.gen_frames(prof, n, seed=8, stride=stride)
    edits = [(2, Field.UDP_DESTINATION, EditOp.SUB, 1), (1, Field.V4_HOP_LIMIT, EditOp.SUB, 1),
             (1, Field.V6_HOP_LIMIT, EditOp.SUB, 1)]
    h_arena = _pinned(torch, arena)
    want = h_arena.numpy().copy()
    e = edits_array(edits)
    d_arena = ctx.host_map(h_arena)
    if stride:
        h_lens = _pinned(torch, lens) if lens is not None else None
        d_lens = ctx.host_map(h_lens) if h_lens is not None else None
        rc = lib.ingot_gpu_parse_modify(ctx._h, d_arena, None, d_lens, stride, n,
                                        int(Chain.UdpParser), e.ctypes.data, len(e), None, None)
        l_np = None if lens is None else lens.cpu().numpy()
        oracle.parse_modify_batch(want, None, l_np, Chain.UdpParser, edits, stride=stride, n=n)
    else:
        h_off, h_lens = _pinned(torch, off), _pinned(torch, lens)
        rc = lib.ingot_gpu_parse_modify(ctx._h, d_arena, ctx.host_map(h_off),
                                        ctx.host_map(h_lens), 0, n, int(Chain.UdpParser),
                                        e.ctypes.data, len(e), None, None)
        oracle.parse_modify_batch(want, off.cpu().numpy(), lens.cpu().numpy(), Chain.UdpParser,
                                  edits)
    assert rc == 0
    torch.cuda.synchronize()
    got = h_arena.numpy()
    diff = np.nonzero(got != want)[0]
    assert diff.size == 0, (diff[:10], got[diff[:10]], want[diff[:10]])
    assert (got != arena.cpu().numpy()).any()  # something was rewritten


def test_parse_packed_from_host_capture_buffer(torch, ctx):
    """A capture buffer in host memory (frames back to back, lengths only):
    ingot_gpu_parse_packed scans the lengths and parses across PCIe; records
    and derived offsets equal the device-resident parse with offsets."""
    lib = _lib.load()
    n = 30_011
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=19)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp)
    torch.cuda.synchronize()
    h_arena, h_lens = _pinned(torch, arena), _pinned(torch, lens)
    h_out = torch.zeros((n, 16), dtype=torch.uint8, pin_memory=True)
    h_off = torch.zeros(n, dtype=torch.int64, pin_memory=True)
    wb = lib.ingot_gpu_packed_workspace_size(n)
    work = torch.empty(wb, dtype=torch.uint8, device="cuda")
    rc = lib.ingot_gpu_parse_packed(ctx._h, ctx.host_map(h_arena), ctx.host_map(h_lens), n,
                                    int(Chain.GenericUlp), ctx.host_map(h_out),
                                    ctx.host_map(h_off), work.data_ptr(), wb, None)
    assert rc == 0
    torch.cuda.synchronize()
    assert h_out.numpy().tobytes() == want.cpu().numpy().tobytes()
    assert (h_off.numpy() == off.cpu().numpy()).all()
