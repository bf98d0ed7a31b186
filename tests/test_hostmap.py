"""Zero-copy host rings (ingot_gpu_host_map): the kernels read frames straight
from pinned host memory across PCIe and may write records into host memory.
Results must be bit-identical to the device-resident path (which
test_gpu_parity.py pins to the oracle) and to the oracle itself.  Needs an
MI355X: `pytest -m gpu`.

These cases run in the main GPU-suite process.  Round 5 ran them in a child
process after two suite runs saw a late hipErrorIllegalAddress at a pageable
D2H copy; the mapping API has since been made to unregister only what it
registered itself, counted per mapping, and
test_mapping_lifecycle_then_pageable_copies exercises exactly that state
before the rest of the suite's pageable copies."""
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
    for h in [h_arena, h_out] + ([h_lens] if stride and h_lens is not None else []) + \
            ([] if stride else [h_off, h_lens]):
        ctx.host_unmap(h)
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
    mapped = [h_arena]
    if stride:
        h_lens = _pinned(torch, lens) if lens is not None else None
        d_lens = ctx.host_map(h_lens) if h_lens is not None else None
        mapped += [h_lens] if h_lens is not None else []
        rc = lib.ingot_gpu_parse_modify(ctx._h, d_arena, None, d_lens, stride, n,
                                        int(Chain.UdpParser), e.ctypes.data, len(e), None, None)
        l_np = None if lens is None else lens.cpu().numpy()
        oracle.parse_modify_batch(want, None, l_np, Chain.UdpParser, edits, stride=stride, n=n)
    else:
        h_off, h_lens = _pinned(torch, off), _pinned(torch, lens)
        mapped += [h_off, h_lens]
        rc = lib.ingot_gpu_parse_modify(ctx._h, d_arena, ctx.host_map(h_off),
                                        ctx.host_map(h_lens), 0, n, int(Chain.UdpParser),
                                        e.ctypes.data, len(e), None, None)
        oracle.parse_modify_batch(want, off.cpu().numpy(), lens.cpu().numpy(), Chain.UdpParser,
                                  edits)
    assert rc == 0
    torch.cuda.synchronize()
    for h in mapped:
        ctx.host_unmap(h)
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
    for h in (h_arena, h_lens, h_out, h_off):
        ctx.host_unmap(h)
    assert h_out.numpy().tobytes() == want.cpu().numpy().tobytes()
    assert (h_off.numpy() == off.cpu().numpy()).all()


def _hip():
    """The HIP runtime torch loaded (same soname as the library's)."""
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipPointerGetAttributes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipGetLastError.restype = ctypes.c_int
    return hip


class _PtrAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def _registered(hip, ptr) -> bool:
    a = _PtrAttr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(ptr))
    hip.hipGetLastError()
    return rc == 0 and a.type == 1  # hipMemoryTypeHost


def test_mapping_lifecycle_then_pageable_copies(torch, ctx):
    """The mapping API's counting, then the pageable D2H copies that faulted
    in round 5 (a 1.6 MB record buffer, a 40 k-frame arena), in this process:
    - a pageable buffer mapped twice is still registered after one unmap and
      parses identically; the second unmap unregisters it; a third is refused;
    - a sub-range of a mapped buffer shares its registration; a range partly
      overlapping it is refused;
    - two byte-disjoint buffers sharing a page are mapped at once (frames in
      one, records written into the other);
    - hipHostMalloc memory (a pinned torch tensor) is never unregistered:
      after map + unmap it still serves a mapped parse and a non_blocking copy;
    - destroying a context releases the registrations of its open mappings."""
    lib = _lib.load()
    hip = _hip()
    n = 20_000
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=5)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp).cpu().numpy()
    a_np, off_d, lens_d = arena.cpu().numpy(), off, lens
    nbytes = a_np.nbytes

    def parse_into(d_arena, d_out):
        assert lib.ingot_gpu_parse(ctx._h, d_arena, off_d.data_ptr(), lens_d.data_ptr(), n,
                                   int(Chain.GenericUlp), d_out, None) == 0
        torch.cuda.synchronize()

    # one pageable buffer: frames, then the records 16 B after their end, in
    # the page where the frames end (the two registrations share that page)
    raw = np.zeros(nbytes + n * 16 + 4 * 4096, np.uint8)
    base = (-raw.ctypes.data) % 4096
    shift = (2048 - nbytes % 4096) % 4096 // 16 * 16
    frames = raw[base + shift:base + shift + nbytes]
    frames[:] = a_np
    r0 = base + shift + (nbytes + 15) // 16 * 16 + 16
    recs = raw[r0:r0 + n * 16]
    assert (frames.ctypes.data + nbytes - 1) // 4096 == recs.ctypes.data // 4096
    dev_out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")

    d1 = ctx.host_map(frames)
    d2 = ctx.host_map(frames)  # a second mapping of the same bytes
    assert d1 == d2 and _registered(hip, frames.ctypes.data)
    ctx.host_unmap(frames)  # one mapping left: still registered and usable
    assert _registered(hip, frames.ctypes.data)
    parse_into(d1, dev_out.data_ptr())
    assert dev_out.cpu().numpy().tobytes() == want.tobytes()
    # a sub-range shares the registration; a straddling range is refused
    sub = frames[4096:8192]
    assert ctx.host_map(sub) == d1 + 4096
    ctx.host_unmap(sub)
    d = ctypes.c_void_p()
    assert lib.ingot_gpu_host_map(ctx._h, frames.ctypes.data + nbytes - 8, 64,
                                  ctypes.byref(d)) == -1
    # records into the neighbour that shares the frames' last page
    d_recs = ctx.host_map(recs)
    recs[:] = 0xEE
    parse_into(d1, d_recs)
    assert recs.tobytes() == want.tobytes()
    ctx.host_unmap(frames)  # frames unregistered, records still mapped
    assert not _registered(hip, frames.ctypes.data)
    assert _registered(hip, recs.ctypes.data)
    assert lib.ingot_gpu_host_unmap(ctx._h, frames.ctypes.data) == -1  # nothing left to unmap
    recs[:] = 0
    parse_into(arena.data_ptr(), d_recs)
    assert recs.tobytes() == want.tobytes()
    ctx.host_unmap(recs)
    assert not _registered(hip, recs.ctypes.data)

    # hipHostMalloc memory: map + unmap never unregisters it
    h_arena = _pinned(torch, arena)
    assert _registered(hip, h_arena.data_ptr())
    d_h = ctx.host_map(h_arena)
    ctx.host_unmap(h_arena)
    assert _registered(hip, h_arena.data_ptr())
    d_h = ctx.host_map(h_arena)
    parse_into(d_h, dev_out.data_ptr())
    assert dev_out.cpu().numpy().tobytes() == want.tobytes()
    ctx.host_unmap(h_arena)
    back = torch.empty_like(arena)
    back.copy_(h_arena, non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(back, arena)

    # a destroyed context releases the registrations it still holds
    other = ingot_amd.Context(0)
    other.host_map(frames)
    assert _registered(hip, frames.ctypes.data)
    other.close()
    assert not _registered(hip, frames.ctypes.data)
    del raw, frames, recs

    # the pageable D2H copies that faulted in round 5, with allocation churn
    big, boff, blens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, 40_000, seed=52)
    rec_dev = torch.empty((100_000, 16), dtype=torch.uint8, device="cuda")
    rec_dev.copy_(torch.arange(100_000 * 16, device="cuda").to(torch.uint8).view(100_000, 16))
    first_big, first_rec = big.cpu().numpy(), rec_dev.cpu().numpy()
    for _ in range(8):
        assert np.array_equal(big.cpu().numpy(), first_big)
        assert np.array_equal(rec_dev.cpu().numpy(), first_rec)
        assert np.array_equal(boff.cpu().numpy()[-5:], boff[-5:].cpu().numpy())
    torch.cuda.synchronize()


def test_registration_shared_across_contexts(torch, ctx):
    """Registrations are per process: a pageable buffer mapped by two
    contexts is registered once, stays registered while either mapping
    lives, and each context unmaps only its own mapping."""
    lib = _lib.load()
    hip = _hip()
    n = 5000
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=9)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp).cpu().numpy()
    raw = np.zeros(arena.numel() + 8192, np.uint8)
    a = raw[(-raw.ctypes.data) % 4096:][:arena.numel()]
    a[:] = arena.cpu().numpy()
    other = ingot_amd.Context(0)
    da, db = ctx.host_map(a), other.host_map(a)
    assert da == db and _registered(hip, a.ctypes.data)
    assert lib.ingot_gpu_host_unmap(other._h, a.ctypes.data + 64) == -1  # not a mapping start
    ctx.host_unmap(a)
    assert _registered(hip, a.ctypes.data)  # the other context's mapping keeps it
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    assert lib.ingot_gpu_parse(other._h, db, off.data_ptr(), lens.data_ptr(), n,
                               int(Chain.GenericUlp), out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == want.tobytes()
    assert lib.ingot_gpu_host_unmap(ctx._h, a.ctypes.data) == -1  # ctx holds no mapping now
    other.host_unmap(a)
    assert not _registered(hip, a.ctypes.data)
    other.close()


def test_mappings_from_many_threads(torch, ctx):
    """The process-wide registration table under contention: 8 threads over
    two contexts, 100 rounds each, map one shared buffer (one registration,
    counted across threads) and their own byte-disjoint 2-KiB slices, two per
    page, then unmap them all.  No call fails, every slice is registered while
    mapped, nothing is left registered afterwards, and a buffer mapped after
    the storm parses bit-exact."""
    import threading

    hip = _hip()
    lib = _lib.load()
    other = ingot_amd.Context(0)
    raw = np.zeros(48 * 4096 + 4096, np.uint8)
    base = raw[(-raw.ctypes.data) % 4096:][:48 * 4096]
    shared = base[:8 * 4096]
    slices = [base[8 * 4096 + i * 2048:8 * 4096 + (i + 1) * 2048] for i in range(64)]
    errors = []

    def worker(t):
        try:
            mine = slices[t::8]  # each page's two slices belong to two threads
            for k in range(100):
                c = (ctx, other)[(t + k) % 2]
                assert c.host_map(shared) != 0
                for s in mine:
                    c.host_map(s)
                    assert _registered(hip, s.ctypes.data)
                for s in mine:
                    c.host_unmap(s)
                c.host_unmap(shared)
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append(f"thread {t}: {e!r}")

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors
    assert not _registered(hip, shared.ctypes.data)
    assert not any(_registered(hip, s.ctypes.data) for s in slices)

    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, 24, seed=12)
    assert arena.numel() <= shared.nbytes
    want = ctx.parse(arena, off, lens, Chain.GenericUlp).cpu().numpy()
    shared[:arena.numel()] = arena.cpu().numpy()
    d = other.host_map(shared)
    out = torch.empty((24, 16), dtype=torch.uint8, device="cuda")
    assert lib.ingot_gpu_parse(other._h, d, off.data_ptr(), lens.data_ptr(), 24,
                               int(Chain.GenericUlp), out.data_ptr(), None) == 0
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == want.tobytes()
    other.host_unmap(shared)
    other.close()
