"""Whole-batch parity at the benchmark sizes: every record (and every flow id
and hash) of a full BASELINE config batch against the oracle over the exact
device bytes — not a sample.  C3: 16,777,216 mixed frames (~13 GB); C4 and
C5: one 8,388,608-frame shard of the 64 M-frame 8-GPU job; C6: 8,388,608
Geneve-over-IPv6 frames; c3r / c3p: the C3 frames as header + payload
chunks / as lengths only.  Needs an MI355X
(`pytest -m gpu`); the oracle runs multi-threaded on the host copy."""
import os

import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


def _mismatches(got, want):
    g = got.reshape(len(want), -1)
    w = want.view(np.uint8).reshape(len(want), -1)
    return np.nonzero((g != w).any(axis=1))[0]


@pytest.mark.parametrize("profile,chain,n,first", [
    ("MIXED", Chain.GenericUlp, 1 << 24, 0),            # C3, BASELINE configs[2]
    ("VLAN_V6EH", Chain.VlanUlp, 1 << 23, 5 << 23),     # C4 shard of rank 5 of 8
    ("GENEVE", Chain.GeneveOverV6Tunnel, 1 << 23, 0),   # C6, the tunnel chain (§8f-1)
])
def test_whole_batch_records_bit_exact(ctx, torch, profile, chain, n, first):
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, first=first)
    recs = ctx.parse(arena, off, lens, chain)
    torch.cuda.synchronize()
    got = recs.cpu().numpy()
    a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
    del arena, recs
    torch.cuda.empty_cache()
    want = oracle.parse_batch(a, o, ln, chain, nthreads=THREADS)
    bad = _mismatches(got, want)
    assert bad.size == 0, (profile, bad[:5])


def test_c3r_whole_batch_parse_read_first_bit_exact(ctx, torch):
    """c3r (the C3 frames as [header chunk | payload chunk], the header-split
    shape) through the bench line's path — ingot_gpu_parse_read_first with
    chunk bounds on demand (INGOT_TUNE_READ_PLAN 17) — every record and
    remainder chunk of the 16.7 M packets against the oracle's parse_read."""
    import bench
    from ingot_amd import abi

    n = 1 << 24
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    recs0 = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, Chain.GenericUlp))
    seg_off, seg_len, pkt_seg, _ = bench.read_chunks(torch, off, None, lens, recs0, "split2",
                                                     "cuda:0")
    first = ingot_amd.first_chunks(seg_off, seg_len, pkt_seg)
    c = ingot_amd.Context(0)
    c.set_tuning(abi.TUNE_READ_PLAN, 17)
    out, chunk = c.parse_read(arena, seg_off, seg_len, pkt_seg, Chain.GenericUlp, first=first)
    torch.cuda.synchronize()
    got, got_chunk = out.cpu().numpy(), chunk.cpu().numpy().view(np.uint16)
    a = arena.cpu().numpy()
    so, sl, ps = seg_off.cpu().numpy(), seg_len.cpu().numpy(), pkt_seg.cpu().numpy()
    del arena, out, chunk, first, seg_off, seg_len, pkt_seg
    torch.cuda.empty_cache()
    want, _, want_chunk = oracle.parse_read_batch(a, so, sl, ps.view(np.uint32), Chain.GenericUlp,
                                                  nthreads=THREADS)
    bad = _mismatches(got, want)
    assert bad.size == 0, bad[:5]
    assert (got_chunk == want_chunk).all()


def test_c3p_whole_batch_packed_offsets_and_records(ctx, torch):
    """C3p (the C3 frames back to back, lengths only): the offsets the
    wavefront prefix scan derives equal the lengths' exclusive prefix sum and
    every record equals the oracle's, all 16.7 M frames."""
    n = 1 << 24
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    off_out = torch.empty(n, dtype=torch.int64, device="cuda")
    recs = ctx.parse_packed(arena, lens, Chain.GenericUlp, off_out=off_out)
    torch.cuda.synchronize()
    got, got_off = recs.cpu().numpy(), off_out.cpu().numpy()
    a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
    del arena, recs, off_out
    torch.cuda.empty_cache()
    assert (got_off == o).all()
    assert (o[1:] == np.cumsum(ln.astype(np.int64))[:-1]).all() and o[0] == 0
    want = oracle.parse_batch(a, o, ln, Chain.GenericUlp, nthreads=THREADS)
    bad = _mismatches(got, want)
    assert bad.size == 0, bad[:5]


def test_config5_whole_shard_flow_ids_and_hashes(ctx, torch):
    """C5 (BASELINE configs[4]) per-GPU shard: the default flows kernel's
    flow ids (16-bit table) and the full 32-bit hashes of the hash-requesting
    kernel, every packet, against the oracle's RSS Toeplitz over the same
    bytes; the histogram equals the oracle's."""
    n = 1 << 23
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, first=1 << 23)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n,
                         workspace=ctx.flow_hist_workspace(n, 1 << 16))
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow2 = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, n=n, hashes=hashes)
    torch.cuda.synchronize()
    g_flow = flow.cpu().numpy().view(np.uint32)
    g_flow2 = flow2.cpu().numpy().view(np.uint32)
    g_hash = hashes.cpu().numpy().view(np.uint32)
    g_hist = hist.cpu().numpy().view(np.uint32)
    a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
    del arena, flow, flow2, hashes, hist
    torch.cuda.empty_cache()
    w_hist, w_hash = oracle.flow_hist(a, o, ln, Chain.VlanUlp)
    w_flow = oracle.flow_hist.last_flows
    bad = np.nonzero(g_flow != w_flow)[0]
    assert bad.size == 0, bad[:5]
    assert np.array_equal(g_flow2, w_flow)
    bad = np.nonzero(g_hash != w_hash)[0]
    assert bad.size == 0, bad[:5]
    assert np.array_equal(g_hist, w_hist)
