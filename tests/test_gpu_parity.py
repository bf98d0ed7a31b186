"""Parity of the gfx950 path against the CPU oracle (bit-exact records and
field blocks), through the C ABI.  Needs an MI355X: `pytest -m gpu`.

* the reference's golden vectors (tests/golden/kats.json) through the device;
* adversarial fuzz frames (every truncation / ihl / data_offset / EH / unknown
  ethertype path), all three chains, records AND every getter;
* each benchmark profile and layout at sizes the oracle finishes in seconds;
* at full benchmark sizes, size-independent properties plus a sampled oracle
  re-check of frames copied back from the device.
"""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile, ParseError
from tests.kat_check import check

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


def host(t):
    return None if t is None else t.cpu().numpy()


TUN = Chain.GeneveOverV6Tunnel
BASE_CHAINS = [c for c in Chain if c != TUN]


def dev_fields(ctx, arena, off, lens, chain, stride=0, n=None):
    """Device field blocks: ingot_fields, or ingot_geneve_fields for the tunnel."""
    if chain == TUN:
        return ctx.geneve_fields(arena, off, lens, stride=stride, n=n)
    return ctx.fields(arena, off, lens, chain, stride=stride, n=n)


def oracle_all(arena, off, lens, chain, stride=0, n=None, fields=True):
    """Oracle (records, field blocks) as raw bytes-comparable numpy arrays."""
    rec = oracle.parse_batch(host(arena), host(off), host(lens), chain, stride=stride, n=n,
                             nthreads=8)
    if not fields:
        return rec, None
    if chain == TUN:
        fld = oracle.geneve_fields_batch(host(arena), host(off), host(lens), stride=stride, n=n)
    else:
        fld = oracle.parse_batch(host(arena), host(off), host(lens), chain, stride=stride, n=n,
                                 fields=True, nthreads=8)[1]
    return rec, fld


def oracle_check(ctx, torch, arena, off, lens, chain, stride=0, n=None, fields=True):
    """Run device records (+fields) and compare byte-for-byte with the oracle."""
    if off is not None:
        n = off.numel()
        recs = ctx.parse(arena, off, lens, chain)
    else:
        recs = ctx.parse_strided(arena, stride, n, chain, lens=lens)
    flds = dev_fields(ctx, arena, off, lens, chain, stride=stride, n=n) if fields else None
    torch.cuda.synchronize()
    w_rec, w_fld = oracle_all(arena, off, lens, chain, stride=stride, n=n, fields=fields)
    g_rec = ingot_amd.records_to_numpy(recs)
    diff = np.nonzero((g_rec.view(np.uint8).reshape(n, 16) !=
                       w_rec.view(np.uint8).reshape(n, 16)).any(axis=1))[0]
    assert diff.size == 0, (f"{diff.size} record mismatches, first {diff[:5]}: "
                            f"gpu {g_rec[diff[0]]} oracle {w_rec[diff[0]]}")
    if fields:
        g_f = flds.cpu().numpy().reshape(n, -1)
        fd = np.nonzero((g_f != w_fld.view(np.uint8).reshape(n, -1)).any(axis=1))[0]
        assert fd.size == 0, (f"{fd.size} field mismatches, first {fd[:5]}: "
                              f"gpu {g_f[fd[0]].view(w_fld.dtype)} oracle {w_fld[fd[0]]}")
    return g_rec


# ---------------------------------------------------------------------------
# golden vectors
# ---------------------------------------------------------------------------
def test_golden_kats_on_device(ctx, torch, kats):
    for chain in Chain:
        group = [k for k in kats["chain_kats"] if Chain[k["chain"]] == chain]
        if not group:
            continue
        frames = [bytes.fromhex(k["frame"]) for k in group]
        recs, flds = ingot_amd.parse_frames(frames, chain)
        for k, f, r, fl in zip(group, frames, recs, flds):
            bad = check(k, r, fl)
            assert not bad, f"{k['name']} ({k['source']}): {bad}"
            orec, ofld = oracle.parse_one(f, chain)
            if chain == TUN:
                ofld = oracle.parse_geneve(f)
            assert r.tobytes() == orec.tobytes(), k["name"]
            assert fl.tobytes() == ofld.tobytes(), k["name"]


def test_reference_tests_read_alike(torch):
    """ingot-examples/src/tests.rs:56-118 and :307-379, through the device."""
    f = bytearray(54)
    f[0:6] = b"\xff" * 6
    f[6:12] = bytes([0xA, 0xB, 0xC, 0xD, 0xE, 0xF])
    f[12:14] = b"\x08\x00"
    f[14] = 0x08
    f[23] = 17
    f[26:30] = bytes([192, 168, 0, 1])
    f[30:34] = bytes([192, 168, 0, 255])
    f[34:46] = bytes(range(12))
    f[46:54] = bytes([0x17, 0xC2, 0x17, 0xC1, 0, 0, 0xFF, 0xFF])
    stack, hint, rest = ingot_amd.UdpParser.parse(bytes(f))
    assert hint is None and rest == b""
    assert stack.eth.source() == bytes([0xA, 0xB, 0xC, 0xD, 0xE, 0xF])
    assert stack.eth.destination() == b"\xff" * 6
    assert stack.eth.ethertype() == 0x0800
    assert stack.l3.protocol() == 17
    assert stack.l3.source() == bytes([192, 168, 0, 1])
    assert stack.l3.ihl() == 8
    assert stack.l3.options_ref() == bytes(range(12))
    assert (stack.l4.source(), stack.l4.destination()) == (6082, 6081)
    assert (stack.l4.length(), stack.l4.checksum()) == (0, 0xFFFF)

    would_be_valid = bytes.fromhex(
        "aa000400ff10aa000400ff010800" "45000024000000" "00f0110000080808" "08c0a80005"
        "00800035" "00080000")
    for cut, label in ((4, "inner_eth"), (14, "inner_l3"), (len(would_be_valid) - 1,
                                                            "inner_ulp")):
        with pytest.raises(ingot_amd.PacketParseError) as e:
            ingot_amd.GenericUlp.parse_slice(would_be_valid[:cut])
        assert e.value.error() == ParseError.TooSmall
        assert e.value.header() == label


# ---------------------------------------------------------------------------
# fuzz + profiles
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("chain", list(Chain))
def test_adversarial_fuzz_bit_exact(ctx, torch, chain):
    # random frames never form a valid tunnel: the tunnel chain gets tunnel fuzz
    prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
    arena, off, lens = ingot_amd.gen_frames(prof, 300_000, seed=11)
    g = oracle_check(ctx, torch, arena, off, lens, chain)
    st = g["status"]
    # the fuzz set must reach every reachable outcome
    assert (st == 0).any()
    assert (st == ParseError.TooSmall).any() and (st == ParseError.Unwanted).any()
    assert (g["err_layer"][st != 0] == 0).any()


@pytest.mark.parametrize("profile,chain", [
    (GenProfile.MIXED, Chain.GenericUlp),
    (GenProfile.MIXED, Chain.UdpParser),
    (GenProfile.VLAN_V6EH, Chain.VlanUlp),
    (GenProfile.VLAN_V6EH, Chain.GenericUlp),
    (GenProfile.FLOWS, Chain.VlanUlp),
])
def test_profile_indexed_bit_exact(ctx, torch, profile, chain):
    arena, off, lens = ingot_amd.gen_frames(profile, 200_000, seed=3)
    g = oracle_check(ctx, torch, arena, off, lens, chain)
    if chain != Chain.UdpParser and not (profile != GenProfile.MIXED and
                                         chain == Chain.GenericUlp):
        assert (g["status"] == 0).all()


@pytest.mark.parametrize("stride,profile", [(64, GenProfile.V4UDP64), (64, GenProfile.ADVERSARIAL),
                                            (128, GenProfile.MIXED), (2048, GenProfile.MIXED),
                                            (48, GenProfile.ADVERSARIAL)])
def test_strided_bit_exact(ctx, torch, stride, profile):
    n = 100_003  # not a multiple of 64
    arena, _, lens = ingot_amd.gen_frames(profile, n, seed=5, stride=stride)
    for chain in Chain:
        oracle_check(ctx, torch, arena, None, lens, chain, stride=stride, n=n,
                     fields=chain == Chain.GenericUlp)


def test_v4udp64_full_batch_exact(ctx, torch):
    """Config 2 exactly: 1,048,576 x 64 B under UdpParser, every record checked."""
    n = 1 << 20
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    g = oracle_check(ctx, torch, arena, None, None, Chain.UdpParser, stride=64, n=n,
                     fields=False)
    assert (g["status"] == 0).all()
    assert (g["payload_off"] == 42).all() and (g["l4_kind"] == 2).all()


@pytest.mark.parametrize("layout", ["indexed", "strided"])
def test_compact_records_bit_exact(ctx, torch, layout):
    """ingot_rec8 == the documented encoding of the oracle's ingot_rec."""
    n = 150_001
    for chain in BASE_CHAINS:
        if layout == "indexed":
            arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, n, seed=21)
            got = ctx.parse_compact(arena, off, lens, chain)
            want = oracle.parse_batch(host(arena), host(off), host(lens), chain, nthreads=8)
        else:
            arena, _, lens = ingot_amd.gen_frames(GenProfile.VLAN_V6EH, n, seed=22, stride=128)
            got = ctx.parse_strided_compact(arena, 128, n, chain, lens=lens)
            want = oracle.parse_batch(host(arena), None, host(lens), chain, stride=128, n=n,
                                      nthreads=8)
        torch.cuda.synchronize()
        w8 = ingot_amd.rec16_to_rec8(want)
        g = got.cpu().numpy().reshape(n, 8)
        bad = np.nonzero((g != w8.view(np.uint8).reshape(n, 8)).any(axis=1))[0]
        assert bad.size == 0, (chain, bad[:5])
    # the tunnel's inner offsets do not fit ingot_rec8: refused, not wrong
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, 100, seed=23)
    with pytest.raises(RuntimeError):
        ctx.parse_compact(arena, off, lens, TUN)


def test_every_window_setting_is_bit_exact(torch):
    """Tuning never changes results: every staged-window size (incl. no
    staging, where every byte comes through the HBM path) on fuzz frames."""
    from ingot_amd.abi import TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED

    arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, 60_000, seed=31)
    sarena, _, slens = ingot_amd.gen_frames(GenProfile.VLAN_V6EH, 40_000, seed=32, stride=256)
    want_i = {c: oracle_all(arena, off, lens, c) for c in Chain}
    want_s = {c: oracle_all(sarena, None, slens, c, stride=256, n=40_000) for c in Chain}
    for w in (2, 3, 4, 5, 6, 8, 9, 100, 22, 23, 24, 25, 26, 28, 29, 1045, 1069, 1099):
        c = ingot_amd.Context(0)
        c.set_tuning(TUNE_WINDOW_INDEXED, w)
        if w in (2, 3, 4, 5, 8, 100):
            c.set_tuning(TUNE_WINDOW_STRIDED, w)
        for chain in Chain:
            r = c.parse(arena, off, lens, chain)
            if w > 20:  # line-completing windows: 8-B records and packed frames too
                r8 = c.parse_compact(arena, off, lens, chain) if chain != TUN else None
                rp = c.parse_packed(arena, lens, chain)
                torch.cuda.synchronize()
                assert rp.cpu().numpy().tobytes() == want_i[chain][0].tobytes(), (w, chain)
                if r8 is not None:
                    w8 = ingot_amd.rec16_to_rec8(want_i[chain][0])
                    assert r8.cpu().numpy().tobytes() == w8.tobytes(), (w, chain)
            f = dev_fields(c, arena, off, lens, chain)
            rs = c.parse_strided(sarena, 256, 40_000, chain, lens=slens)
            fs = dev_fields(c, sarena, None, slens, chain, stride=256, n=40_000)
            torch.cuda.synchronize()
            assert r.cpu().numpy().tobytes() == want_i[chain][0].tobytes(), (w, chain)
            assert f.cpu().numpy().tobytes() == want_i[chain][1].tobytes(), (w, chain)
            assert rs.cpu().numpy().tobytes() == want_s[chain][0].tobytes(), (w, chain)
            assert fs.cpu().numpy().tobytes() == want_s[chain][1].tobytes(), (w, chain)


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 1000])
def test_small_and_ragged_batches(ctx, torch, n):
    arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, max(n, 1), seed=n + 1)
    if n == 0:
        off, lens = off[:0], lens[:0]
        recs = ctx.parse(arena, off, lens, Chain.GenericUlp)
        torch.cuda.synchronize()
        assert recs.shape == (0, 16)
        return
    oracle_check(ctx, torch, arena, off, lens, Chain.GenericUlp)


def test_window_boundary_and_long_chains(ctx, torch):
    """Headers that end exactly at, or run far past, the 128-B LDS window
    (long IPv4/TCP options, long EH chains) take the HBM path for the bytes
    beyond the window; results must not change."""
    frames = []
    rng = np.random.default_rng(1)
    for doff in range(5, 16):
        for ihl in range(5, 16):
            v4 = bytearray(ihl * 4)
            v4[0] = 0x40 | ihl
            v4[9] = 6
            tcp = bytearray(doff * 4)
            tcp[12] = doff << 4
            f = bytes(12) + b"\x08\x00" + bytes(v4) + bytes(tcp)
            for extra in (0, 1, 7):
                frames.append(f + bytes(extra))
            frames.append(f[:-1])
    for n_eh in range(0, 12):
        for ext in (0, 1, 3, 30):
            v6 = bytearray(40)
            v6[0] = 0x60
            v6[6] = 0 if n_eh else 17
            body = b""
            for k in range(n_eh):
                nh = 60 if k + 1 < n_eh else 17
                body += bytes([nh, ext]) + rng.integers(0, 256, 6 + 8 * ext,
                                                          dtype=np.uint8).tobytes()
            f = bytes(12) + b"\x86\xdd" + bytes(v6) + body + bytes([0, 1, 0, 2, 0, 8, 0, 0])
            frames.append(f)
            frames.append(f[:-9])
    # random misalignment
    for chain in Chain:
        recs, flds = ingot_amd.parse_frames(frames, chain)
        for i, f in enumerate(frames):
            orec, ofld = oracle.parse_one(f, chain)
            if chain == TUN:
                ofld = oracle.parse_geneve(f)
            assert recs[i].tobytes() == orec.tobytes(), (i, recs[i], orec)
            assert flds[i].tobytes() == ofld.tobytes(), i


# ---------------------------------------------------------------------------
# full benchmark sizes: properties + sampled re-check
# ---------------------------------------------------------------------------
def test_config3_full_size_properties(ctx, torch):
    """Config 3 at its full size: 16,777,216 mixed 64-1500 B frames (~13 GB)."""
    n = 16 * (1 << 20)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    recs = ctx.parse(arena, off, lens, Chain.GenericUlp)
    torch.cuda.synchronize()
    r = recs.view(torch.int32).view(n, 4)
    status = recs[:, 0]
    assert int((status != 0).sum()) == 0
    l3 = recs[:, 2].to(torch.int64)
    frac_v6 = float((l3 == 2).double().mean())
    assert 0.49 < frac_v6 < 0.51
    payload = r[:, 3] & 0xFFFF
    assert bool((payload.to(torch.int64) <= lens.to(torch.int64)).all())
    # determinism: a second run is identical
    recs2 = ctx.parse(arena, off, lens, Chain.GenericUlp)
    torch.cuda.synchronize()
    assert torch.equal(recs, recs2)
    # sampled oracle re-check on the exact device bytes
    idx = np.random.default_rng(0).choice(n, 4096, replace=False)
    offs = host(off)[idx]
    ls = host(lens)[idx]
    frames = [host(arena[int(o):int(o) + int(ln)]).tobytes() for o, ln in zip(offs, ls)]
    got = ingot_amd.records_to_numpy(recs[torch.as_tensor(idx, device=recs.device)])
    for k, f in enumerate(frames):
        orec, _ = oracle.parse_one(f, Chain.GenericUlp)
        assert got[k].tobytes() == orec.tobytes(), idx[k]
    del arena, off, lens, recs, recs2
    torch.cuda.empty_cache()


def test_config4_shard_full_size_and_shard_consistency(ctx, torch):
    """Config 4 at its per-GPU size: one 8,388,608-frame shard of the 64 M
    VLAN/QinQ + IPv6-EH batch (VlanUlp).  Properties over the whole shard, a
    sampled oracle re-check, and shard consistency: the generator is pure in
    (seed, index), so rank r's shard equals frames [r*n, (r+1)*n) of one
    larger generation — the 8-GPU batch is the 1-GPU batch cut in eight."""
    from ingot_amd import dist as idist

    n = 8 * (1 << 20)
    first, n = idist.shard(3, 8, n)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.VLAN_V6EH, n, first=first)
    recs = ctx.parse(arena, off, lens, Chain.VlanUlp)
    torch.cuda.synchronize()
    assert int((recs[:, 0] != 0).sum()) == 0
    nvlan = recs[:, 4].to(torch.int64)
    assert 0.45 < float((nvlan > 0).double().mean()) < 0.55
    assert int((nvlan > 2).sum()) == 0
    v6 = recs[:, 2] == 2
    assert 0.45 < float(v6.double().mean()) < 0.55
    assert int((recs[:, 5][v6] > 0).sum()) > 0  # extension headers occur
    idx = np.random.default_rng(1).choice(n, 2048, replace=False)
    offs, ls = host(off)[idx], host(lens)[idx]
    got = ingot_amd.records_to_numpy(recs[torch.as_tensor(idx, device=recs.device)])
    for k, (o, ln) in enumerate(zip(offs, ls)):
        orec, _ = oracle.parse_one(host(arena[int(o):int(o) + int(ln)]).tobytes(), Chain.VlanUlp)
        assert got[k].tobytes() == orec.tobytes(), idx[k]
    # shard consistency: the first 1000 frames of this shard, regenerated as
    # part of a batch that starts 1000 frames earlier, have the same lengths,
    # header bytes and records (payload filler depends on the arena position)
    a2, o2, l2 = ingot_amd.gen_frames(GenProfile.VLAN_V6EH, 2000, first=first - 1000)
    assert torch.equal(l2[1000:].cpu(), lens[:1000].cpu())
    r2 = ctx.parse(a2, o2, l2, Chain.VlanUlp)
    torch.cuda.synchronize()
    assert torch.equal(r2[1000:], recs[:1000])
    poff = ingot_amd.records_to_numpy(recs[:1000])["payload_off"]
    for k in range(0, 1000, 7):
        f1 = arena[int(off[k]):int(off[k]) + int(poff[k])]
        f2 = a2[int(o2[1000 + k]):int(o2[1000 + k]) + int(poff[k])]
        assert torch.equal(f1, f2), k
    del arena, off, lens, recs
    torch.cuda.empty_cache()


def test_config5_full_size_flow_histogram(ctx, torch):
    """Config 5 at its per-GPU size (8,388,608 frames, 65,536 bins): the
    histogram is the bincount of the per-packet flow ids, counts every Ok
    packet with an L3 layer exactly once, and sampled flow ids equal the
    oracle's hash of the frame."""
    n = 8 * (1 << 20)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n, hashes=hashes,
                         workspace=ctx.flow_hist_workspace(n, 1 << 16))
    recs = ctx.parse(arena, off, lens, Chain.VlanUlp)
    torch.cuda.synchronize()
    f = flow.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    counted = f != 0xFFFFFFFF
    want = torch.bincount(f[counted], minlength=1 << 16)
    assert torch.equal(hist.to(torch.int64), want)
    ok_l3 = (recs[:, 0] == 0) & (recs[:, 2] != 0)
    assert torch.equal(counted, ok_l3)
    assert int(hist.to(torch.int64).sum()) == int(ok_l3.sum())
    idx = np.random.default_rng(2).choice(n, 2048, replace=False)
    offs, ls = host(off)[idx], host(lens)[idx]
    g_hash = hashes.cpu().numpy().view(np.uint32)[idx]
    for k, (o, ln) in enumerate(zip(offs, ls)):
        fr = host(arena[int(o):int(o) + int(ln)])
        _, w = oracle.flow_hist(np.concatenate([fr, np.zeros(8, np.uint8)]), np.array([0]),
                                np.array([int(ln)]), Chain.VlanUlp)
        assert g_hash[k] == w[0], idx[k]
    del arena, off, lens, recs, flow, hashes
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# maximum sizes: 65,535-byte frames, offsets near the u16 limit
# ---------------------------------------------------------------------------
def _max_frames():
    """Frames at the ABI's size limits, built field by field: an IPv6 frame
    whose extension-header chain (31 x 2,048-B RFC 6564 headers) puts the UDP
    header ~63.5 KB in; a 65,535-byte IPv4 frame with ihl 15 and TCP
    data_offset 15; the same two cut inside the last header; and a frame that
    ends exactly at its last header."""
    eth6 = bytes(12) + b"\x86\xdd"
    eh = []
    for k in range(31):
        nh = 60 if k < 30 else 17  # Destination Options ... -> UDP
        eh.append(bytes([nh, 255]) + bytes(6 + 8 * 255))
    v6 = bytes([0x60, 0, 0, 0, 0, 0, 60, 64]) + bytes(32)
    udp = b"\x12\x34\x56\x78\x00\x08\x00\x00"
    f1 = eth6 + v6 + b"".join(eh) + udp
    f1 = f1 + bytes(65535 - len(f1))
    v4 = bytes([0x4F, 0, 0, 0, 0, 0, 0, 0, 64, 6, 0, 0]) + bytes(8) + bytes(40)
    tcp = b"\x00\x50\x01\xbb" + bytes(8) + bytes([0xF0, 0x18]) + bytes(6) + bytes(40)
    f2 = bytes(12) + b"\x08\x00" + v4 + tcp
    f2 = f2 + bytes(65535 - len(f2))
    hdr1 = 14 + 40 + 31 * 2048 + 8
    return [f1, f2, f1[:hdr1 - 3], f1[:14 + 40 + 30 * 2048 + 100], f2[:14 + 60 + 59],
            f1[:hdr1], f2[:14 + 60 + 60]]


@pytest.mark.parametrize("chain", BASE_CHAINS)
def test_maximum_size_frames(ctx, torch, chain):
    """Records and every getter of 65,535-byte frames (offsets near the u16
    limit, headers ~63 KB past the staged window) equal the oracle's, in the
    packed layout and in 65,520-byte slots."""
    from tests.frames import pack

    frames = _max_frames() * 70  # > one 64-packet tile
    a_np, o_np, l_np = pack(frames)
    arena = torch.from_numpy(a_np).cuda()
    off = torch.from_numpy(o_np.astype(np.int64)).cuda()
    lens = torch.from_numpy(l_np.astype(np.uint16)).cuda()
    r = ctx.parse(arena, off, lens, chain)
    f = dev_fields(ctx, arena, off, lens, chain)
    torch.cuda.synchronize()
    w_rec, w_fld = oracle_all(arena, off, lens, chain)
    assert r.cpu().numpy().tobytes() == w_rec.tobytes()
    assert f.cpu().numpy().tobytes() == w_fld.tobytes()
    if chain == Chain.GenericUlp:
        rr = ingot_amd.records_to_numpy(r)
        assert int(rr["payload_off"][0]) == 14 + 40 + 31 * 2048 + 8  # 63,558
        assert int(rr["status"][0]) == 0 and int(rr["n_v6ext"][0]) == 31
    # fixed slots of the largest stride the ABI takes (65,520 B)
    stride = 65520
    n = 14
    slots = np.zeros(stride * n + 256, np.uint8)
    sl = np.zeros(n, np.uint16)
    for i, fr in enumerate(frames[:n]):
        b = fr[:stride]
        slots[i * stride:i * stride + len(b)] = np.frombuffer(b, np.uint8)
        sl[i] = len(b)
    sarena = torch.from_numpy(slots).cuda()
    slens = torch.from_numpy(sl).cuda()
    rs = ctx.parse_strided(sarena, stride, n, chain, lens=slens)
    torch.cuda.synchronize()
    ws = oracle.parse_batch(slots, None, sl, chain, stride=stride, n=n)
    assert rs.cpu().numpy().tobytes() == ws.tobytes()


# ---------------------------------------------------------------------------
# arenas at any alignment (the staging aligns absolute addresses)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mis", [1, 3, 8, 15, 17])
def test_misaligned_arena_base(ctx, torch, mis):
    """The same frames in an arena whose base address is not 16-B aligned:
    records, getters, parse_packed, parse_read, flows and in-place rewrites
    equal the aligned arena's (and rewrites touch only the frames' bytes)."""
    from ingot_amd import EditOp, Field

    n = 20_011
    arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, n, seed=mis)
    big = torch.zeros(arena.numel() + 64, dtype=torch.uint8, device="cuda")
    big[mis:mis + arena.numel()] = arena
    view = big[mis:mis + arena.numel()]
    assert view.data_ptr() % 16 == mis % 16
    for chain in Chain:
        assert torch.equal(ctx.parse(view, off, lens, chain), ctx.parse(arena, off, lens, chain))
        assert torch.equal(dev_fields(ctx, view, off, lens, chain),
                           dev_fields(ctx, arena, off, lens, chain))
    assert torch.equal(ctx.parse_packed(view, lens, Chain.GenericUlp),
                       ctx.parse(arena, off, lens, Chain.GenericUlp))
    f1 = ctx.flow_hist(view, off, lens, Chain.VlanUlp)
    f2 = ctx.flow_hist(arena, off, lens, Chain.VlanUlp)
    assert torch.equal(f1, f2)
    # chunk lists: every frame one chunk
    pkt_seg = torch.arange(0, n + 1, dtype=torch.int32, device="cuda")
    r1, c1 = ctx.parse_read(view, off, lens.view(torch.int16), pkt_seg, Chain.GenericUlp)
    r2, c2 = ctx.parse_read(arena, off, lens.view(torch.int16), pkt_seg, Chain.GenericUlp)
    assert torch.equal(r1, r2) and torch.equal(c1, c2)
    # in-place rewrite: same bytes afterwards, padding around the view intact
    edits = [(2, Field.UDP_DESTINATION, EditOp.SUB, 1), (1, Field.V4_HOP_LIMIT, EditOp.SUB, 1),
             (2, Field.TCP_FLAGS, EditOp.XOR, 0x10)]
    a2 = arena.clone()
    ctx.parse_modify(view, off, lens, Chain.GenericUlp, edits)
    ctx.parse_modify(a2, off, lens, Chain.GenericUlp, edits)
    torch.cuda.synchronize()
    assert torch.equal(view, a2)
    assert int(big[:mis].abs().sum()) == 0 and int(big[mis + arena.numel():].sum()) == 0
