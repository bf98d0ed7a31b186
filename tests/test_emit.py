"""Batched Emit (ingot's `Emit`, ingot-types/src/emit.rs:8-120):
ingot_gpu_emit_packets / ingot_gpu_emit_headers against the oracle's
restatement, pinned by the tests/golden emit vectors (easy_tuple_emit,
roundtrip_emit_parse_unchanged, the reference tunnel frame re-encapsulated);
the host serialiser of owned headers (ingot_amd.emit) against the same
vectors; and emitted packets parsed back (Geneve over IPv6, contiguous and as
two-chunk packets through parse_read)."""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, EmitSource, Field, GenProfile
from ingot_amd import emit as E

TUN = Chain.GeneveOverV6Tunnel


def _build(stack) -> bytes:
    """A golden `stack` through the host serialiser (nested EH / option lists)."""
    out = b""
    for name, kw in stack:
        kw = dict(kw)
        for key in ("v6ext", "options"):
            if key in kw:
                kw[key] = _build(kw[key])
        for key in ("source", "destination", "data"):
            if isinstance(kw.get(key), list):
                kw[key] = bytes(kw[key])
        out += getattr(E, name)(**kw)
    return out


def _sets(kat, n=1, device=None, torch=None):
    """The KAT's setters; per-packet sources get n copies of the value (numpy,
    or a cuda tensor when torch is given)."""
    out = []
    for s in kat["sets"]:
        at, field, src, add = s[0], Field[s[1]], EmitSource[s[2]], s[3]
        if src in (EmitSource.U16, EmitSource.U32):
            dt = np.uint16 if src == EmitSource.U16 else np.uint32
            vals = np.full(n, s[4], dtype=dt)
            if torch is not None:
                vals = torch.from_numpy(vals.view(np.int16 if dt == np.uint16 else np.int32)
                                        ).to(device)
            out.append((at, field, src, add, vals))
        else:
            out.append((at, field, src, add))
    return out


def test_host_serialiser_matches_emit_kats(kats):
    for kat in kats["emit_kats"]:
        assert _build(kat["stack"]).hex() == kat["hdr"], kat["name"]


def test_oracle_emit_kats(kats):
    for kat in kats["emit_kats"]:
        if kat["after"] is None:
            continue
        hdr, pay = bytes.fromhex(kat["hdr"]), bytes.fromhex(kat["payload"])
        src = np.frombuffer(pay + bytes(16), dtype=np.uint8).copy()
        dst = np.zeros(len(hdr) + len(pay) + 8, np.uint8)
        oracle.emit_batch(hdr, _sets(kat), src, [0], [len(pay)], dst, [3])
        assert dst[3:3 + len(hdr) + len(pay)].tobytes().hex() == kat["after"], kat["name"]
        assert not dst[:3].any() and not dst[3 + len(hdr) + len(pay):].any()


def test_emitted_tunnel_frame_parses_back(kats):
    """The re-encapsulated reference frame parses as GeneveOverV6Tunnel with
    the setter values as its getters (oracle parse)."""
    kat = next(k for k in kats["emit_kats"] if k["name"] == "encap_per_packet_fields")
    g = oracle.parse_geneve(bytes.fromhex(kat["after"]))
    assert g["inner"]["rec"]["status"] == 0
    o = g["outer"]
    assert (int(o["outer_v6_payload_len"]), int(o["outer_udp_length"])) == (70, 70)
    assert (int(o["outer_udp_source"]), int(o["geneve_vni"])) == (0xC0DE, 0x123456)


# --------------------------------------------------------------------------
# On the device
# --------------------------------------------------------------------------
@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _u64(torch, a):
    return torch.from_numpy(np.asarray(a, dtype=np.uint64).view(np.int64)).cuda()


def _u16(torch, a):
    return torch.from_numpy(np.asarray(a, dtype=np.uint16).view(np.int16)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("dmis", [0, 1, 7, 15])
@pytest.mark.parametrize("smis", [0, 5, 12])
def test_emit_kats_on_device(ctx, torch, kats, dmis, smis):
    for kat in kats["emit_kats"]:
        if kat["after"] is None:
            continue
        hdr, pay = bytes.fromhex(kat["hdr"]), bytes.fromhex(kat["payload"])
        src = np.zeros(smis + len(pay) + 64, np.uint8)
        src[smis:smis + len(pay)] = np.frombuffer(pay, np.uint8)
        dst = _dev(torch, np.full(dmis + len(hdr) + len(pay) + 64, 0xEE, np.uint8))
        ctx.emit_packets(hdr, _sets(kat, 1, "cuda", torch), _dev(torch, src), _u64(torch, [smis]),
                         _u16(torch, [len(pay)]), dst, _u64(torch, [dmis]))
        got = dst.cpu().numpy()
        n = len(hdr) + len(pay)
        assert got[dmis:dmis + n].tobytes().hex() == kat["after"], (kat["name"], dmis, smis)
        assert (got[:dmis] == 0xEE).all() and (got[dmis + n:] == 0xEE).all()
        # the header block alone, at the same misalignment
        out = _dev(torch, np.full(dmis + len(hdr) + 64, 0xEE, np.uint8))
        ctx.emit_header_blocks(hdr, _sets(kat, 1, "cuda", torch), _u16(torch, [len(pay)]), out,
                               out_off=_u64(torch, [dmis]))
        o = out.cpu().numpy()
        assert o[dmis:dmis + len(hdr)].tobytes().hex() == kat["after"][:2 * len(hdr)]
        assert (o[:dmis] == 0xEE).all() and (o[dmis + len(hdr):] == 0xEE).all()


def _opte_stack():
    return (E.ethernet(bytes.fromhex("a84025777776"), bytes.fromhex("a84025777777"), 0x86DD)
            + E.ipv6(bytes.fromhex("fd000000f7010100000000000000000" + "2"),
                     bytes.fromhex("fd000000f7010100000000000000000" + "1"), 17,
                     hop_limit=0xF0, flow_label=0x12345)
            + E.udp(0, 6081)
            + E.geneve(0, options=E.geneve_opt(0x0129, 0) + E.geneve_opt(0x0102, 0x80,
                                                                            bytes(4))))


def _fuzz_sets(torch, n, rng):
    ports = rng.integers(0, 1 << 16, n, dtype=np.uint64).astype(np.uint16)
    vnis = rng.integers(0, 1 << 24, n, dtype=np.uint64).astype(np.uint32)
    host = [(14, Field.V6_PAYLOAD_LEN, EmitSource.LENGTH, -40),
            (54, Field.UDP_LENGTH, EmitSource.LENGTH, 0),
            (54, Field.UDP_SOURCE, EmitSource.U16, 0x10, ports),
            (62, Field.GENEVE_VNI, EmitSource.U32, 0, vnis),
            (14, Field.V6_FLOW_LABEL, EmitSource.U32, 7, vnis),
            (62, Field.GENEVE_FLAGS, EmitSource.VALUE, 0x40)]
    dev = [h if len(h) == 4 else (*h[:4], torch.from_numpy(
        h[4].view(np.int16 if h[4].dtype == np.uint16 else np.int32)).cuda()) for h in host]
    return host, dev


@pytest.mark.gpu
@pytest.mark.parametrize("profile,n", [("MIXED", 60_001), ("ADVERSARIAL", 40_000),
                                       ("GENEVE", 30_000)])
def test_emit_packets_fuzz_vs_oracle(ctx, torch, profile, n):
    """Whole packets: frames from the generator (their bytes are the payload),
    packed back to back in the destination with random gaps (0-40 B, so
    every misalignment meets every other), every setter source; the whole
    destination arena, gaps included, equals the oracle's."""
    rng = np.random.default_rng(7 + n)
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=9)
    hdr = _opte_stack()
    host_sets, dev_sets = _fuzz_sets(torch, n, rng)
    ln = lens.cpu().numpy()
    gaps = rng.integers(0, 41, n)
    tot = len(hdr) + ln.astype(np.int64)
    dst_off = np.cumsum(np.r_[0, (tot + gaps)[:-1]]) + 5
    size = int(dst_off[-1] + tot[-1] + 64)
    fill = rng.integers(0, 256, size, dtype=np.uint8)
    dst = _dev(torch, fill)
    ctx.emit_packets(hdr, dev_sets, arena, off, lens, dst, _u64(torch, dst_off))
    want = fill.copy()
    oracle.emit_batch(hdr, host_sets, arena.cpu().numpy(), off.cpu().numpy(), ln, want, dst_off)
    got = dst.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (profile, bad[:10])


@pytest.mark.gpu
def test_emit_jumbo_and_empty_payloads(ctx, torch):
    """Payloads from 0 B to 9,000 B (several 1 KiB passes per packet) and the
    largest header block (256 B)."""
    rng = np.random.default_rng(11)
    n = 3000
    ln = rng.integers(0, 9001, n).astype(np.uint16)
    ln[::7] = 0
    src_off = np.cumsum(np.r_[0, ln[:-1].astype(np.int64) + rng.integers(0, 20, n - 1)]) + 3
    src = rng.integers(0, 256, int(src_off[-1] + ln[-1] + 64), dtype=np.uint8)
    hdr = bytes(rng.integers(0, 256, 256, dtype=np.uint8))
    sets = [(200, Field.UDP_LENGTH, EmitSource.LENGTH, 0),
            (0, Field.ETH_ETHERTYPE, EmitSource.VALUE, 0x88B5),
            (220, Field.TCP_SEQUENCE, EmitSource.LENGTH, 1 << 31)]
    tot = 256 + ln.astype(np.int64)
    dst_off = np.cumsum(np.r_[0, tot[:-1]]) + 9
    fill = rng.integers(0, 256, int(dst_off[-1] + tot[-1] + 32), dtype=np.uint8)
    dst = _dev(torch, fill)
    ctx.emit_packets(hdr, sets, _dev(torch, src), _u64(torch, src_off), _u16(torch, ln), dst,
                     _u64(torch, dst_off))
    want = fill.copy()
    oracle.emit_batch(hdr, sets, src, src_off, ln, want, dst_off)
    assert (dst.cpu().numpy() == want).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 65, 257])
def test_emit_partial_groups_and_max_payload(ctx, torch, n):
    """Batches that leave the last packet group partial (a workgroup's waves
    then share fewer packets than they have lanes, some subgroups none) and
    payloads up to the u16 maximum (65,535 B: one packet's span alone is
    4,100 chunks)."""
    rng = np.random.default_rng(100 + n)
    ln = rng.integers(0, 2000, n).astype(np.uint16)
    ln[rng.integers(0, n, max(1, n // 8))] = 65535
    src_off = np.cumsum(np.r_[0, ln[:-1].astype(np.int64) + rng.integers(0, 20, n - 1)]) + 1
    src = rng.integers(0, 256, int(src_off[-1] + ln[-1] + 64), dtype=np.uint8)
    hdr = _opte_stack()
    sets = [(14, Field.V6_PAYLOAD_LEN, EmitSource.LENGTH, -40),
            (54, Field.UDP_LENGTH, EmitSource.LENGTH, 0)]
    tot = len(hdr) + ln.astype(np.int64)
    dst_off = np.cumsum(np.r_[0, tot[:-1] + rng.integers(0, 9, n - 1)]) + 7
    fill = rng.integers(0, 256, int(dst_off[-1] + tot[-1] + 32), dtype=np.uint8)
    dst = _dev(torch, fill)
    ctx.emit_packets(hdr, sets, _dev(torch, src), _u64(torch, src_off), _u16(torch, ln), dst,
                     _u64(torch, dst_off))
    want = fill.copy()
    oracle.emit_batch(hdr, sets, src, src_off, ln, want, dst_off)
    bad = np.nonzero(dst.cpu().numpy() != want)[0]
    assert bad.size == 0, (n, bad[:10])


@pytest.mark.gpu
def test_emit_gather_copy_without_headers(ctx, torch):
    """hdr_len 0: a gather copy (decapsulation: each tunnel frame's inner
    frame copied out from the offset the parse found)."""
    n = 20_000
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, n, seed=4)
    gf = ingot_amd.geneve_fields_to_numpy(ctx.geneve_fields(arena, off, lens))
    inner = gf["outer"]["inner_eth_off"].astype(np.int64)
    ok = gf["inner"]["rec"]["status"] == 0
    o = off.cpu().numpy().view(np.uint64).astype(np.int64)
    ln = lens.cpu().numpy().astype(np.int64)
    src_off = np.where(ok, o + inner, o)
    il = np.where(ok, ln - inner, 0).astype(np.uint16)
    dst_off = np.cumsum(np.r_[0, il[:-1].astype(np.int64)])
    dst = torch.zeros(int(dst_off[-1] + il[-1] + 16), dtype=torch.uint8, device="cuda")
    ctx.emit_packets(b"", [], arena, _u64(torch, src_off), _u16(torch, il), dst,
                     _u64(torch, dst_off))
    want = np.zeros(dst.numel(), np.uint8)
    oracle.emit_batch(b"", [], arena.cpu().numpy(), src_off, il, want, dst_off)
    assert (dst.cpu().numpy() == want).all()
    # the copied inner frames parse exactly as the tunnel parse's inner layers
    recs = ingot_amd.records_to_numpy(ctx.parse(dst, _u64(torch, dst_off), _u16(torch, il),
                                                Chain.GenericUlp))
    k = np.nonzero(ok)[0]
    assert (recs["status"][k] == gf["inner"]["rec"]["status"][k]).all()
    assert (recs["l4_kind"][k] == gf["inner"]["rec"]["l4_kind"][k]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["slots", "headroom"])
def test_emit_headers_modes(ctx, torch, mode):
    """Header blocks only: into fixed slots (the header chunk of a two-chunk
    packet) or into each frame's headroom (emit_suffix: the packet becomes
    contiguous in place); equal to the oracle, frame bytes untouched."""
    rng = np.random.default_rng(5)
    n = 50_000
    hdr = _opte_stack()
    H = len(hdr)
    ln = rng.integers(0, 1500, n).astype(np.uint16)
    host_sets, dev_sets = _fuzz_sets(torch, n, rng)
    if mode == "slots":
        stride = 96
        out = _dev(torch, np.full(n * stride + 16, 0xEE, np.uint8))
        ctx.emit_header_blocks(hdr, dev_sets, _u16(torch, ln), out, stride=stride)
        want = np.full(n * stride + 16, 0xEE, np.uint8)
        oracle.emit_batch(hdr, host_sets, None, None, ln, want, None, stride=stride, copy=False)
    else:
        room = rng.integers(0, 9, n)  # spare bytes beyond the header block
        frame_off = np.cumsum(np.r_[0, (ln[:-1].astype(np.int64) + H + room[:-1])]) + H + room[0]
        size = int(frame_off[-1] + ln[-1] + 16)
        fill = rng.integers(0, 256, size, dtype=np.uint8)
        out = _dev(torch, fill)
        ctx.emit_header_blocks(hdr, dev_sets, _u16(torch, ln), out,
                               out_off=_u64(torch, frame_off - H))
        want = fill.copy()
        oracle.emit_batch(hdr, host_sets, None, None, ln, want, frame_off - H, copy=False)
    got = out.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (mode, bad[:10])


@pytest.mark.gpu
def test_emit_then_parse_contiguous_and_two_chunk(ctx, torch):
    """Encapsulate generator frames, then parse the result as
    GeneveOverV6Tunnel both ways: contiguous packets (emit_packets) and
    two-chunk packets [header block slot | original frame] through parse_read
    (emit_headers) — the same records, whose inner layers are the original
    frames' GenericUlp parse shifted by the header block."""
    n = 40_000
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=13)
    hdr = _opte_stack()
    H = len(hdr)
    sets = [(14, Field.V6_PAYLOAD_LEN, EmitSource.LENGTH, -40),
            (54, Field.UDP_LENGTH, EmitSource.LENGTH, 0)]
    ln = lens.cpu().numpy().astype(np.int64)
    dst_off = np.cumsum(np.r_[0, ln[:-1] + H])
    dst = torch.zeros(int(dst_off[-1] + ln[-1] + H + 64), dtype=torch.uint8, device="cuda")
    ctx.emit_packets(hdr, sets, arena, off, lens, dst, _u64(torch, dst_off))
    tl = _u16(torch, ln + H)
    contiguous = ingot_amd.records_to_numpy(ctx.parse(dst, _u64(torch, dst_off), tl, TUN))
    stride = (H + 15) // 16 * 16
    slots = torch.zeros(n * stride + 64, dtype=torch.uint8, device="cuda")
    ctx.emit_header_blocks(hdr, sets, lens, slots, stride=stride)
    # one pool holding the header slots, then the frames
    pool = torch.cat([slots, arena])
    so = np.empty(2 * n, np.uint64)
    sl = np.empty(2 * n, np.uint16)
    so[0::2] = np.arange(n, dtype=np.uint64) * stride
    sl[0::2] = H
    so[1::2] = off.cpu().numpy().view(np.uint64) + slots.numel()
    sl[1::2] = ln
    ps = np.arange(0, 2 * n + 1, 2, dtype=np.uint32)
    rec = ctx.parse_read(pool, _u64(torch, so), _u16(torch, sl),
                         torch.from_numpy(ps.view(np.int32)).cuda(), TUN)
    two = ingot_amd.records_to_numpy(rec[0] if isinstance(rec, tuple) else rec)
    assert (contiguous["status"] == 0).all()
    for k in ("status", "l3_kind", "l4_kind", "l3_off", "l4_off", "payload_off", "flags"):
        assert (two[k] == contiguous[k]).all(), k
    plain = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, Chain.GenericUlp))
    okp = plain["status"] == 0
    assert (contiguous["l4_off"][okp] == plain["l4_off"][okp] + H).all()
    assert (contiguous["payload_off"][okp] == plain["payload_off"][okp] + H).all()


@pytest.mark.gpu
def test_emit_argument_errors(ctx, torch):
    import ctypes

    lib = ingot_amd.load_library()
    h = (ctypes.c_uint8 * 300)()
    buf = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    p = buf.data_ptr()
    s = ingot_amd.emit_sets_array([(0, Field.UDP_LENGTH, EmitSource.LENGTH, 0)])
    sp = s.ctypes.data_as(ctypes.c_void_p)
    a = ctypes.addressof(h)
    # header block too long, too many sets, field outside the block
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 257, None, 0, p, 1, p, None, 512, None) == -1
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 64, sp, 9, p, 1, p, None, 64, None) == -1
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 5, sp, 1, p, 1, p, None, 64, None) == -1
    # a setter offset past the block (at + byte offset would wrap in 16 bits)
    for at in (65535, 65534, 256):
        far = ingot_amd.emit_sets_array([(at, Field.UDP_DESTINATION, EmitSource.VALUE, 7)])
        assert lib.ingot_gpu_emit_headers(ctx._h, a, 64, far.ctypes.data_as(ctypes.c_void_p), 1,
                                          p, 1, p, None, 64, None) == -1, at
    # a U16 source without values; an unknown source / field
    bad = ingot_amd.emit_sets_array([(0, Field.UDP_SOURCE, EmitSource.U16, 0)])
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 8, bad.ctypes.data_as(ctypes.c_void_p), 1, p,
                                      1, p, None, 64, None) == -1
    bad = ingot_amd.emit_sets_array([(0, Field.UDP_SOURCE, 9, 0)])
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 8, bad.ctypes.data_as(ctypes.c_void_p), 1, p,
                                      1, p, None, 64, None) == -1
    # slots narrower than the block: ERANGE; missing buffers: EINVAL
    assert lib.ingot_gpu_emit_headers(ctx._h, a, 64, None, 0, p, 1, p, None, 32, None) == -5
    assert lib.ingot_gpu_emit_packets(ctx._h, a, 8, None, 0, p, None, p, 1, p, p, None) == -1
    assert lib.ingot_gpu_emit_packets(ctx._h, a, 8, None, 0, None, None, None, 0, None, None,
                                      None) == 0
    assert lib.ingot_gpu_emit_packets(None, a, 8, None, 0, p, p, p, 1, p, p, None) == -1
