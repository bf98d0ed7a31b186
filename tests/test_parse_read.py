"""parse_read over multi-chunk packets (ingot-macros/src/
parse.rs:511-537): the device path (ingot_gpu_parse_read / *_fields_read)
against the oracle's restatement, which tests/test_oracle_golden.py pins to
the reference's multichunk / early-accept / straddle vectors."""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from tests.kat_check import check

pytestmark = pytest.mark.gpu
TUN = Chain.GeneveOverV6Tunnel
# header boundaries of the common chains, where splits are most interesting
EDGES = np.array([0, 1, 13, 14, 15, 18, 22, 30, 34, 38, 42, 54, 58, 62, 70, 74, 88, 94, 108,
                  116, 128])


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


def split(frames, seed):
    """Cut every frame into 1-4 chunks (edges biased to header boundaries,
    some empty chunks)."""
    rng = np.random.default_rng(seed)
    out = []
    for f in frames:
        k = int(rng.integers(0, 4))
        cuts = []
        for _ in range(k):
            c = int(rng.choice(EDGES)) if rng.random() < 0.6 else int(rng.integers(0, len(f) + 1))
            cuts.append(min(c, len(f)))
        cuts = sorted(cuts)
        bounds = [0] + cuts + [len(f)]
        chunks = [f[a:b] for a, b in zip(bounds, bounds[1:])]
        if rng.random() < 0.05:
            chunks.insert(int(rng.integers(0, len(chunks) + 1)), b"")
        out.append(chunks)
    return out


def frames_of(profile, n, seed):
    arena, off, lens = ingot_amd.gen_frames(profile, n, seed=seed)
    a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
    return [a[o[i]:o[i] + ln[i]].tobytes() for i in range(n)]


def run_device(ctx, torch, packets, chain, fields):
    arena, seg_off, seg_len, pkt_seg = oracle.segments(packets)
    dev = lambda x, dt: torch.from_numpy(x.view(dt)).cuda()  # noqa: E731
    d = (dev(arena, np.uint8), dev(seg_off, np.int64), dev(seg_len, np.int16),
         dev(pkt_seg, np.int32))
    out, chunk = ctx.parse_read(*d, chain, fields=fields)
    recs, _ = ctx.parse_read(*d, chain)
    torch.cuda.synchronize()
    return (out.cpu().numpy(), recs.cpu().numpy(), chunk.cpu().numpy().view(np.uint16),
            (arena, seg_off, seg_len, pkt_seg))


def test_read_kats_on_device(ctx, torch, kats):
    for kat in kats["read_kats"]:
        chain = Chain[kat["chain"]]
        kind = "geneve" if chain == TUN else "fields"
        chunks = [bytes.fromhex(c) for c in kat["chunks"]]
        out, recs, chunk, _ = run_device(ctx, torch, [chunks], chain, kind)
        dt = ingot_amd.GENEVE_FIELDS_DTYPE if chain == TUN else ingot_amd.FIELDS_DTYPE
        fld = out.reshape(-1).view(dt)[0]
        rec = recs.reshape(-1).view(ingot_amd.REC_DTYPE)[0]
        bad = check(kat, rec, fld, chunk=int(chunk[0]))
        assert not bad, f"{kat['name']}: {bad}"
        orec, ofld, och = oracle.parse_read(chunks, chain, fields=kind)
        assert rec.tobytes() == orec.tobytes() and fld.tobytes() == ofld.tobytes(), kat["name"]
        assert int(chunk[0]) == och


@pytest.mark.parametrize("chain", list(Chain))
def test_read_fuzz_bit_exact(ctx, torch, chain):
    prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
    frames = frames_of(prof, 40_000, seed=51 + int(chain))
    frames += frames_of(GenProfile.GENEVE if chain == TUN else GenProfile.VLAN_V6EH, 20_000,
                        seed=61)
    packets = split(frames, seed=int(chain))
    kind = "geneve" if chain == TUN else "fields"
    out, recs, chunk, segs = run_device(ctx, torch, packets, chain, kind)
    w_rec, w_fld, w_chunk = oracle.parse_read_batch(*segs, chain, fields=kind)
    n = len(packets)
    bad = np.nonzero((recs.reshape(n, 16) != w_rec.view(np.uint8).reshape(n, 16)).any(1))[0]
    assert bad.size == 0, (bad[:5], recs[bad[0]].view(ingot_amd.REC_DTYPE)[0], w_rec[bad[0]],
                           [len(c) for c in packets[bad[0]]])
    width = w_fld.dtype.itemsize
    fb = np.nonzero((out.reshape(n, width) != w_fld.view(np.uint8).reshape(n, width)).any(1))[0]
    assert fb.size == 0, (fb[:5], out[fb[0]].view(w_fld.dtype), w_fld[fb[0]])
    assert np.array_equal(chunk, w_chunk)
    st = w_rec["status"]
    assert (st == 0).any() and (st == ingot_amd.ParseError.StraddledHeader).any()


def test_reference_read_tests_read_alike(torch):
    """ingot-examples/src/tests.rs:120-187, 277-305, 381-423 via the mirror."""
    eth = bytes([0xFF] * 6 + [0xA, 0xB, 0xC, 0xD, 0xE, 0xF]) + b"\x86\xdd"
    v6 = bytearray(40)
    v6[6] = 17
    v6[23] = 1
    udp = bytes([0x17, 0xC2, 0x17, 0xC1, 0, 128, 0xFF, 0xFF])
    mystack = ingot_amd.UdpParser.parse_read([eth, bytes(v6), udp, b"\xaa" * 128])
    hdr = mystack.headers
    assert hdr.eth.source() == bytes([0xA, 0xB, 0xC, 0xD, 0xE, 0xF])
    assert hdr.l3.next_header() == 17 and hdr.l3.next_layer() == 17
    assert (hdr.l4.source(), hdr.l4.destination(), hdr.l4.length()) == (6082, 6081, 128)
    assert mystack.last_chunk is None
    assert mystack.data == [b"\xaa" * 128]

    arp = bytes([0xA8, 0x40, 0x25, 0x77, 0x77, 0x76, 0xA8, 0x40, 0x25, 0x77, 0x77, 0x77, 8, 6])
    parsed = ingot_amd.GenericUlp.parse_read([arp, bytes(range(8))])
    assert len(parsed.last_chunk) == 8 and parsed.data == []

    pkt = bytes.fromhex("aa000400ff10aa000400ff010800" "45000024000000" "00f0110000080808"
                        "08c0a80005" "00800035" "00080000")
    with pytest.raises(ingot_amd.PacketParseError) as e:
        ingot_amd.GenericUlp.parse_read([pkt[:16], pkt[16:]])
    assert (e.value.error(), e.value.header()) == (ingot_amd.ParseError.StraddledHeader,
                                                   "inner_l3")
    with pytest.raises(ingot_amd.PacketParseError) as e:
        ingot_amd.GenericUlp.parse_read([pkt[:16]])
    assert (e.value.error(), e.value.header()) == (ingot_amd.ParseError.TooSmall, "inner_l3")


def test_read_single_chunk_matches_parse(ctx, torch):
    """Whole frames as single chunks, C3-style traffic: every record equals
    parse_slice's except where a non-final layer ends the frame."""
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, 50_000, seed=71)
    pkt_seg = torch.arange(50_001, dtype=torch.int32, device="cuda")
    recs, chunk = ctx.parse_read(arena, off, lens, pkt_seg, Chain.GenericUlp)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp)
    torch.cuda.synchronize()
    assert torch.equal(recs, want)
    assert int(chunk.abs().max()) == 0


def split_many(frames, seed):
    """Cut every frame into 1-8 chunks (many short ones: every header in its
    own chunk, chunks past the fourth, empty chunks)."""
    rng = np.random.default_rng(seed)
    out = []
    for f in frames:
        k = int(rng.integers(0, 8))
        cuts = sorted(min(int(rng.choice(EDGES)) if rng.random() < 0.7
                          else int(rng.integers(0, len(f) + 1)), len(f)) for _ in range(k))
        bounds = [0] + cuts + [len(f)]
        out.append([f[a:b] for a, b in zip(bounds, bounds[1:])])
    return out


@pytest.mark.parametrize("plan", [0, 1, 11, 17])
def test_every_read_plan_is_bit_exact(torch, plan):
    """INGOT_TUNE_READ_PLAN: how chunk 0 is staged in LDS (line-completing
    3-5 pieces, or 4) never changes a record, a field block or the
    remainder's chunk index (1-8 chunks per packet, every chain)."""
    from ingot_amd.abi import TUNE_READ_PLAN

    c = ingot_amd.Context(0)
    c.set_tuning(TUNE_READ_PLAN, plan)
    for chain in Chain:
        prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
        frames = frames_of(prof, 15_000, seed=81 + int(chain))
        frames += frames_of(GenProfile.GENEVE if chain == TUN else GenProfile.VLAN_V6EH, 10_000,
                            seed=91)
        packets = split_many(frames, seed=plan * 7 + int(chain))
        kind = "geneve" if chain == TUN else "fields"
        out, recs, chunk, segs = run_device(c, torch, packets, chain, kind)
        w_rec, w_fld, w_chunk = oracle.parse_read_batch(*segs, chain, fields=kind)
        n = len(packets)
        bad = np.nonzero((recs.reshape(n, 16) != w_rec.view(np.uint8).reshape(n, 16)).any(1))[0]
        assert bad.size == 0, (chain, bad[:5], [len(x) for x in packets[bad[0]]])
        width = w_fld.dtype.itemsize
        fb = np.nonzero((out.reshape(n, width) != w_fld.view(np.uint8).reshape(n, width))
                        .any(1))[0]
        assert fb.size == 0, (chain, fb[:5])
        assert np.array_equal(chunk, w_chunk)


def test_reference_bench_shape(ctx, torch):
    """The reference's parse-read-v4 shape (ingot-examples/benches/packet.rs:
    130-134): one chunk per header, 14 / 20 / 8 B, then the payload, over the
    C2 frames; records equal the oracle's, the walk ends in the exhausted
    UDP chunk (index 2) and the payload chunk is left unread."""
    n = 20_000
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    a = arena.cpu().numpy()
    packets = [[a[64 * i:64 * i + 14].tobytes(), a[64 * i + 14:64 * i + 34].tobytes(),
                a[64 * i + 34:64 * i + 42].tobytes(), a[64 * i + 42:64 * i + 64].tobytes()]
               for i in range(n)]
    _, recs, chunk, segs = run_device(ctx, torch, packets, Chain.UdpParser, "fields")
    w_rec, _, w_chunk = oracle.parse_read_batch(*segs, Chain.UdpParser)
    assert recs.tobytes() == w_rec.tobytes()
    assert np.array_equal(chunk, w_chunk) and (w_chunk == 2).all()
    assert (w_rec["status"] == 0).all()


@pytest.mark.parametrize("chain", list(Chain))
def test_dense_chunk_table_matches(ctx, torch, chain):
    """ingot_gpu_parse_read_dense ((offset << 16) | length per chunk) gives
    the records, field blocks and chunk indices of the two-array form and
    of the oracle, 1-8 chunks per packet."""
    prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
    frames = frames_of(prof, 20_000, seed=101 + int(chain))
    packets = split_many(frames, seed=103 + int(chain))
    kind = "geneve" if chain == TUN else "fields"
    out, recs, chunk, segs = run_device(ctx, torch, packets, chain, kind)
    arena, seg_off, seg_len, pkt_seg = segs
    dense = (seg_off.astype(np.uint64) << np.uint64(16)) | seg_len.astype(np.uint64)
    d = (torch.from_numpy(arena).cuda(), torch.from_numpy(dense.view(np.int64)).cuda(),
         torch.from_numpy(pkt_seg.view(np.int32)).cuda())
    r2, c2 = ctx.parse_read_dense(*d, chain)
    f2, _ = ctx.parse_read_dense(*d, chain, fields=kind)
    torch.cuda.synchronize()
    assert r2.cpu().numpy().tobytes() == recs.tobytes()
    assert f2.cpu().numpy().tobytes() == out.tobytes()
    assert np.array_equal(c2.cpu().numpy().view(np.uint16), chunk)
    w_rec, _, w_chunk = oracle.parse_read_batch(*segs, chain)
    assert recs.tobytes() == w_rec.tobytes() and np.array_equal(chunk, w_chunk)
    # the dense call ignores INGOT_TUNE_READ_PLAN (17 once
    # switched it to another kernel)
    from ingot_amd.abi import TUNE_READ_PLAN

    c = ingot_amd.Context(0)
    c.set_tuning(TUNE_READ_PLAN, 17)
    r3, c3 = c.parse_read_dense(*d, chain)
    torch.cuda.synchronize()
    assert r3.cpu().numpy().tobytes() == recs.tobytes()
    assert np.array_equal(c3.cpu().numpy().view(np.uint16), chunk)


def scatter(packets, seed):
    """Place each packet's chunks in its own 256-B region in random order with
    random gaps (some before chunk 0, some inside chunk 0's staged window with
    gaps between them), and now and then let a chunk alias an earlier one's
    bytes (a repeated chunk).  Returns the chunk tables."""
    rng = np.random.default_rng(seed)
    region = 256
    arena = np.zeros(region * len(packets) + 64, dtype=np.uint8)
    offs, lens, pkt = [], [], [0]
    for i, chunks in enumerate(packets):
        base = region * i
        order = rng.permutation(len(chunks))
        pos = base + int(rng.integers(0, 16))
        at = {}
        for j in order:
            c = chunks[j]
            if pos + len(c) > base + region:
                pos = base  # too long for this layout: overlap is fine when content-equal
                c = b""
            arena[pos:pos + len(c)] = np.frombuffer(c, dtype=np.uint8)
            at[j] = (pos, len(c))
            pos += len(c) + int(rng.integers(0, 12))
        seq = [at[j] for j in range(len(chunks))]
        if len(seq) > 1 and rng.random() < 0.1:  # repeat chunk 0 as chunk 1
            seq.insert(1, seq[0])
        for o, ln in seq:
            offs.append(o)
            lens.append(ln)
        pkt.append(len(offs))
    return (arena, np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint16),
            np.array(pkt, dtype=np.uint32))


@pytest.mark.parametrize("plan", [0, 1])
def test_scattered_and_aliased_chunks(torch, plan):
    """Chunks out of memory order, with gaps, partly inside chunk 0's staged
    window and partly outside, and repeated chunks: the reads of later
    chunks come from wherever their bytes are (chunk 0's window or L2/HBM),
    records and chunk indices equal the oracle's."""
    from ingot_amd.abi import TUNE_READ_PLAN

    c = ingot_amd.Context(0)
    c.set_tuning(TUNE_READ_PLAN, plan)
    for chain in Chain:
        prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
        frames = frames_of(prof, 12_000, seed=131 + int(chain))
        frames += frames_of(GenProfile.GENEVE if chain == TUN else GenProfile.VLAN_V6EH, 8_000,
                            seed=137)
        packets = [[bytes(x) for x in p] for p in split_many(frames, seed=139 + int(chain))]
        arena, so, sl, ps = scatter(packets, seed=149 + int(chain))
        d = (torch.from_numpy(arena).cuda(), torch.from_numpy(so.view(np.int64)).cuda(),
             torch.from_numpy(sl.view(np.int16)).cuda(), torch.from_numpy(ps.view(np.int32)).cuda())
        recs, chunk = c.parse_read(*d, chain)
        torch.cuda.synchronize()
        w_rec, _, w_chunk = oracle.parse_read_batch(arena, so, sl, ps, chain)
        n = len(packets)
        r = recs.cpu().numpy()
        bad = np.nonzero((r.reshape(n, 16) != w_rec.view(np.uint8).reshape(n, 16)).any(1))[0]
        assert bad.size == 0, (chain, bad[:5])
        assert np.array_equal(chunk.cpu().numpy().view(np.uint16), w_chunk)


@pytest.mark.parametrize("lazy", [False, True])
@pytest.mark.parametrize("chain", list(Chain))
def test_first_chunk_descriptor_path_is_bit_exact(ctx, torch, chain, lazy):
    """ingot_gpu_parse_read_first: chunk 0's descriptor per packet, loaded
    beside the chunk bounds (lazy: INGOT_TUNE_READ_PLAN 17, the bounds loaded
    by the walk only when it leaves chunk 0 or fails in it).  Records and the
    remainder's chunk index equal the oracle's (and so ingot_gpu_parse_read's)
    over 1-8 chunks per packet, empty chunks and packets without chunks,
    including the read KATs."""
    from ingot_amd.abi import TUNE_READ_PLAN

    if lazy:
        ctx = ingot_amd.Context(0)
        ctx.set_tuning(TUNE_READ_PLAN, 17)
    prof = GenProfile.GENEVE_ADVERSARIAL if chain == TUN else GenProfile.ADVERSARIAL
    frames = frames_of(prof, 30_000, seed=71 + int(chain))
    frames += frames_of(GenProfile.GENEVE if chain == TUN else GenProfile.MIXED, 10_000, seed=73)
    packets = split_many(frames, seed=11 + int(chain)) + [[]] * 3 + [[b""], [b"", b""]]
    arena, seg_off, seg_len, pkt_seg = oracle.segments(packets)
    dev = lambda x, dt: torch.from_numpy(x.view(dt)).cuda()  # noqa: E731
    d = (dev(arena, np.uint8), dev(seg_off, np.int64), dev(seg_len, np.int16),
         dev(pkt_seg, np.int32))
    first = ingot_amd.first_chunks(d[1], d[2], d[3])
    recs, chunk = ctx.parse_read(*d, chain, first=first)
    torch.cuda.synchronize()
    w_rec, _, w_chunk = oracle.parse_read_batch(arena, seg_off, seg_len, pkt_seg, chain)
    n = len(packets)
    got = recs.cpu().numpy().reshape(n, 16)
    bad = np.nonzero((got != w_rec.view(np.uint8).reshape(n, 16)).any(1))[0]
    assert bad.size == 0, (chain, bad[:5], [len(x) for x in packets[bad[0]]])
    assert np.array_equal(chunk.cpu().numpy().view(np.uint16), w_chunk)


@pytest.mark.parametrize("path", ["two_array", "first", "first_lazy", "dense"])
def test_layer_order_audit_on_device(ctx, torch, kats, path):
    """The layer-boundary audit (tests/test_read_order.py): every golden frame
    through every chain, cut at each layer boundary into [head],
    [head | tail] and [head | empty | tail] and at every byte into two chunks.
    Device records and chunk indices equal the oracle's, which equal the
    driver model's (parse.rs:357-416: slice step before the from=
    conversion)."""
    from ingot_amd.abi import TUNE_READ_PLAN
    from tests.test_read_order import audit_cases, compare, expected

    cases = audit_cases(kats)
    want = expected(cases)
    c = ctx
    if path == "first_lazy":
        c = ingot_amd.Context(0)
        c.set_tuning(TUNE_READ_PLAN, 17)
    for chain in Chain:
        sub = [x for x in cases if x[0] == chain]
        sub_want = [w for x, w in zip(cases, want) if x[0] == chain]
        arena, seg_off, seg_len, pkt_seg = oracle.segments([x[1] for x in sub])
        dev = lambda x, dt: torch.from_numpy(x.view(dt)).cuda()  # noqa: E731
        d = (dev(arena, np.uint8), dev(seg_off, np.int64), dev(seg_len, np.int16),
             dev(pkt_seg, np.int32))
        if path == "dense":
            dense = (seg_off.astype(np.uint64) << np.uint64(16)) | seg_len.astype(np.uint64)
            recs, chunk = c.parse_read_dense(d[0], dev(dense, np.int64), d[3], chain)
        elif path == "two_array":
            recs, chunk = c.parse_read(*d, chain)
        else:
            recs, chunk = c.parse_read(*d, chain, first=ingot_amd.first_chunks(d[1], d[2], d[3]))
        torch.cuda.synchronize()
        rec = recs.cpu().numpy().view(ingot_amd.REC_DTYPE).reshape(-1)
        ch = chunk.cpu().numpy().view(np.uint16)
        bad = compare(sub, sub_want, rec, ch)
        assert not bad, (path, chain.name, len(bad), bad[:5])
        w_rec, _, w_chunk = oracle.parse_read_batch(arena, seg_off, seg_len, pkt_seg, chain)
        assert rec.tobytes() == w_rec.tobytes() and np.array_equal(ch, w_chunk), (path, chain)


def test_first_chunks_helper(torch):
    """first_chunks(): (offset << 16) | length of each packet's chunk 0, 0
    for a packet without chunks."""
    so = torch.tensor([100, 7, 3000, 5], dtype=torch.int64)
    sl = torch.tensor([14, 20, -1, 1], dtype=torch.int16)  # -1: a 65,535-B chunk
    ps = torch.tensor([0, 2, 2, 3, 4], dtype=torch.int32)
    f = ingot_amd.first_chunks(so, sl, ps).tolist()
    assert f == [(100 << 16) | 14, 0, (3000 << 16) | 65535, (5 << 16) | 1]
