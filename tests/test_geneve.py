"""GeneveOverV6Tunnel (ingot-examples/src/packets.rs:27-40), the §8f-1 chain.

CPU (oracle) tests: the tunnel chain restated in oracle/ingot_oracle.c is
pinned by the reference's Geneve vectors in tests/golden/kats.json
(test_oracle_golden.py); here, metamorphic properties that tie it to the
already-pinned GenericUlp chain — wrapping any frame in a valid outer
Eth/IPv6/UDP/Geneve leaves its GenericUlp result unchanged, shifted by the
outer length and by 4 layer labels.

GPU tests (`-m gpu`): records and 384-B field blocks bit-exact against the
oracle on tunnel fuzz and on the C6 traffic profile, in both layouts and at
every staged-window size; the per-packet mirror reads like the reference
test; RSS flows over the inner 5-tuple; full-size properties.
"""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile, ParseError
from ingot_amd.abi import REC_ACCEPTED, REC_INNER
from tests.frames import build_frames, geneve_outer, pack

TUN = Chain.GeneveOverV6Tunnel
OPTE_IN = bytes.fromhex(
    "a84025777776a8402577777786dd" "60000000" "001011f0"
    + "fd000000" "00f70101" "00000000" "00000002" "fd000000" "00f70101" "00000000" "00000001"
    + "1e6117c100140000" "01006558" "0004d200" "01290000"
    + "aa000400ff10aa000400ff010800"
    + "45000024000000" "00f0110000080808" "08c0a80005" "0080003500080000" "0001020304050607")


def _opts(rng):
    k = int(rng.integers(0, 4))
    if k == 0:
        return ()
    if k == 1:
        return ((0x0129, 0, b""),)
    if k == 2:
        return ((0x0129, 0, b""), (0x0102, int(rng.integers(0, 256)), bytes(4)))
    return ((0x0102, 0x80, bytes(8)),)


def test_opte_frame_is_the_reference_bytes(kats):
    k = next(k for k in kats["chain_kats"] if k["name"] == "test_tunnelled_unconditionals")
    assert OPTE_IN.hex() == k["frame"]


def test_wrapping_preserves_generic_ulp_result():
    """oracle(GeneveOverV6Tunnel, outer + F) == oracle(GenericUlp, F), with
    layers 0..2 -> 4..6 and every offset shifted by len(outer)."""
    rng = np.random.default_rng(7)
    inner = build_frames(3000, seed=8, vlan=True, broken=0.2)
    inner += [bytes(int(rng.integers(0, 256)) for _ in range(int(rng.integers(0, 40))))
              for _ in range(500)]
    for f in inner:
        outer = geneve_outer(rng, _opts(rng), hbh=bool(rng.random() < 0.3))
        o = len(outer)
        r_in, _ = oracle.parse_one(f, Chain.GenericUlp)
        g = oracle.parse_geneve(outer + f)
        r = g["inner"]["rec"]
        assert int(r["status"]) == int(r_in["status"])
        if r_in["status"] != 0:
            assert int(r["err_layer"]) == int(r_in["err_layer"]) + 4
        else:
            assert int(r["err_layer"]) == 0xFF
        if len(f) < 14:
            continue  # inner_eth failed: the record still describes the outer walk
        assert int(r["flags"]) == int(r_in["flags"]) | REC_INNER
        for k in ("l3_kind", "l4_kind", "n_vlan", "n_v6ext", "l4_proto", "ethertype"):
            assert int(r[k]) == int(r_in[k]), k
        for k in ("l3_off", "l4_off", "payload_off"):
            want = int(r_in[k]) + o if (k == "payload_off" or int(r_in[k])) else 0
            assert int(r[k]) == want, k
        assert int(g["outer"]["inner_eth_off"]) == o
        # the inner getters are GenericUlp's, offsets shifted
        _, f_in = oracle.parse_one(f, Chain.GenericUlp)
        for name in ("eth_ethertype", "v4_total_len", "v6_flow_label", "l4_source",
                     "tcp_sequence", "udp_length", "icmp_ty"):
            assert int(g["inner"][name]) == int(f_in[name]), name


def test_outer_getters_match_builder():
    rng = np.random.default_rng(9)
    for _ in range(300):
        opts = _opts(rng)
        vni = int(rng.integers(0, 1 << 24))
        flags = int(rng.integers(0, 256))
        hbh = bool(rng.random() < 0.5)
        outer = geneve_outer(rng, opts, hbh=hbh, vni=vni, flags=flags)
        g = oracle.parse_geneve(outer + OPTE_IN[74:])
        t = g["outer"]
        assert int(g["inner"]["rec"]["status"]) == 0
        assert int(t["geneve_vni"]) == vni
        assert int(t["geneve_flags"]) == flags & 0xC0  # from_bits_truncate
        assert int(t["geneve_n_opts"]) == len(opts)
        assert int(t["outer_v6_n_ext"]) == int(hbh)
        assert int(t["outer_udp_destination"]) == 6081
        assert int(t["geneve_critical"]) == int(any(ty & 0x80 for _, ty, _ in opts))
        for i, (cls, ty, data) in enumerate(opts):
            e = t["geneve_opt"][i]
            assert (int(e["opt_class"]), int(e["option_type"]), int(e["length"])) == \
                (cls, ty, len(data) // 4)


def test_every_truncation_of_the_reference_frame():
    labels = ingot_amd.CHAIN_LABELS[TUN]
    bounds = [(14, 0), (54, 1), (62, 2), (74, 3), (88, 4), (108, 5), (116, 6)]
    for cut in range(len(OPTE_IN) + 1):
        r = oracle.parse_geneve(OPTE_IN[:cut])["inner"]["rec"]
        want = next((lay for end, lay in bounds if cut < end), None)
        if want is None:
            assert int(r["status"]) == 0
        else:
            assert (ParseError(int(r["status"])), labels[int(r["err_layer"])]) == \
                (ParseError.TooSmall, labels[want]), cut


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
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


def _check(ctx, torch, arena, off, lens, stride=0, n=None, fields=True):
    if off is not None:
        n = off.numel()
        recs = ctx.parse(arena, off, lens, TUN)
    else:
        recs = ctx.parse_strided(arena, stride, n, TUN, lens=lens)
    flds = ctx.geneve_fields(arena, off, lens, stride=stride, n=n) if fields else None
    torch.cuda.synchronize()
    want = oracle.parse_batch(host(arena), host(off), host(lens), TUN, stride=stride, n=n,
                              nthreads=8)
    g = ingot_amd.records_to_numpy(recs)
    bad = np.nonzero(g.view(np.uint8).reshape(n, 16) != want.view(np.uint8).reshape(n, 16))[0]
    assert bad.size == 0, f"{np.unique(bad).size} record mismatches: {g[bad[0]]} vs {want[bad[0]]}"
    if fields:
        wf = oracle.geneve_fields_batch(host(arena), host(off), host(lens), stride=stride, n=n)
        gf = flds.cpu().numpy().reshape(n, 384)
        fb = np.nonzero((gf != wf.view(np.uint8).reshape(n, 384)).any(axis=1))[0]
        assert fb.size == 0, (f"{fb.size} field mismatches, first {fb[:5]}: "
                              f"{gf[fb[0]].view(wf.dtype)} vs {wf[fb[0]]}")
    return g


@pytest.mark.gpu
def test_reference_test_reads_alike(torch):
    """ingot-examples/src/tests.rs:189-275 through the device mirror."""
    opte_in, hint, rest = ingot_amd.GeneveOverV6Tunnel.parse(OPTE_IN)
    assert opte_in.outer_encap.options_ref() == bytes([0x01, 0x29, 0, 0])
    assert len(opte_in.outer_encap.options_ref()) == 4
    assert opte_in.inner_eth.ethertype() == 0x0800
    assert opte_in.inner_l3 is not None
    assert opte_in.inner_ulp is not None
    assert opte_in.outer_encap.vni() == 0x4D2
    assert opte_in.outer_encap.options()[0].opt_class == 0x0129
    assert opte_in.outer_v6.next_header() == 17
    assert opte_in.outer_udp.destination() == 0x17C1
    assert rest == bytes(range(8))
    arp = bytearray(OPTE_IN)
    arp[74 + 12:74 + 14] = b"\x08\x06"
    opte_in, _, rest = ingot_amd.GeneveOverV6Tunnel.parse(bytes(arp))
    assert opte_in.inner_l3 is None
    assert opte_in.inner_ulp is None
    assert int(opte_in.rec["flags"]) & REC_ACCEPTED
    with pytest.raises(ingot_amd.PacketParseError) as e:
        ingot_amd.GeneveOverV6Tunnel.parse(OPTE_IN[:70])
    assert (e.value.header(), e.value.error()) == ("outer_encap", ParseError.TooSmall)


@pytest.mark.gpu
def test_tunnel_fuzz_bit_exact(ctx, torch):
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE_ADVERSARIAL, 200_000, seed=41)
    g = _check(ctx, torch, arena, off, lens)
    st, lay = g["status"], g["err_layer"]
    # every label and both outcomes are reached
    assert (st == 0).any()
    for layer in range(7):
        assert ((st != 0) & (lay == layer)).any(), layer
    assert (st == ParseError.Unwanted).any() and (st == ParseError.TooSmall).any()
    assert ((g["flags"] & REC_ACCEPTED) != 0).any()


@pytest.mark.gpu
def test_c6_profile_indexed_and_strided(ctx, torch):
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, 200_000, seed=42)
    g = _check(ctx, torch, arena, off, lens)
    assert (g["status"] == 0).all()
    assert ((g["flags"] & REC_INNER) != 0).all()
    acc = (g["flags"] & REC_ACCEPTED) != 0
    assert 0.01 < acc.mean() < 0.03  # inner ARP p .02
    sarena, _, slens = ingot_amd.gen_frames(GenProfile.GENEVE, 100_003, seed=43, stride=2048)
    _check(ctx, torch, sarena, None, slens, stride=2048, n=100_003)
    sarena, _, slens = ingot_amd.gen_frames(GenProfile.GENEVE_ADVERSARIAL, 100_003, seed=44,
                                            stride=256)
    _check(ctx, torch, sarena, None, slens, stride=256, n=100_003)


@pytest.mark.gpu
def test_tunnel_every_window_setting(torch):
    from ingot_amd.abi import TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED

    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE_ADVERSARIAL, 50_000, seed=45)
    for w in (2, 3, 4, 5, 6, 8, 9, 100):
        c = ingot_amd.Context(0)
        c.set_tuning(TUNE_WINDOW_INDEXED, w)
        if w not in (6, 9):
            c.set_tuning(TUNE_WINDOW_STRIDED, w)
        _check(c, torch, arena, off, lens)


@pytest.mark.gpu
def test_tunnel_flows_use_the_inner_tuple(ctx, torch):
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, 100_000, seed=46)
    hist = torch.zeros(4096, dtype=torch.int32, device="cuda")
    hashes = torch.zeros(100_000, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, TUN, hist=hist, hashes=hashes)
    torch.cuda.synchronize()
    want_h, want_hash = oracle.flow_hist(host(arena), host(off), host(lens), TUN, bins=4096)
    assert np.array_equal(hist.cpu().numpy().view(np.uint32), want_h)
    assert np.array_equal(hashes.cpu().numpy().view(np.uint32), want_hash)
    assert np.array_equal(flow.cpu().numpy().view(np.uint32), oracle.flow_hist.last_flows)


@pytest.mark.gpu
def test_tunnel_api_refusals(ctx, torch):
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, 64, seed=47)
    with pytest.raises(RuntimeError):
        ctx.fields(arena, off, lens, TUN)
    with pytest.raises(RuntimeError):
        ctx.parse_strided_compact(arena, 2048, 1, TUN)


@pytest.mark.gpu
def test_c6_full_size_properties(ctx, torch):
    """The C6 bench batch (4,194,304 tunnel frames): every frame Ok, the inner
    frame start equals the outer layers' length, a sample re-checked."""
    n = 1 << 22
    arena, off, lens = ingot_amd.gen_frames(GenProfile.GENEVE, n, seed=ingot_amd.GEN_SEED)
    recs = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, TUN))
    torch.cuda.synchronize()
    assert (recs["status"] == 0).all()
    assert ((recs["flags"] & REC_INNER) != 0).all()
    l3 = recs["l3_kind"] != 0
    # inner eth = l3_off - 14 >= 54 + 8 + 8 (+ options / HBH)
    assert (recs["l3_off"][l3].astype(np.int64) - 14 >= 70).all()
    idx = np.random.default_rng(5).choice(n, 20_000, replace=False)
    a, o, ln = host(arena), host(off), host(lens)
    for i in idx[:2000]:
        want = oracle.parse_one(a[o[i]:o[i] + ln[i]].tobytes(), TUN)[0]
        assert recs[i].tobytes() == want.tobytes(), i
