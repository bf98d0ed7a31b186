"""Flow classification (config 5): RSS Toeplitz hash of the parsed 5-tuple and
the per-flow histogram.  Build-defined (ingot has no flow hash); the hash is
pinned by Microsoft's published RSS verification vectors
(tests/golden/kats.json "rss_kats"), the tuple extraction by the oracle."""
import ipaddress

import numpy as np
import pytest

import oracle
from ingot_amd import Chain
from tests.frames import build_frames, pack


def test_rss_verification_vectors(kats):
    rss = kats["rss_kats"]
    key = bytes.fromhex(rss["key"])
    assert key == oracle.RSS_KEY
    for v in rss["vectors"]:
        src = ipaddress.ip_address(v["src"]).packed
        dst = ipaddress.ip_address(v["dst"]).packed
        ports = v["sport"].to_bytes(2, "big") + v["dport"].to_bytes(2, "big")
        assert oracle.toeplitz(key, src + dst) == v["hash_addrs"], v
        assert oracle.toeplitz(key, src + dst + ports) == v["hash_ports"], v
        # appending zero bytes never changes a Toeplitz hash (used by the kernel)
        assert oracle.toeplitz(key, src + dst + bytes(4)) == v["hash_addrs"]


def _key_windows(key: bytes, nbits: int = 288):
    """W[b] = the 32 key bits starting at input bit b (FlowArgs::w, api.cpp)."""
    k = int.from_bytes(key, "big")
    kb = len(key) * 8
    return [(k >> (kb - 32 - b)) & 0xFFFFFFFF for b in range(nbits)]


def _toeplitz16_bit_parity(words, W):
    """k_flows_bits' form of the hash (walk.h toeplitz9_bits16): bit q of the
    low 16 bits = parity(XOR_k words[k] & W[32 k + 31 - q])."""
    h = 0
    for q in range(16):
        t = 0
        for k, x in enumerate(words):
            t ^= x & W[32 * k + 31 - q]
        h |= (bin(t).count("1") & 1) << q
    return h


def test_bit_parity_form_is_the_toeplitz_hash(kats):
    """The table-free hash of the default C5 kernel equals the Toeplitz hash's
    low 16 bits (the flow bin), on the RSS vectors and on random 36-B inputs."""
    key = bytes.fromhex(kats["rss_kats"]["key"])
    W = _key_windows(key)
    inputs = []
    for v in kats["rss_kats"]["vectors"]:
        src = ipaddress.ip_address(v["src"]).packed
        dst = ipaddress.ip_address(v["dst"]).packed
        ports = v["sport"].to_bytes(2, "big") + v["dport"].to_bytes(2, "big")
        inputs.append(src + dst + ports)
    rng = np.random.default_rng(5)
    inputs += [rng.integers(0, 256, 36, dtype=np.uint8).tobytes() for _ in range(200)]
    for data in inputs:
        data = data + bytes(36 - len(data))
        words = [int.from_bytes(data[4 * k:4 * k + 4], "big") for k in range(9)]
        assert _toeplitz16_bit_parity(words, W) == oracle.toeplitz(key, data) & 0xFFFF


def test_flow_hash_of_parsed_frames(kats):
    v = kats["rss_kats"]["vectors"][0]
    src = ipaddress.ip_address(v["src"]).packed
    dst = ipaddress.ip_address(v["dst"]).packed
    v4 = bytes([0x45, 0, 0, 0, 0, 0, 0, 0, 64, 6, 0, 0]) + src + dst
    tcp = v["sport"].to_bytes(2, "big") + v["dport"].to_bytes(2, "big") + bytes(8) + \
        bytes([0x50, 0]) + bytes(6)
    frame = bytes(12) + b"\x08\x00" + v4 + tcp
    hist, h = oracle.flow_hist(np.frombuffer(frame + bytes(8), np.uint8), np.array([0]),
                               np.array([len(frame)]), Chain.GenericUlp, bins=1 << 16)
    assert h[0] == v["hash_ports"] and hist[h[0] & 0xFFFF] == 1 and hist.sum() == 1
    # ICMP: addresses only
    v4i = bytes([0x45, 0, 0, 0, 0, 0, 0, 0, 64, 1, 0, 0]) + src + dst
    fi = bytes(12) + b"\x08\x00" + v4i + bytes(8)
    _, h = oracle.flow_hist(np.frombuffer(fi + bytes(8), np.uint8), np.array([0]),
                            np.array([len(fi)]), Chain.GenericUlp)
    assert h[0] == v["hash_addrs"]
    # errors and ARP-accepted frames are not counted
    for f in (frame[:30], bytes(12) + b"\x08\x06" + bytes(28)):
        hist, h = oracle.flow_hist(np.frombuffer(f + bytes(8), np.uint8), np.array([0]),
                                   np.array([len(f)]), Chain.GenericUlp)
        assert hist.sum() == 0 and h[0] == 0


def test_histogram_accumulates_and_matches_per_packet_hashes():
    frames = build_frames(3000, seed=4)
    arena, off, lens = pack(frames)
    hist, h = oracle.flow_hist(arena, off, lens, Chain.GenericUlp, bins=1024)
    counted = np.array([oracle.flow_hist(np.frombuffer(f + bytes(8), np.uint8), np.array([0]),
                                         np.array([len(f)]), Chain.GenericUlp)[0].sum()
                        for f in frames[:200]])
    assert set(np.unique(counted)) <= {0, 1}
    want = np.bincount(h[np.array([oracle.flow_hist(
        np.frombuffer(f + bytes(8), np.uint8), np.array([0]), np.array([len(f)]),
        Chain.GenericUlp)[0].sum() for f in frames]) == 1] & 1023, minlength=1024)
    assert (hist == want).all()
    hist2, _ = oracle.flow_hist(arena, off, lens, Chain.GenericUlp, bins=1024, hist=hist.copy())
    assert (hist2 == 2 * hist).all()


# ---------------------------------------------------------------------------
# device
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("profile,chain,stride", [
    ("FLOWS", "VlanUlp", None), ("ADVERSARIAL", "GenericUlp", None),
    ("MIXED", "UdpParser", None), ("VLAN_V6EH", "GenericUlp", 256), ("V4UDP64", "UdpParser", 64),
])
def test_flow_hist_bit_exact(profile, chain, stride):
    import torch

    import ingot_amd
    from ingot_amd import GenProfile

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 200_000
    ctx = ingot_amd.Context(0)
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=7, stride=stride)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain[chain], hist=hist, stride=stride or 0, n=n,
                         hashes=hashes, workspace=ctx.flow_hist_workspace(n, 1 << 16))
    torch.cuda.synchronize()
    host = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731
    w_hist, w_hash = oracle.flow_hist(host(arena), host(off), host(lens), Chain[chain],
                                      stride=stride or 0, n=n)
    w_flow = oracle.flow_hist.last_flows
    g_hash = hashes.cpu().numpy().view(np.uint32)
    bad = np.nonzero(g_hash != w_hash)[0]
    assert bad.size == 0, (bad[:5], g_hash[bad[:5]], w_hash[bad[:5]])
    assert (flow.cpu().numpy().view(np.uint32) == w_flow).all()
    assert (hist.cpu().numpy().view(np.uint32) == w_hist).all()
    # accumulation across calls; a histogram-free call (flows only) and small bins
    ctx.flow_hist(arena, off, lens, Chain[chain], hist=hist, stride=stride or 0, n=n)
    torch.cuda.synchronize()
    assert (hist.cpu().numpy().view(np.uint32) == 2 * w_hist).all()
    h64 = torch.zeros(64, dtype=torch.int32, device="cuda")
    ctx.flow_hist(arena, off, lens, Chain[chain], hist=h64, stride=stride or 0, n=n)
    torch.cuda.synchronize()
    w64 = np.bincount(w_hash[w_flow != 0xFFFFFFFF] & 63, minlength=64)
    assert (h64.cpu().numpy() == w64).all()
    if profile == "FLOWS":
        # Zipf(1.1) head: the top bin holds a large share
        assert w_hist.max() > 0.05 * w_hist.sum()


@pytest.mark.gpu
@pytest.mark.parametrize("tune", [{}, {"win": 3}, {"win": 4}, {"win": 5}, {"win": 8},
                                  {"blocks": 7}, {"blocks": 1, "win": 3}, {"blocks": 3},
                                  {"win": 25}, {"win": 26}, {"win": 28},
                                  {"win": 25, "blocks": 3}, {"win": 1045}, {"win": 1056},
                                  {"win": 1058}, {"win": 1025}, {"win": 1035}, {"fk": 15}])
@pytest.mark.parametrize("profile,chain,stride", [
    ("FLOWS", "VlanUlp", None), ("ADVERSARIAL", "GenericUlp", None),
    ("GENEVE_ADVERSARIAL", "GeneveOverV6Tunnel", None), ("VLAN_V6EH", "VlanUlp", 256),
])
def test_flow_kernels_every_setting(tune, profile, chain, stride):
    """Every staged window (so both the LDS burst and the word-by-word
    fallback of the hash input read) and tiny grid caps (many tiles per wave,
    ragged tail): flow ids and hashes bit-exact against the oracle."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile
    from ingot_amd.abi import (TUNE_FLOW_KERNEL, TUNE_MAX_BLOCKS, TUNE_WINDOW_INDEXED,
                               TUNE_WINDOW_STRIDED)

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 100_003
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_FLOW_KERNEL, tune.get("fk", 0))
    if "win" in tune and not (stride and tune["win"] > 20):  # 20 + k: offset-addressed only
        ctx.set_tuning(TUNE_WINDOW_STRIDED if stride else TUNE_WINDOW_INDEXED, tune["win"])
    if "blocks" in tune:
        ctx.set_tuning(TUNE_MAX_BLOCKS, tune["blocks"])
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=13, stride=stride)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain[chain], hist=hist, stride=stride or 0, n=n,
                         hashes=hashes, workspace=ctx.flow_hist_workspace(n, 1 << 16))
    torch.cuda.synchronize()
    host = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731
    w_hist, w_hash = oracle.flow_hist(host(arena), host(off), host(lens), Chain[chain],
                                      stride=stride or 0, n=n)
    w_flow = oracle.flow_hist.last_flows
    g_hash = hashes.cpu().numpy().view(np.uint32)
    bad = np.nonzero(g_hash != w_hash)[0]
    assert bad.size == 0, (bad[:5], g_hash[bad[:5]], w_hash[bad[:5]])
    assert (flow.cpu().numpy().view(np.uint32) == w_flow).all()
    assert (hist.cpu().numpy().view(np.uint32) == w_hist).all()


@pytest.mark.gpu
@pytest.mark.parametrize("table", [0, 32])
@pytest.mark.parametrize("tune", [{}, {"win": 3}, {"win": 4}, {"win": 8}, {"blocks": 5},
                                  {"blocks": 3}, {"win": 25}, {"win": 1025}, {"win": 1056},
                                  {"fk": 15}])
@pytest.mark.parametrize("bins", [1 << 16, 1024])
@pytest.mark.parametrize("profile,chain,stride", [
    ("FLOWS", "VlanUlp", None), ("ADVERSARIAL", "GenericUlp", None),
    ("GENEVE_ADVERSARIAL", "GeneveOverV6Tunnel", None), ("VLAN_V6EH", "VlanUlp", 256),
])
def test_flow_bins_without_hashes(table, tune, bins, profile, chain, stride):
    """No full hash requested and bins <= 65,536: the kernel uses the 16-bit
    lookup table (OUT_FLOWS16) unless INGOT_TUNE_FLOW_TABLE = 32 forces the
    32-bit one.  Flow ids and the histogram equal the oracle's either way."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile
    from ingot_amd.abi import (TUNE_FLOW_KERNEL, TUNE_FLOW_TABLE, TUNE_MAX_BLOCKS,
                               TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED)

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 100_003
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_FLOW_TABLE, table)
    ctx.set_tuning(TUNE_FLOW_KERNEL, tune.get("fk", 0))
    if "win" in tune and not (stride and tune["win"] > 20):  # 20 + k: offset-addressed only
        ctx.set_tuning(TUNE_WINDOW_STRIDED if stride else TUNE_WINDOW_INDEXED, tune["win"])
    if "blocks" in tune:
        ctx.set_tuning(TUNE_MAX_BLOCKS, tune["blocks"])
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=17, stride=stride)
    hist = torch.zeros(bins, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain[chain], hist=hist, stride=stride or 0, n=n,
                         workspace=ctx.flow_hist_workspace(n, bins))
    torch.cuda.synchronize()
    host = lambda t: None if t is None else t.cpu().numpy()  # noqa: E731
    w_hist, _ = oracle.flow_hist(host(arena), host(off), host(lens), Chain[chain],
                                 stride=stride or 0, n=n, bins=bins)
    w_flow = oracle.flow_hist.last_flows
    g = flow.cpu().numpy().view(np.uint32)
    bad = np.nonzero(g != w_flow)[0]
    assert bad.size == 0, (bad[:5], g[bad[:5]], w_flow[bad[:5]])
    assert (hist.cpu().numpy().view(np.uint32) == w_hist).all()


@pytest.mark.gpu
@pytest.mark.parametrize("ws", [False, True])
@pytest.mark.parametrize("bins", [1, 2, 4096, 1 << 16, 1 << 17, 1 << 20])
def test_flow_hist_bin_regimes(bins, ws):
    """Every histogram regime (workspace rows + reduce for <= 65,536 bins, LDS
    bin ranges, wave-aggregated atomics) equals the bincount of the flow ids,
    which the test above pins to the oracle; accumulation into a non-zero
    histogram too."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 300_000
    ctx = ingot_amd.Context(0)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=11)
    hist = torch.full((bins,), 3, dtype=torch.int32, device="cuda")
    work = ctx.flow_hist_workspace(n, bins) if ws else None
    assert (work is not None) == (ws and bins <= 65536)
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n, workspace=work)
    torch.cuda.synchronize()
    f = flow.cpu().numpy().view(np.uint32)
    want = np.bincount(f[f != 0xFFFFFFFF], minlength=bins) + 3
    assert (hist.cpu().numpy().view(np.uint32) == want).all()


@pytest.mark.gpu
def test_flow_hist_many_slices():
    """> 256 x 65,535 flow ids: the 16-bit pass splits into more slices than
    CUs so no per-block counter can wrap, even for a single hot flow."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    big = 256 * 65535 + 4097
    assert ctx.flow_hist_workspace_size(big, 1 << 16) == 0  # > 256 slices: range pass
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, big, stride=64)
    for n in (256 * 65535, big, 129 * 65535 + 1):
        work = ctx.flow_hist_workspace(n, 1 << 16)
        hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
        flow = ctx.flow_hist(arena, None, None, Chain.UdpParser, hist=hist, stride=64, n=n,
                             workspace=work)
        torch.cuda.synchronize()
        f = flow.cpu().numpy().view(np.uint32)
        want = np.bincount(f[f != 0xFFFFFFFF], minlength=1 << 16)
        assert (hist.cpu().numpy().view(np.uint32) == want).all()
        # one flow for every packet: a single bin counts them all without wrapping
        h1 = torch.zeros(1, dtype=torch.int32, device="cuda")
        ctx.flow_hist(arena, None, None, Chain.UdpParser, hist=h1, stride=64, n=n,
                      workspace=ctx.flow_hist_workspace(n, 1))
        torch.cuda.synchronize()
        assert int(h1.cpu()[0]) == int((f != 0xFFFFFFFF).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("win", [0, 1056])
@pytest.mark.parametrize("bins", [1, 2, 4096, 1 << 16])
def test_flow_bins_extreme_bin_counts(win, bins):
    """The table-free default kernel (win 0) and k_parse's flows mode (an
    explicit window) at the bin-mask extremes (one bin, two bins, the 16-bit
    maximum): flow ids and histogram equal the oracle's."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile
    from ingot_amd.abi import TUNE_WINDOW_INDEXED

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = 4097
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_WINDOW_INDEXED, win)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=bins + win)
    hist = torch.zeros(bins, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, bins=bins, n=n,
                         workspace=ctx.flow_hist_workspace(n, bins))
    torch.cuda.synchronize()
    w_hist, _ = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                                 Chain.VlanUlp, n=n, bins=bins)
    assert (flow.cpu().numpy().view(np.uint32) == oracle.flow_hist.last_flows).all()
    assert (hist.cpu().numpy().view(np.uint32) == w_hist).all()


@pytest.mark.gpu
@pytest.mark.parametrize("tune", [{}, {"win": 1056}, {"table": 32}, {"blocks": 3}])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097, 262_145])
def test_flow_ids_ragged_batches(n, tune):
    """Ragged batch sizes on every flows grid (k_flows_bits one tile per
    wave, k_parse's flows mode with the 16-bit table, the 32-bit table's
    persistent grid, a grid cap): flow ids equal the oracle's."""
    import torch

    import ingot_amd
    from ingot_amd import GenProfile
    from ingot_amd.abi import TUNE_FLOW_TABLE, TUNE_MAX_BLOCKS, TUNE_WINDOW_INDEXED

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_WINDOW_INDEXED, tune.get("win", 0))
    ctx.set_tuning(TUNE_FLOW_TABLE, tune.get("table", 0))
    ctx.set_tuning(TUNE_MAX_BLOCKS, tune.get("blocks", 0))
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=n + 7)
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, n=n)
    torch.cuda.synchronize()
    oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(), Chain.VlanUlp,
                     n=n)
    assert (flow.cpu().numpy().view(np.uint32) == oracle.flow_hist.last_flows).all()
