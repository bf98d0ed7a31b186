"""The multi-tile ring kernel (INGOT_TUNE_PIPELINE; on by default for slot
rings without a length array) returns exactly the oracle's records, for every
tiles-per-wave setting, the auto grid (0) and the one-tile kernel (1), every
pipeline depth (INGOT_TUNE_PIPE_DEPTH) and cache policy
(INGOT_TUNE_CACHE_POLICY)."""
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd.abi import TUNE_CACHE_POLICY, TUNE_PIPE_DEPTH, TUNE_PIPELINE

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tpw,depth,pol", [(0, 0, 0), (1, 0, 0), (2, 0, 0), (3, 0, 0),
                                           (8, 0, 0), (16, 0, 0), (0, 3, 0), (2, 3, 1),
                                           (5, 3, 2), (0, 4, 3), (3, 4, 0), (1, 0, 3),
                                           (0, 0, 4), (1, 0, 4), (0, 0, 11), (0, 0, 19),
                                           (0, 0, 27), (0, 0, 35), (0, 0, 43), (1, 0, 26), (0, 0, 75),
                                           (0, 0, 267), (1, 0, 386)])
@pytest.mark.parametrize("n", [1, 63, 65, 100_003, 1 << 20])
def test_pipelined_ring_bit_exact(tpw, depth, pol, n):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_PIPELINE, tpw)
    ctx.set_tuning(TUNE_PIPE_DEPTH, depth)
    ctx.set_tuning(TUNE_CACHE_POLICY, pol)
    for prof, stride in ((GenProfile.V4UDP64, 64), (GenProfile.ADVERSARIAL, 64),
                         (GenProfile.MIXED, 128)):
        arena, _, _ = ingot_amd.gen_frames(prof, n, seed=n + tpw, stride=stride)
        for chain in (Chain.UdpParser, Chain.GenericUlp, Chain.VlanUlp):
            got = ctx.parse_strided(arena, stride, n, chain)
            got8 = ctx.parse_strided_compact(arena, stride, n, chain)
            torch.cuda.synchronize()
            want = oracle.parse_batch(arena.cpu().numpy(), None, None, chain, stride=stride, n=n,
                                      nthreads=8)
            assert got.cpu().numpy().tobytes() == want.tobytes(), (prof, chain)
            assert got8.cpu().numpy().tobytes() == ingot_amd.rec16_to_rec8(want).tobytes()


@pytest.mark.parametrize("tpw", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("n", [1, 63, 65, 100_003])
def test_prefetching_indexed_kernel_bit_exact(tpw, n):
    """INGOT_TUNE_PIPELINE >= 2 on frames addressed by offset (16-B records):
    several tiles per wave with the next tile's descriptors loaded a tile
    ahead (k_parse<..., PF>).  Records equal the oracle's on adversarial and
    mixed / VLAN-EH frames, every non-tunnel chain, ragged sizes."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_PIPELINE, tpw)
    for prof in (GenProfile.ADVERSARIAL, GenProfile.MIXED, GenProfile.VLAN_V6EH):
        arena, off, lens = ingot_amd.gen_frames(prof, n, seed=n + 3 * tpw)
        a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
        for chain in (Chain.UdpParser, Chain.GenericUlp, Chain.VlanUlp):
            got = ctx.parse(arena, off, lens, chain)
            torch.cuda.synchronize()
            want = oracle.parse_batch(a, o, ln, chain, nthreads=8)
            assert got.cpu().numpy().tobytes() == want.tobytes(), (prof, chain)


@pytest.mark.parametrize("remap", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("tpw", [0, 3])
@pytest.mark.parametrize("n", [65, 100_003, 1 << 20])
def test_xcd_remapped_ring_bit_exact(remap, tpw, n):
    """INGOT_TUNE_XCD_REMAP = 1: the slot-ring kernel's blocks renumbered
    XCD-major cover every tile exactly once — records equal the oracle's."""
    import torch

    from ingot_amd.abi import TUNE_XCD_REMAP

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_XCD_REMAP, remap)
    ctx.set_tuning(TUNE_PIPELINE, tpw)
    for prof in (GenProfile.V4UDP64, GenProfile.ADVERSARIAL):
        arena, _, _ = ingot_amd.gen_frames(prof, n, seed=n + 5, stride=64)
        for chain in (Chain.UdpParser, Chain.VlanUlp):
            got = ctx.parse_strided(arena, 64, n, chain)
            torch.cuda.synchronize()
            want = oracle.parse_batch(arena.cpu().numpy(), None, None, chain, stride=64, n=n,
                                      nthreads=8)
            assert got.cpu().numpy().tobytes() == want.tobytes(), (prof, chain)
