"""The double-buffered ring kernel (INGOT_TUNE_PIPELINE; on by default for
slot rings without a length array) returns exactly the oracle's records, for
every tiles-per-wave setting, the auto grid (0) and the one-tile kernel (1)."""
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile
from ingot_amd.abi import TUNE_PIPELINE

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tpw", [0, 1, 2, 3, 8, 16])
@pytest.mark.parametrize("n", [1, 63, 65, 100_003, 1 << 20])
def test_pipelined_ring_bit_exact(tpw, n):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    ctx.set_tuning(TUNE_PIPELINE, tpw)
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
