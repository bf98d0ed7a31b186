"""Lengths-only packed frames (ingot_gpu_parse_packed): offsets derived on
the device by a scan of tile sums plus a wavefront prefix scan per tile.
Records equal ingot_gpu_parse's over the same frames with explicit offsets
(test_gpu_parity.py pins those to the oracle), and the derived offsets equal
the exclusive prefix sum of the lengths.  Needs an MI355X: `pytest -m gpu`."""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, GenProfile, _lib

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


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 100_003])
@pytest.mark.parametrize("profile,chain", [("ADVERSARIAL", Chain.GenericUlp),
                                           ("MIXED", Chain.UdpParser),
                                           ("VLAN_V6EH", Chain.VlanUlp),
                                           ("GENEVE_ADVERSARIAL", Chain.GeneveOverV6Tunnel)])
def test_packed_equals_indexed(torch, ctx, n, profile, chain):
    arena, off, lens = ingot_amd.gen_frames(GenProfile[profile], n, seed=n)
    # gen_frames packs back to back: off is the exclusive prefix sum of lens
    assert torch.equal(off[1:], off[:-1] + lens[:-1].to(torch.int64))
    want = ctx.parse(arena, off, lens, chain)
    off_out = torch.full((n,), -1, dtype=torch.int64, device="cuda")
    got = ctx.parse_packed(arena, lens, chain, off_out=off_out)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert torch.equal(off_out, off)
    if n <= 1000:
        w = oracle.parse_batch(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(), chain)
        assert got.cpu().numpy().tobytes() == w.tobytes()


def test_packed_config3_full_size(torch, ctx):
    """16,777,216 mixed frames (~13 GB): 262,144 tiles through the scan."""
    n = 1 << 24
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp)
    off_out = torch.empty(n, dtype=torch.int64, device="cuda")
    got = ctx.parse_packed(arena, lens, Chain.GenericUlp, off_out=off_out)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert torch.equal(off_out, off)
    del arena, off, lens, want, got, off_out
    torch.cuda.empty_cache()


def test_packed_argument_errors(torch, ctx):
    lib = _lib.load()
    arena, _, lens = ingot_amd.gen_frames(GenProfile.MIXED, 1000, seed=2)
    out = torch.empty((1000, 16), dtype=torch.uint8, device="cuda")
    need = lib.ingot_gpu_packed_workspace_size(1000)
    assert need >= 16 * 4 + 8  # one u32 per tile + one u64 per group
    work = torch.empty(need + 16, dtype=torch.uint8, device="cuda")
    h, a, ln, o, w = ctx._h, arena.data_ptr(), lens.data_ptr(), out.data_ptr(), work.data_ptr()
    assert lib.ingot_gpu_parse_packed(h, a, ln, 1000, 1, o, None, w, need - 1, None) == -5
    assert lib.ingot_gpu_parse_packed(h, a, ln, 1000, 1, o, None, w + 4, need, None) == -1
    assert lib.ingot_gpu_parse_packed(h, a, ln, 1000, 9, o, None, w, need, None) == -1
    assert lib.ingot_gpu_parse_packed(h, a, None, 1000, 1, o, None, w, need, None) == -1
    assert lib.ingot_gpu_parse_packed(h, None, None, 0, 1, None, None, None, 0, None) == 0
    assert lib.ingot_gpu_parse_packed(h, a, ln, 1000, 1, o, None, w, need, None) == 0
    torch.cuda.synchronize()
