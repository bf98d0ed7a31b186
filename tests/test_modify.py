"""In-place header rewrite: ingot_gpu_parse_modify against the
oracle's setter restatement, pinned by tests/golden modify/setter vectors
(parse-and-decr-v4, bitset neighbours, unaligned bitfield setters)."""
import numpy as np
import pytest

import ingot_amd
import oracle
from ingot_amd import Chain, EditOp, Field, GenProfile

pytestmark = pytest.mark.gpu
TUN = Chain.GeneveOverV6Tunnel

EDITS = {
    Chain.UdpParser: [(2, Field.UDP_DESTINATION, EditOp.SUB, 1),
                      (1, Field.V4_HOP_LIMIT, EditOp.SUB, 1),
                      (1, Field.V6_HOP_LIMIT, EditOp.SUB, 1),
                      (1, Field.V4_DSCP, EditOp.XOR, 0x2A),
                      (1, Field.V6_FLOW_LABEL, EditOp.ADD, 0xFFFFF),
                      (0, Field.ETH_ETHERTYPE, EditOp.OR, 0)],
    Chain.GenericUlp: [(2, Field.TCP_FLAGS, EditOp.AND, 0xEF), (2, Field.TCP_DATA_OFFSET,
                                                                  EditOp.SET, 5),
                       (2, Field.ICMP_CODE, EditOp.ADD, 3), (1, Field.V4_FLAGS, EditOp.SET, 2),
                       (1, Field.V4_FRAGMENT_OFFSET, EditOp.ADD, 4097),
                       (2, Field.UDP_CHECKSUM, EditOp.SET, 0)],
    Chain.VlanUlp: [(1, Field.VLAN_VID, EditOp.ADD, 1, 0), (1, Field.VLAN_PRIORITY, EditOp.SET,
                                                             7, 1),
                    (1, Field.VLAN_DEI, EditOp.XOR, 1, 0), (3, Field.TCP_SEQUENCE, EditOp.ADD,
                                                             0x80000001),
                    (2, Field.V6_ECN, EditOp.SET, 3)],
    TUN: [(3, Field.GENEVE_VNI, EditOp.SET, 0xABCDEF), (3, Field.GENEVE_FLAGS, EditOp.OR, 0x80),
          (1, Field.V6_HOP_LIMIT, EditOp.SUB, 1), (2, Field.UDP_SOURCE, EditOp.XOR, 0xFFFF),
          (4, Field.ETH_ETHERTYPE, EditOp.SET, 0x0800), (5, Field.V4_HOP_LIMIT, EditOp.SUB, 1),
          (6, Field.TCP_WINDOW_SIZE, EditOp.SUB, 100)],
}


@pytest.fixture(scope="module")
def torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def ctx(torch):
    return ingot_amd.Context(0)


def test_modify_kats_on_device(ctx, torch, kats):
    for kat in kats["modify_kats"]:
        chain = Chain[kat["chain"]]
        f = bytes.fromhex(kat["frame"])
        edits = [(e[0], Field[e[1]], EditOp[e[2]], e[3], *e[4:]) for e in kat["edits"]]
        buf = torch.zeros(((len(f) + 15) // 16 + 4) * 16, dtype=torch.uint8)
        buf[:len(f)] = torch.frombuffer(bytearray(f), dtype=torch.uint8)
        arena = buf.cuda()
        off = torch.zeros(1, dtype=torch.int64, device="cuda")
        lens = torch.tensor([len(f)], dtype=torch.int32, device="cuda").to(torch.uint16)
        ctx.parse_modify(arena, off, lens, chain, edits)
        torch.cuda.synchronize()
        assert arena[:len(f)].cpu().numpy().tobytes().hex() == kat["after"], kat["name"]


@pytest.mark.parametrize("chain", list(Chain))
def test_modify_fuzz_bit_exact(ctx, torch, chain):
    prof = {Chain.UdpParser: GenProfile.MIXED, Chain.GenericUlp: GenProfile.ADVERSARIAL,
            Chain.VlanUlp: GenProfile.VLAN_V6EH, TUN: GenProfile.GENEVE}[chain]
    for p, seed in ((prof, 81), (GenProfile.GENEVE_ADVERSARIAL if chain == TUN
                                 else GenProfile.ADVERSARIAL, 82)):
        arena, off, lens = ingot_amd.gen_frames(p, 100_000, seed=seed)
        before = arena.cpu().numpy()
        recs = torch.empty((100_000, 16), dtype=torch.uint8, device="cuda")
        ctx.parse_modify(arena, off, lens, chain, EDITS[chain], out=recs)
        torch.cuda.synchronize()
        want = before.copy()
        w_rec = oracle.parse_modify_batch(want, off.cpu().numpy(), lens.cpu().numpy(), chain,
                                          EDITS[chain])
        got = arena.cpu().numpy()
        assert recs.cpu().numpy().tobytes() == w_rec.tobytes()
        diff = np.nonzero(got != want)[0]
        assert diff.size == 0, (diff[:10], got[diff[:10]], want[diff[:10]])
        assert (got != before).any()  # the edits did something


def test_modify_strided_decr(ctx, torch):
    """The C2 batch as parse-and-decr-v4: every UDP destination - 1."""
    n = 1 << 20
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    before = arena[:n * 64].view(n, 64)[:, 36:38].cpu().numpy().copy()
    ctx.parse_modify(arena, None, None, Chain.UdpParser,
                     [(2, Field.UDP_DESTINATION, EditOp.SUB, 1)], stride=64, n=n)
    torch.cuda.synchronize()
    after = arena[:n * 64].view(n, 64).cpu().numpy()
    b = before[:, 0].astype(np.int32) << 8 | before[:, 1]
    a = after[:, 36].astype(np.int32) << 8 | after[:, 37]
    assert ((b - 1) & 0xFFFF == a).all()
    rest = np.delete(after, [36, 37], axis=1)
    assert rest.tobytes() == np.delete(
        ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)[0][:n * 64].view(n, 64).cpu()
        .numpy(),
        [36, 37], axis=1).tobytes()


@pytest.mark.parametrize("tune", [dict(), dict(wb=16), dict(wb=64), dict(depth=3, wb=64),
                                  dict(pipe=3, pol=1), dict(pipe=1), dict(pipe=16, pol=3)])
@pytest.mark.parametrize("n", [1, 65, 100_003])
def test_modify_ring_bit_exact(ctx, torch, tune, n):
    """The slot-ring rewrite kernel (k_modify_pipe: staged edits, lane-linear
    write-back) for every write-back unit, depth, grid and cache policy, on
    64-B and 128-B slots (edits past the 64-B window go straight to HBM)."""
    from ingot_amd.abi import (TUNE_CACHE_POLICY, TUNE_PIPE_DEPTH, TUNE_PIPELINE,
                               TUNE_WRITEBACK)

    c = ingot_amd.Context(0)
    c.set_tuning(TUNE_WRITEBACK, tune.get("wb", 0))
    c.set_tuning(TUNE_PIPE_DEPTH, tune.get("depth", 0))
    c.set_tuning(TUNE_PIPELINE, tune.get("pipe", 0))
    c.set_tuning(TUNE_CACHE_POLICY, tune.get("pol", 0))
    for prof, stride in ((GenProfile.V4UDP64, 64), (GenProfile.ADVERSARIAL, 64),
                         (GenProfile.MIXED, 128), (GenProfile.VLAN_V6EH, 128)):
        for chain in (Chain.UdpParser, Chain.GenericUlp, Chain.VlanUlp):
            arena, _, _ = ingot_amd.gen_frames(prof, n, seed=n + stride, stride=stride)
            want = arena.cpu().numpy().copy()
            recs = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
            c.parse_modify(arena, None, None, chain, EDITS[chain], stride=stride, n=n, out=recs)
            torch.cuda.synchronize()
            w_rec = oracle.parse_modify_batch(want, None, None, chain, EDITS[chain],
                                              stride=stride, n=n, nthreads=8)
            assert recs.cpu().numpy().tobytes() == w_rec.tobytes(), (prof, chain)
            got = arena.cpu().numpy()
            diff = np.nonzero(got != want)[0]
            assert diff.size == 0, (prof, chain, diff[:10], got[diff[:10]], want[diff[:10]])
