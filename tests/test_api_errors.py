"""The C ABI's error behaviour with a live context (include/ingot_gpu.h):
bad arguments are negative API codes before any launch, empty batches
succeed without touching pointers, malformed packets are never API errors.
Needs an MI355X: `pytest -m gpu`."""
import ctypes

import numpy as np
import pytest

import ingot_amd
from ingot_amd import Chain, GenProfile, _lib
from ingot_amd.abi import (TUNE_FLOW_KERNEL, TUNE_PIPE_DEPTH, TUNE_READ_PLAN, TUNE_SLOW_PATH,
                           TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED)

pytestmark = pytest.mark.gpu

EINVAL, ERANGE = -1, -5


@pytest.fixture(scope="module")
def env():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = ingot_amd.Context(0)
    arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, 1000, seed=3)
    out = torch.empty((1000, 256), dtype=torch.uint8, device="cuda")
    return torch, ctx, _lib.load(), arena, off, lens, out


def test_parse_argument_errors(env):
    torch, ctx, lib, arena, off, lens, out = env
    h, a, o, ln, r = ctx._h, arena.data_ptr(), off.data_ptr(), lens.data_ptr(), out.data_ptr()
    assert lib.ingot_gpu_parse(h, a, o, ln, 1000, 7, r, None) == EINVAL  # no such chain
    assert lib.ingot_gpu_parse(h, a, o, ln, 1000, -1, r, None) == EINVAL
    assert lib.ingot_gpu_parse(h, a, o, ln, 1000, 0, None, None) == EINVAL  # no output
    assert lib.ingot_gpu_parse(h, a, None, ln, 1000, 0, r, None) == EINVAL  # no offsets
    assert lib.ingot_gpu_parse(h, None, None, None, 0, 0, None, None) == 0  # empty batch
    # slot rings: stride a multiple of 16 in (0, 65535], arena 16-B aligned
    for stride in (0, 8, 24, 65536):
        assert lib.ingot_gpu_parse_strided(h, a, stride, None, 10, 0, r, None) == ERANGE, stride
    assert lib.ingot_gpu_parse_strided(h, a + 4, 64, None, 10, 0, r, None) == EINVAL
    # 8-B records are not offered for the tunnel; its field blocks are 384 B
    assert lib.ingot_gpu_parse_compact(h, a, o, ln, 10, int(Chain.GeneveOverV6Tunnel), r,
                                       None) == EINVAL
    assert lib.ingot_gpu_fields(h, a, o, ln, 0, 10, int(Chain.GeneveOverV6Tunnel), r,
                                None) == EINVAL
    torch.cuda.synchronize()


def test_parse_read_dense_argument_errors(env):
    torch, ctx, lib, arena, off, lens, out = env
    h, a, o, r = ctx._h, arena.data_ptr(), off.data_ptr(), out.data_ptr()
    ps = torch.arange(11, dtype=torch.int32, device="cuda")
    p = ps.data_ptr()
    TUN = int(Chain.GeneveOverV6Tunnel)
    assert lib.ingot_gpu_parse_read_dense(h, a, o, p, 10, TUN, 1, r, None, None) == EINVAL
    assert lib.ingot_gpu_parse_read_dense(h, a, o, p, 10, 1, 2, r, None, None) == EINVAL
    assert lib.ingot_gpu_parse_read_dense(h, a, o, p, 10, 1, 3, r, None, None) == EINVAL
    assert lib.ingot_gpu_parse_read_dense(h, a, None, p, 10, 1, 0, r, None, None) == EINVAL
    assert lib.ingot_gpu_parse_read_dense(h, None, None, None, 0, 1, 0, None, None, None) == 0
    torch.cuda.synchronize()


def test_modify_and_flow_argument_errors(env):
    torch, ctx, lib, arena, off, lens, out = env
    h, a, o, ln = ctx._h, arena.data_ptr(), off.data_ptr(), lens.data_ptr()
    from ingot_amd import EditOp, Field, edits_array

    ok = edits_array([(2, Field.UDP_DESTINATION, EditOp.SUB, 1)])
    many = edits_array([(2, Field.UDP_DESTINATION, EditOp.SUB, 1)] * 17)  # > INGOT_MAX_EDITS
    bad_layer = edits_array([(3, Field.UDP_DESTINATION, EditOp.SUB, 1)])  # UdpParser: 3 layers
    p = lambda e: e.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert lib.ingot_gpu_parse_modify(h, a, o, ln, 0, 10, 0, p(many), 17, None, None) == EINVAL
    assert lib.ingot_gpu_parse_modify(h, a, o, ln, 0, 10, 0, p(bad_layer), 1, None,
                                      None) == EINVAL
    assert lib.ingot_gpu_parse_modify(h, a, o, ln, 0, 10, 0, None, 1, None, None) == EINVAL
    raw = ok.copy()
    raw.view(np.uint8)[1] = 200  # no such field
    assert lib.ingot_gpu_parse_modify(h, a, o, ln, 0, 10, 0, p(raw), 1, None, None) == EINVAL
    flow = torch.empty(1000, dtype=torch.int32, device="cuda")
    hist = torch.zeros(1000, dtype=torch.int32, device="cuda")
    for bins in (0, 3, 1000, 1 << 25):  # a power of two <= 2^24
        assert lib.ingot_gpu_flow_hist(h, a, o, ln, 0, 10, 2, None, bins, flow.data_ptr(),
                                       None, hist.data_ptr(), None) == ERANGE, bins
    assert lib.ingot_gpu_flow_hist(h, a, o, ln, 0, 10, 2, None, 64, None, None,
                                   hist.data_ptr(), None) == EINVAL
    torch.cuda.synchronize()


def test_tuning_errors_and_defaults(env):
    torch, ctx, lib, *_ = env
    c = ingot_amd.Context(0)
    # the variants that lost were removed: their values are EINVAL
    pruned = [(TUNE_SLOW_PATH, v) for v in (1, 2)] + \
        [(TUNE_READ_PLAN, v) for v in (2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 13, 14, 15, 16, 18)] + \
        [(TUNE_FLOW_KERNEL, v) for v in range(1, 15)] + [(TUNE_FLOW_KERNEL, 16)]
    for key, val in [(TUNE_WINDOW_INDEXED, 7), (TUNE_WINDOW_STRIDED, 6), (TUNE_PIPE_DEPTH, 1),
                     (99, 0)] + pruned:
        assert lib.ingot_gpu_ctx_set_tuning(c._h, key, val) == EINVAL, (key, val)
    assert c.get_tuning(TUNE_WINDOW_INDEXED) == 0  # untouched by the rejected calls
    c.set_tuning(TUNE_WINDOW_INDEXED, 5)
    assert c.get_tuning(TUNE_WINDOW_INDEXED) == 5
    c.set_tuning(TUNE_WINDOW_INDEXED, 0)  # back to the measured default


def test_malformed_packets_are_never_api_errors(env):
    """Garbage bytes, zero-length and truncated frames: the call succeeds and
    every record carries the packet's ParseError (error.rs:21-44)."""
    torch, ctx, lib, *_ = env
    rng = np.random.default_rng(9)
    n = 5000
    lens_np = rng.integers(0, 200, n).astype(np.uint16)
    off_np = np.concatenate([[0], np.cumsum(lens_np[:-1].astype(np.int64))])
    arena = torch.from_numpy(rng.integers(0, 256, int(lens_np.sum()) + 64, dtype=np.uint8)).cuda()
    off = torch.from_numpy(off_np).cuda()
    lens = torch.from_numpy(lens_np).cuda()
    for chain in Chain:
        recs = ctx.parse(arena, off, lens, chain)
        torch.cuda.synchronize()
        st = recs[:, 0].cpu().numpy()
        assert ((st >= 0) & (st <= 8)).all()
        assert (st[lens_np < 14] == 3).all()  # TooSmall at the first layer
