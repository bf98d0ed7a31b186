#!/usr/bin/env python3
"""Measurement tool: the single-batch ring kernel (k_parse_pipe, one stream)
over batches of 1..20 M C2 frames in ONE arena — tiles per wave grow with the
batch while the code stays the same — against the persistent ring consumer
over the same frames as 1 M-frame batches.  Separates "long-lived waves are
slower" from "the ring kernel's code is slower".

    python tools/pipe_len.py
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    m = 1 << 20
    N = 20 * m
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, N, stride=64)
    out = torch.empty((N, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    for k in (1, 2, 5, 10, 20):
        n = k * m
        # consecutive launches read consecutive k-M windows of the 1.28 GB
        # arena (never the same bytes twice in 20 launches: no cache reuse)
        wins = [arena[i * n * 64:(i + 1) * n * 64] for i in range(20 // k)]
        wouts = [out[i * n:(i + 1) * n] for i in range(20 // k)]
        r = bench.Runner(torch, lib, ctx, Chain.UdpParser, n, 64, wins, None, None, wouts, [s],
                         16)
        r.run(5)
        ms, _ = r.run(20)
        res[f"pipe_{k}M"] = round(ms * 1e3 / 20 / k, 3)  # us per 1 M frames
    # the ring over the same frames as 1 M batches (views into the one arena)
    views = [arena[b * m * 64:(b + 1) * m * 64] for b in range(20)]
    outs = [out[b * m:(b + 1) * m] for b in range(20)]
    # the 20 M launch under other cache policies and record widths
    from ingot_amd.abi import TUNE_CACHE_POLICY
    r = bench.Runner(torch, lib, ctx, Chain.UdpParser, N, 64, [arena], None, None, [out], [s], 16)
    for pol in (3, 4, 11, 19, 27, 1, 75):
        ctx.set_tuning(TUNE_CACHE_POLICY, pol)
        r.run(2)
        ms, _ = r.run(6)
        res[f"pipe_20M_pol{pol}"] = round(ms * 1e3 / 6 / 20, 3)
    ctx.set_tuning(TUNE_CACHE_POLICY, 0)
    out8 = torch.empty((N, 8), dtype=torch.uint8, device="cuda")
    r8 = bench.Runner(torch, lib, ctx, Chain.UdpParser, N, 64, [arena], None, None, [out8], [s], 8)
    r8.run(2)
    ms, _ = r8.run(6)
    res["pipe_20M_rec8"] = round(ms * 1e3 / 6 / 20, 3)
    for G in (1, 5, 20):
        rr = bench.RingRunner(torch, lib, ctx, Chain.UdpParser, m, 64, views, outs, [s], 16, G)
        rr.warm(20)
        ms, _ = rr.run(20 * 4)
        res[f"ring_G{G}"] = round(ms * 1e3 / 80, 3)
    print(json.dumps(res, indent=1))
    Path(ROOT / "gpurun_out" / "pipe_len.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
