#!/usr/bin/env python3
"""Measurement tool: does the record buffers' footprint change the C2 rate?
The 16 MiB of records per 1 M-frame batch are written with device-scope
stores; whether they reach HBM inside the region depends on whether the
buffers the run rotates through fit the 256 MiB Infinity Cache.  Times the
driver's C2 schedule (two staggered streams of per-batch launches,
doorbell-gated, 20-step regions after a 5-step warm-up, 8 arena copies) with
R = 2, 8, 16, 32, 64 record buffers rotated, and the persistent ring
consumer (one launch of 20 batches) with 8, 20 and 64 buffers; plus
2,000-step regions of the launches at R = 8 and 64.

    python tools/record_footprint.py [--reps 5]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "record_footprint.json"))
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, abi

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    n = 1 << 20
    a0, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    arenas = [a0] + [a0.clone() for _ in range(7)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(64)]
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    gate = bench.Gate(ingot_amd, ctx, 6.0)
    gate0 = bench.Gate(ingot_amd, ctx, 0.0)

    class Rot(bench.Runner):
        """bench.Runner with arenas rotated over 8 and records over R."""

        def __init__(self, R):
            super().__init__(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, None, None, outs,
                             streams, 16)
            h, c = ctx._h, int(Chain.UdpParser)
            ap_ = [a.data_ptr() for a in arenas]
            op_ = [o.data_ptr() for o in outs[:R]]
            sp_ = [s.cuda_stream for s in streams]
            self.launch = lambda k: lib.ingot_gpu_parse_strided(h, ap_[k % 8], 64, None, n, c,
                                                                 op_[k % R], sp_[k % 2])

    runners = {f"launches_R{R}": (Rot(R), gate) for R in (2, 8, 16, 32, 64)}
    for R in (8, 20, 64):
        runners[f"ring_R{R}"] = (bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas,
                                                  outs[:R], streams[:1], 16, 20), gate0)
    # the ring consumer at its best-known shape with the small record ring:
    # 3 / 4 blocks per CU (INGOT_TUNE_RING_GRID), 8 buffers
    grids = {}
    for gsz in (3, 4):
        runners[f"ring_R8_grid{gsz}"] = (bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n,
                                                          64, arenas, outs[:8], streams[:1], 16,
                                                          20), gate0)
        grids[f"ring_R8_grid{gsz}"] = gsz
    res = {k: [] for k in runners}
    for r in range(args.reps):
        for name, (rr, g) in runners.items():
            ctx.set_tuning(abi.TUNE_RING_GRID, grids.get(name, 0))
            if isinstance(rr, bench.RingRunner):
                rr.warm(5, g)
            else:
                rr.run(5, g)
            torch.cuda.synchronize()
            ms, _ = rr.run(20, g)
            res[name].append(ms * 1e3 / 20)
        print(f"rep {r}: " + " ".join(f"{k}={v[-1]:.3f}" for k, v in res.items()), flush=True)
    ctx.set_tuning(abi.TUNE_RING_GRID, 0)
    steady = {}
    for name in ("launches_R8", "launches_R64"):
        rr, g = runners[name]
        rr.run(100, g)
        ms, _ = rr.run(2000, g)
        steady[name] = round(ms * 1e3 / 2000, 3)
    out = {"us_per_step_20": {k: round(statistics.median(v), 3) for k, v in res.items()},
           "steady_2000": steady, "raw": res}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps({k: v for k, v in out.items() if k != "raw"}, indent=1))


if __name__ == "__main__":
    main()
