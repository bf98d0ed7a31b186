#!/usr/bin/env python3
"""Measurement tool: interleaved A/B of the C2 timed region exactly as the
driver's default `bench.py` times it (K doorbell-gated steps after W warm-up
steps, 8 rotated arenas, per-batch launches of k_parse_pipe) over the launch
schedule's free parameters: streams, the stagger between them, tiles per wave
(INGOT_TUNE_PIPELINE) and the cache policy.

    python tools/c2_region_ab.py [--steps 20] [--warmup 5] [--reps 9] [--variants a,b]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

# name -> (streams, stagger us, tiles per wave (0 = default grid), policy (0 = default)[, xcd remap])
VARIANTS = {
    "s2_st6": (2, 6.0, 0, 0),
    "s2_hw": (2, 6.0, 0, 0, 4),
    "s2_regions": (2, 6.0, 0, 0, 5),
    "s1_regions": (1, 0.0, 0, 0, 5),
    "s1_hw": (1, 0.0, 0, 0, 4),
    "s2_st3": (2, 3.0, 0, 0),
    "s2_st4.5": (2, 4.5, 0, 0),
    "s2_st7.5": (2, 7.5, 0, 0),
    "s2_st9": (2, 9.0, 0, 0),
    "s2_st0": (2, 0.0, 0, 0),
    "s3_st4": (3, 4.0, 0, 0),
    "s3_st2": (3, 2.0, 0, 0),
    "s2_tpw6": (2, 6.0, 6, 0),
    "s2_tpw10": (2, 6.0, 10, 0),
    "s2_tpw12": (2, 6.0, 12, 0),
    "s2_tpw16": (2, 6.0, 16, 0),
    "s2_pol27": (2, 6.0, 0, 27),
    "s2_pol3": (2, 6.0, 0, 3),
    "s1": (1, 0.0, 0, 0),
    "s2_xcd": (2, 6.0, 0, 0, 1),
    "s1_xcd": (1, 0.0, 0, 0, 1),
    "s2_run": (2, 6.0, 0, 0, 2),
    "s2_xcd_run": (2, 6.0, 0, 0, 3),
    "s1_run": (1, 0.0, 0, 0, 2),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--variants", default="")
    ap.add_argument("--steady", type=int, default=0, help="also time one N-step region each")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "c2_region_ab.json"))
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, abi

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    n, stride, reps = 1 << 20, 64, 8
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=stride)
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(reps)]
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    variants = dict(VARIANTS)
    if args.variants:
        variants = {k: VARIANTS[k] for k in args.variants.split(",")}
    gates = {st: bench.Gate(ingot_amd, ctx, st) for st in {v[1] for v in variants.values()}}
    runners = {k: bench.Runner(torch, lib, ctx, Chain.UdpParser, n, stride, arenas, None, None,
                               outs, streams[:v[0]], 16) for k, v in variants.items()}

    def knobs(v):
        ctx.set_tuning(abi.TUNE_PIPELINE, v[2])
        ctx.set_tuning(abi.TUNE_CACHE_POLICY, v[3])
        ctx.set_tuning(abi.TUNE_XCD_REMAP, v[4] if len(v) > 4 else 0)

    res = {k: [] for k in variants}
    for r in range(args.reps):
        for name, v in variants.items():
            knobs(v)
            rr, g = runners[name], gates[v[1]]
            rr.run(args.warmup, g)
            torch.cuda.synchronize()
            ms, _ = rr.run(args.steps, g)
            res[name].append(ms * 1e3 / args.steps)
        print(f"rep {r}: " + " ".join(f"{k}={v[-1]:.3f}" for k, v in res.items()), flush=True)
    steady = {}
    if args.steady:
        for name, v in variants.items():
            knobs(v)
            runners[name].run(100, gates[v[1]])
            ms, _ = runners[name].run(args.steady, gates[v[1]])
            steady[name] = round(ms * 1e3 / args.steady, 3)
    knobs((0, 0, 0, 0))
    rd = 64 * n
    summary = {k: {"median_us_per_step": round(statistics.median(v), 3),
                   "min": round(min(v), 3), "max": round(max(v), 3),
                   "Gpkt_s": round(n / statistics.median(v) / 1e3, 2),
                   "read_frac": round(rd / (statistics.median(v) * 1e-6) / 8e12, 4)}
               for k, v in res.items()}
    out = {"steps": args.steps, "warmup": args.warmup, "reps": args.reps,
           "variants": {k: dict(zip(("streams", "stagger_us", "tiles_per_wave", "policy", "xcd"), v))
                        for k, v in variants.items()},
           "summary": summary, "steady_us_per_step": steady, "raw": res}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    for k, v in summary.items():
        print(k, v, steady.get(k, ""))


if __name__ == "__main__":
    main()
