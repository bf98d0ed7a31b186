#!/usr/bin/env python3
"""Measurement tool: staggered stream starts (ingot_gpu_stream_delay) on a
gated multi-stream region, interleaved A/B in one process.

For each stagger value (us between consecutive streams' first launches), a
region of K steps is timed exactly as bench.py times it (doorbell-held start,
earliest start -> latest end on the device clock), after a W-step warm-up run
like the driver's (--steps 20 --warmup 5), rounds interleaved over the values.

    python tools/stagger_ab.py --config c2 --stagger 0 --stagger 4 --stagger 6 > out.json
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
    ap.add_argument("--config", default="c2")
    ap.add_argument("--stagger", type=float, action="append", default=[])
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--steps", type=int, action="append", default=[])
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--record", type=int, default=16)
    args = ap.parse_args()
    staggers = args.stagger or [0.0]
    ks = args.steps or [20]
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    prof, n, stride, chain_name, _ = bench.CONFIGS[args.config]
    chain = Chain[chain_name]
    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, stride=stride)
    R = max(4, -(-(512 << 20) // arena.numel()))
    arenas = [arena] + [arena.clone() for _ in range(R - 1)]
    outs = [torch.empty((n, args.record), dtype=torch.uint8, device="cuda") for _ in range(R)]
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    gates = {s: bench.Gate(ingot_amd, ctx, s) for s in staggers}
    run = bench.Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs, streams,
                       args.record)
    run.run(50, gates[staggers[0]])
    res = {(s, k): [] for s in staggers for k in ks}
    for _ in range(args.rounds):
        for k in ks:
            for s in staggers:
                g = gates[s]
                if args.warmup:
                    run.run(args.warmup, g)
                torch.cuda.synchronize()
                ms, _ = run.run(k, g)
                res[(s, k)].append(ms * 1e3 / k)
    out = {"config": args.config, "streams": args.streams, "record": args.record,
           "warmup": args.warmup, "rounds": args.rounds, "us_per_step": {}}
    for (s, k), v in res.items():
        med = statistics.median(v)
        out["us_per_step"][f"stagger={s:g},steps={k}"] = {
            "median": round(med, 3), "min": round(min(v), 3),
            "Gpkt_s_median": round(n / med / 1e3, 2), "all": [round(x, 2) for x in v]}
        print(f"{args.config} stagger={s:<5g} steps={k:<5d} median {med:8.3f} us/step "
              f"min {min(v):8.3f}  {n / med / 1e3:7.2f} Gpkt/s", file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
