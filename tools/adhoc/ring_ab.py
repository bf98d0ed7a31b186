#!/usr/bin/env python3
"""Interleaved A/B of the C2 timed region as the driver runs it (K-step
regions after a W-step warm-up, doorbell-gated): the per-batch launches on
two staggered streams (round-2 headline) against the persistent ring
consumer (ingot_gpu_parse_ring) over its grid / depth / cache-policy knobs.

    python tools/ring_ab.py [--steps 20] [--warmup 5] [--reps 15] [--out F]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--variants", default="")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "ring_ab.json"))
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, abi

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    n, stride = 1 << 20, 64
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=stride)
    reps = 8
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(64)]
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    gate = bench.Gate(ingot_amd, ctx, 6.0)
    gate0 = bench.Gate(ingot_amd, ctx, 0.0)  # no stagger
    G = bench.ring_group(args.steps)

    knobs = {"grid": abi.TUNE_RING_GRID, "depth": abi.TUNE_PIPE_DEPTH,
             "pol": abi.TUNE_CACHE_POLICY, "groups": abi.TUNE_RING_GROUPS,
             "tpw": abi.TUNE_PIPELINE}
    variants = {
        "pipe2": None,
        "pipe1": None,
        "pipe2_half": None,
        "pipe2_d3": {"pipe": 2, "depth": 3},
        "pipe2_d4": {"pipe": 2, "depth": 4},
        "pipe2_g3": {"pipe": 2, "tpw": 6},
        "pipe2_pol19": {"pipe": 2, "pol": 19},
        "pipe2_pol27": {"pipe": 2, "pol": 27},
        "pipe2_nostagger": None,
        "ring_G1": {"G": 1},
        "ring2": {"S": 2},
        "ring2_g1": {"S": 2, "grid": 1},
        "ring2_q": {"S": 2, "G": 10},
        "ring_G1_o8": {"G": 1, "outs": 8},
        "ring_o8": {"outs": 8},
        "pipe1_o64": None,
        "ring": {},
        "ring_g1": {"grid": 1},
        "ring_g3": {"grid": 3},
        "ring_q2": {"groups": 2},
        "ring_g4_q2": {"grid": 4, "groups": 2},
        "ring_g4_q4": {"grid": 4, "groups": 4},
        "ring_g3_q2": {"grid": 3, "groups": 2},
        "ring_g4": {"grid": 4},
        "ring_d3": {"depth": 3},
        "ring_d4": {"depth": 4},
        "ring_g4_d3": {"grid": 4, "depth": 3},
        "ring_nt": {"pol": 3},
        "ring_plain": {"pol": 4},
    }
    if args.variants:
        keep = args.variants.split(",")
        variants = {k: v for k, v in variants.items() if k in keep}

    def set_knobs(kv):
        kv = {k: v for k, v in (kv or {}).items() if k in knobs}
        for k, key in knobs.items():
            ctx.set_tuning(key, (kv or {}).get(k, 0))

    def runner(name):
        if name == "pipe2_half":
            return bench.HalfOffsetRunner(torch, lib, ctx, Chain.UdpParser, n, stride, arenas,
                                          outs[:reps], streams[:2], 16)
        if variants[name] is None or "pipe" in variants[name]:
            ns = 1 if name.startswith("pipe1") else 2
            o = outs if name.endswith("_o64") else outs[:reps]
            a = arenas * (len(o) // reps)  # same arena rotation, one record buffer per step
            return bench.Runner(torch, lib, ctx, Chain.UdpParser, n, stride, a, None, None,
                                o, streams[:ns], 16)
        kv = variants[name]
        return bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n, stride, arenas,
                                outs[:kv.get("outs", 64)], streams[:kv.get("S", 1)], 16,
                                kv.get("G", G))

    runners = {k: runner(k) for k in variants}
    res = {k: [] for k in variants}
    for r in range(args.reps):
        for name, kv in variants.items():
            set_knobs(kv)
            rr = runners[name]
            gt = gate0 if name in ("pipe2_half", "pipe2_nostagger") else gate
            if isinstance(rr, bench.RingRunner):
                rr.warm(args.warmup, gt)
            else:
                rr.run(args.warmup, gt)
            torch.cuda.synchronize()
            ms, _ = rr.run(args.steps, gt)
            res[name].append(ms * 1e3 / args.steps)
        print(f"rep {r}: " + " ".join(f"{k}={v[-1]:.3f}" for k, v in res.items()), flush=True)
    set_knobs(None)
    # steady state: 2,000-step regions
    steady = {}
    for name in ("pipe2", "pipe2_half", "ring", "ring2"):
        if name not in runners:
            continue
        rr = runners[name]
        if isinstance(rr, bench.RingRunner):
            rr = bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n, stride, arenas, outs,
                                  streams[:variants[name].get("S", 1)], 16,
                                  bench.ring_group(2000))
        gt = gate0 if name == "pipe2_half" else gate
        rr.run(200, gt)
        ms, _ = rr.run(2000, gt)
        steady[name] = ms * 1e3 / 2000
    rd = 64 * n
    summary = {k: {"median_us_per_step": round(statistics.median(v), 3),
                   "min": round(min(v), 3), "max": round(max(v), 3),
                   "Gpkt_s": round(n / statistics.median(v) / 1e3, 2),
                   "read_frac": round(rd / (statistics.median(v) * 1e-6) / 8e12, 4)}
               for k, v in res.items()}
    out = {"steps": args.steps, "warmup": args.warmup, "reps": args.reps, "group": G,
           "summary": summary, "steady_2000_us_per_step": steady, "raw": res}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(summary, indent=1))
    print("steady", steady)


if __name__ == "__main__":
    main()
