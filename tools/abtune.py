#!/usr/bin/env python3
"""Measurement tool: interleaved A/B of tuning variants on one dataset, in one
process (cdna_hip_programming.md §5.4 rule 24: separate invocations add
cross-process/device variance that looks like a kernel property).

    python tools/abtune.py --config c3 --var win_i=4 --var win_i=5 --var win_i=9
    python tools/abtune.py --config c2 --var streams=1 --var streams=2 --var rec=8

A variant is a comma list of key=value: win_i, win_s, blocks, pipe, depth, pol,
wb, ftab, slow, plan, fk, streams, rec, fonly (1: the flows kernel alone, no
histogram), mode (parse|flows|modify: the runner; default the config's).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--var", action="append", default=[])
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch

    import bench
    import ingot_amd
    from ingot_amd import Chain, GenProfile
    from ingot_amd.abi import (TUNE_CACHE_POLICY, TUNE_MAX_BLOCKS, TUNE_PIPE_DEPTH,
                               TUNE_PIPELINE, TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED,
                               TUNE_WRITEBACK, TUNE_FLOW_TABLE, TUNE_SLOW_PATH,
                               TUNE_READ_PLAN, TUNE_FLOW_KERNEL)

    prof, n, stride, chain_name, _ = bench.CONFIGS[args.config]
    chain = Chain[chain_name]
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, stride=stride)
    reps = max(4, -(-(512 << 20) // arena.numel()))
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(reps)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    lib = ingot_amd.load_library()
    steps = args.steps or max(20, int(2e5 / max(1, n / 1e4)))
    segs = None
    if bench.MODES.get(args.config) == "read":
        c0 = ingot_amd.Context(0)
        recs0 = ingot_amd.records_to_numpy(
            c0.parse_strided(arena, stride, n, chain) if stride is not None else
            c0.parse(arena, off, lens, chain))
        rl = (lens if lens is not None else
              torch.full((n,), stride, dtype=torch.int32, device="cuda").to(torch.uint16))
        segs = bench.read_chunks(torch, off, stride, rl.to(torch.int32), recs0,
                                 bench.READ_CHUNKS[args.config], "cuda")[:3]
    variants = args.var or ["win_i=5"]
    runners = {}
    for v in variants:
        kv = dict(x.split("=") for x in v.split(",") if x)
        ctx = ingot_amd.Context(0)
        if "win_i" in kv:
            ctx.set_tuning(TUNE_WINDOW_INDEXED, int(kv["win_i"]))
        if "win_s" in kv:
            ctx.set_tuning(TUNE_WINDOW_STRIDED, int(kv["win_s"]))
        if "blocks" in kv:
            ctx.set_tuning(TUNE_MAX_BLOCKS, int(kv["blocks"]))
        if "pipe" in kv:
            ctx.set_tuning(TUNE_PIPELINE, int(kv["pipe"]))
        if "depth" in kv:
            ctx.set_tuning(TUNE_PIPE_DEPTH, int(kv["depth"]))
        if "pol" in kv:
            ctx.set_tuning(TUNE_CACHE_POLICY, int(kv["pol"]))
        if "wb" in kv:
            ctx.set_tuning(TUNE_WRITEBACK, int(kv["wb"]))
        if "ftab" in kv:
            ctx.set_tuning(TUNE_FLOW_TABLE, int(kv["ftab"]))
        if "slow" in kv:
            ctx.set_tuning(TUNE_SLOW_PATH, int(kv["slow"]))
        if "plan" in kv:
            ctx.set_tuning(TUNE_READ_PLAN, int(kv["plan"]))
        if "fk" in kv:
            ctx.set_tuning(TUNE_FLOW_KERNEL, int(kv["fk"]))
        ns, rb = int(kv.get("streams", 1)), int(kv.get("rec", 16))
        mode = kv.get("mode", bench.MODES.get(args.config, "parse"))
        if mode == "flows":
            hists = [torch.zeros(bench.FLOW_BINS, dtype=torch.int32, device="cuda")
                     for _ in range(reps)]
            fids = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(reps)]
            r = bench.FlowRunner(torch, lib, ctx, chain, n, arenas, off, lens, hists, fids,
                                 streams[:ns], lambda h: None,
                                 flows_only=kv.get("fonly") == "1")
        elif mode == "read":
            r = bench.ReadRunner(torch, lib, ctx, chain, n, arenas, *segs, outs, streams[:ns])
        elif mode == "packed":
            r = bench.PackedRunner(torch, lib, ctx, chain, n, arenas, lens, outs, streams[:ns])
        elif mode == "modify":
            r = bench.ModifyRunner(torch, lib, ctx, chain, n, stride, arenas, off, lens,
                                   streams[:ns])
        else:
            r = bench.Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs,
                             streams[:ns], rb)
        runners[v] = (ctx, r)
    res = {v: [] for v in variants}
    for _ in range(args.rounds):
        for v, (_, r) in runners.items():
            r.run(5)
            ms, _ = r.run(steps)
            res[v].append(ms * 1e3 / steps)
    summary = {}
    for v, xs in res.items():
        summary[v] = {"us_min": round(min(xs), 3), "us_median": round(statistics.median(xs), 3),
                      "Gpkt_s_best": round(n / min(xs) / 1e3, 3), "all": [round(x, 2) for x in xs]}
        print(f"{args.config} {v:28s} min {min(xs):10.2f} us  med {statistics.median(xs):10.2f} us"
              f"  {n / min(xs) / 1e3:7.2f} Gpkt/s", flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
