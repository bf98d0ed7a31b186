#!/usr/bin/env python3
"""Measurement tool: A/B of compile-time variants of the native library.

Each variant is a libingot_gpu.so built with extra hipcc defines into
tools/variants/<name>/ (tools/build_variants.sh); "default" is the in-tree
library.  Variants run round robin, each in its own child process (one
library per process), on the same device-generated batch; every child times
the config-5 flow kernel (flow_hist, single stream) and the plain parse of
the same frames, and reports a checksum of its flow ids so a variant that
changes results is visible (the hash stub is expected to).

    python tools/abvariant.py default lookup1 stub [--rounds 3]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def child(spec: str, n: int, reps: int) -> dict:
    """spec = name[@key=value,...]: a library variant plus ctx tuning
    (key = INGOT_TUNE_* suffix, e.g. default@WINDOW_INDEXED=4)."""
    import ingot_amd._lib as L

    name, _, tune = spec.partition("@")
    if name != "default":
        L.LIB_PATH = ROOT / "tools" / "variants" / name / "libingot_gpu.so"
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    for kv in filter(None, tune.split(",")):
        k, v = kv.split("=")
        ctx.set_tuning(getattr(ingot_amd.abi, "TUNE_" + k), int(v))
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=20250808)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    flows = torch.zeros(n, dtype=torch.int32, device="cuda")
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    ws = ctx.flow_hist_workspace(n, 1 << 16)
    s = torch.cuda.current_stream()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            best = us if best is None else min(best, us)
        return round(best, 2)

    res = {"variant": spec,
           "flow_hist_us": timed(lambda: ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist,
                                                       flow=flows, workspace=ws)),
           "parse_us": timed(lambda: ctx.parse(arena, off, lens, Chain.VlanUlp, out=out))}
    ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist, flow=flows, workspace=ws)
    torch.cuda.synchronize()
    res["flow_checksum"] = int(flows.to(torch.int64).sum().item())
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--child")
    args = ap.parse_args()
    if args.child:
        print(json.dumps(child(args.child, args.n, args.reps)), flush=True)
        return
    rows = []
    for r in range(args.rounds):
        for v in args.variants:
            p = subprocess.run([sys.executable, __file__, "--child", v, "--n", str(args.n),
                                "--reps", str(args.reps), "x"], capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(p.stdout, p.stderr, flush=True)
                sys.exit(p.returncode)
            row = json.loads(p.stdout.strip().splitlines()[-1])
            row["round"] = r
            rows.append(row)
            print(json.dumps(row), flush=True)
    summary = {}
    for v in args.variants:
        mine = [x for x in rows if x["variant"] == v]
        summary[v] = {"flow_hist_us_min": min(x["flow_hist_us"] for x in mine),
                      "parse_us_min": min(x["parse_us"] for x in mine),
                      "flow_checksums": sorted({x["flow_checksum"] for x in mine})}
    print(json.dumps(summary, indent=1))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "abvariant.json").write_text(json.dumps({"rows": rows,
                                                                   "summary": summary}, indent=1))


if __name__ == "__main__":
    main()
