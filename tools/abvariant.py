#!/usr/bin/env python3
"""Measurement tool: A/B of builds (or tunings) of the native library.

Each variant is a libingot_gpu.so in tools/variants/<name>/ (built by
tools/build_variants.sh, or a whole other tree by tools/build_tree_variant.sh
— e.g. the previous commit); "default" is the in-tree library.  A spec
name@KEY=VALUE,... adds ctx tuning (KEY = INGOT_TUNE_* suffix).  Variants run
round robin, each in its own child process (one library per process; the
parent never touches the GPU), on the same device-generated batches; every
child times, one stream, the dominant kernel of each workload (best of 3
windows of `reps` launches) and reports a checksum of its outputs so a
variant that changes results is visible.

    python tools/abvariant.py default head [--rounds 3] [--workloads c3,c4,c5]
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


WORKLOADS = {
    # name: (profile, frames, slot stride or None, chain)
    "c2": ("V4UDP64", 1 << 20, 64, "UdpParser"),
    "c3": ("MIXED", 1 << 24, None, "GenericUlp"),
    "c4": ("VLAN_V6EH", 1 << 23, None, "VlanUlp"),
    "c5": ("FLOWS", 1 << 23, None, "VlanUlp"),
    "c6": ("GENEVE", 1 << 23, None, "GeneveOverV6Tunnel"),
}


def child(spec: str, workloads: list, reps: int) -> dict:
    """spec = name[@key=value,...]: a library variant plus ctx tuning."""
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
    s = torch.cuda.current_stream()

    def timed(fn):
        fn(0)
        torch.cuda.synchronize()
        best = None
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(reps):
                fn(k)
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            best = us if best is None else min(best, us)
        return round(best, 2)

    res = {"variant": spec}
    for w in workloads:
        prof, n, stride, chain_name = WORKLOADS[w]
        chain = Chain[chain_name]
        # arena copies rotated so that a launch reads HBM, not the 256 MiB MALL
        copies = 8 if stride else 2
        data = [ingot_amd.gen_frames(GenProfile[prof], n, seed=20250808, stride=stride)
                for _ in range(copies)]
        out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
        if stride:
            res[f"{w}_parse_us"] = timed(lambda k: ctx.parse_strided(
                data[k % copies][0], stride, n, chain, out=out))
        else:
            res[f"{w}_parse_us"] = timed(lambda k: ctx.parse(
                data[k % copies][0], data[0][1], data[0][2], chain, out=out))
        torch.cuda.synchronize()
        res[f"{w}_records_checksum"] = int(out[:, :8].to(torch.int64).sum().item())
        if w == "c5":
            hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
            flows = torch.zeros(n, dtype=torch.int32, device="cuda")
            ws = ctx.flow_hist_workspace(n, 1 << 16)
            res["c5_flow_hist_us"] = timed(lambda k: ctx.flow_hist(
                data[k % copies][0], data[0][1], data[0][2], chain, hist, flow=flows,
                workspace=ws))
            torch.cuda.synchronize()
            res["c5_flow_checksum"] = int(flows.to(torch.int64).sum().item())
            res["c5_flows_over_parse"] = round(res["c5_flow_hist_us"] / res["c5_parse_us"], 4)
        del data, out
        torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workloads", default="c5")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--child")
    args = ap.parse_args()
    wl = [w for w in args.workloads.split(",") if w]
    if args.child:
        print(json.dumps(child(args.child, wl, args.reps)), flush=True)
        return
    rows = []
    for r in range(args.rounds):
        for v in args.variants:
            p = subprocess.run([sys.executable, __file__, "--child", v, "--workloads",
                                args.workloads, "--reps", str(args.reps), "x"],
                               capture_output=True, text=True, timeout=600)
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
        summary[v] = {}
        for k in mine[0]:
            if k.endswith("_us") or k.endswith("_over_parse"):
                summary[v][k + "_min"] = min(x[k] for x in mine)
            elif k.endswith("checksum"):
                summary[v][k + "s"] = sorted({x[k] for x in mine})
    print(json.dumps(summary, indent=1))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "abvariant.json").write_text(json.dumps({"rows": rows,
                                                                   "summary": summary}, indent=1))


if __name__ == "__main__":
    main()
