#!/usr/bin/env python3
"""Measurement tool: the C5 flows kernel (parse + RSS Toeplitz 5-tuple hash,
a 4-B flow id per frame) against the plain parse (16-B records) over the SAME
frames (8,388,608 FLOWS frames, packed, VlanUlp), interleaved on one stream in
one process, each launch timed with HIP events.  Run it under
`rocprofv3 --kernel-trace --stats` for the per-dispatch means of both kernels,
and under tools/pmc_kernels.py for their HBM bytes.

    python tools/c5_same_run.py [--reps 10] [--tune KEY=VALUE ...] [--out F]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--frames", type=int, default=1 << 23)
    ap.add_argument("--variant", action="append", default=[],
                    help="an extra flows variant: KEY=VALUE[,KEY=VALUE] (abi.TUNE_<KEY>), "
                         "applied to its launches only")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "c5_same_run.json"))
    args = ap.parse_args()

    import numpy as np
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, abi

    ctx = ingot_amd.Context(0)
    n = args.frames
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n)
    flow = torch.empty(n, dtype=torch.int32, device="cuda")
    recs = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    def flows_with(spec):
        tune = [(getattr(abi, "TUNE_" + kv.split("=")[0].upper()), int(kv.split("=")[1]))
                for kv in spec.split(",") if kv]

        def go():
            for k, v in tune:
                ctx.set_tuning(k, v)
            ctx.flow_hist(arena, off, lens, Chain.VlanUlp, bins=65536, flow=flow)
            for k, _ in tune:
                ctx.set_tuning(k, 0)
        return go

    def parse():
        ctx.parse(arena, off, lens, Chain.VlanUlp, out=recs)

    kinds = {"flows": flows_with(""), "parse": parse}
    for spec in args.variant:
        kinds["flows@" + spec] = flows_with(spec)
    for fn in kinds.values():  # warm
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in kinds}
    for r in range(args.reps):
        for name, fn in kinds.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3)
        print(f"rep {r}: " + " ".join(f"{k}={v[-1]:.1f}" for k, v in res.items()), flush=True)

    # algorithmic bytes: per frame min(len,128) + max(0, H-128)
    # + 10 descriptor bytes read; 4 (flow id) or 16 (record) written
    r = ingot_amd.records_to_numpy(recs)
    ln = lens.cpu().numpy().astype(np.int64)
    h = r["payload_off"].astype(np.int64)
    rd = int((np.minimum(ln, 128) + np.maximum(0, h - 128) + 10).sum())
    alg = {k: rd + (16 if k == "parse" else 4) * n for k in kinds}
    out = {"frames": n, "profile": "FLOWS", "chain": "VlanUlp", "variants": args.variant,
           "read_bytes": rd, "algorithmic_bytes": alg, "us": res,
           "summary": {k: {"median_us": round(statistics.median(v), 2),
                           "min_us": round(min(v), 2),
                           "frac": round(alg[k] / (statistics.median(v) * 1e-6) / 8e12, 4)}
                       for k, v in res.items()}}
    m = out["summary"]
    out["flows_vs_parse"] = round(m["flows"]["median_us"] / m["parse"]["median_us"], 4)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out["summary"]), out["flows_vs_parse"])


if __name__ == "__main__":
    main()
