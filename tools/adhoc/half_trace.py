#!/usr/bin/env python3
"""Measurement tool: the two C2 two-stream schedules under a kernel trace.
Runs one 20-step region (after a 5-step warm-up) of the staggered schedule
(bench.Runner + a 6-us stream delay) and of the half-offset schedule
(bench.HalfOffsetRunner: stream 1 opens with half a batch and closes with
the other half, both streams start together); `--analyze TRACE` then splits
the k_parse_pipe dispatches of the trace by region and reports each region's
span, the stretches where one stream ran alone and the per-dispatch times.

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 tools/half_trace.py
    python tools/half_trace.py --analyze D/run_kernel_trace.csv
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

ORDER = ("stagger", "half")  # warm-up + timed region each, in this order


def run():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    n = 1 << 20
    a0, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    arenas = [a0] + [a0.clone() for _ in range(7)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(8)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    runners = {
        "stagger": (bench.Runner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, None, None,
                                 outs, streams, 16), bench.Gate(ingot_amd, ctx, 6.0)),
        "half": (bench.HalfOffsetRunner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, outs,
                                        streams, 16), bench.Gate(ingot_amd, ctx, 0.0)),
    }
    res = {}
    for name in ORDER:
        r, g = runners[name]
        r.run(5, g)
        torch.cuda.synchronize()
        ms, _ = r.run(20, g)
        res[name] = round(ms * 1e3 / 20, 3)
    print(json.dumps({"us_per_step_events": res}))


def analyze(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_parse_pipe" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    # dispatches per region: stagger 5 + 20; half plan(5) + plan(20)
    counts = {"stagger": (5, 20), "half": (6, 21)}
    i, out = 0, {}
    for name in ORDER:
        w, k = counts[name]
        reg = rows[i + w:i + w + k]
        i += w + k
        t0 = min(int(r["Start_Timestamp"]) for r in reg)
        d = [(r[qkey], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3)
             for r in reg]
        end = max(e for _, _, e in d)
        # time with exactly one dispatch running
        ev = sorted([(s, 1) for _, s, _ in d] + [(e, -1) for _, _, e in d])
        solo = cur = 0.0
        last, act = 0.0, 0
        for t, dv in ev:
            if act == 1:
                solo += t - last
            act += dv
            last = t
        out[name] = {"region_us": round(end, 3), "us_per_step": round(end / 20, 3),
                     "one_dispatch_running_us": round(solo, 3),
                     "dispatch_us": [round(e - s, 2) for _, s, e in d],
                     "starts_us": [round(s, 2) for _, s, _ in d],
                     "streams": [q for q, _, _ in d]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze")
    a = ap.parse_args()
    analyze(a.analyze) if a.analyze else run()
