#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of the default `python bench.py` run into
bench.py's phases and average the parse kernel's dispatch duration in each,
so the profile of the exact bench command can be checked against the JSON
line: `roofline.launch_mean_us` is the single-stream pass's per-launch time,
and in that phase each dispatch runs alone on the GPU.

bench.py's dispatch order for one config (parse kernel only): warmup W and
timed K steps (2 streams: launches overlap), one algorithmic-bytes parse, the
single-stream pass (min(W, 50) + min(K, 1000)), then the variants
(min(W, 50) + min(K, 1000) each).

    python tools/rocprof_phases.py gpurun_out/prof_bench_default/run_kernel_trace.csv \
        --kernel k_parse_pipe --warmup 100 --steps 2000 > profiles/r01_c2_bench_phases.json
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="k_parse_pipe")
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--steps", type=int, default=2000)
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    t0 = [int(r["Start_Timestamp"]) for r in rows]
    t1 = [int(r["End_Timestamp"]) for r in rows]
    W, K = args.warmup, args.steps
    w_iso, k_iso = min(W, 50), min(K, 1000)
    phases = {}
    i = 0

    def take(name, count):
        nonlocal i
        seg = slice(i, i + count)
        dd = d[seg]
        if dd:
            span = (t1[i + count - 1] - t0[i]) / 1e3 if count else 0.0
            phases[name] = {"dispatches": len(dd), "mean_us": round(statistics.fmean(dd), 3),
                            "median_us": round(statistics.median(dd), 3),
                            "span_us_per_dispatch": round(span / len(dd), 3)}
        i += count

    take("warmup (2 streams)", W)
    take("timed region (2 streams, overlapping)", K)
    take("algorithmic-bytes parse", 1)
    take("single-stream warmup", w_iso)
    take("single-stream pass (roofline.launch_mean_us)", k_iso)
    for v in ("streams1_rec16", "streams2_rec8", "streams1_rec8", "streams4_rec16"):
        take(f"variant {v} warmup", w_iso)
        take(f"variant {v}", k_iso)
    out = {"trace": args.trace, "kernel": args.kernel, "dispatches_total": len(d),
           "dispatches_assigned": i, "phases": phases,
           "all_dispatches_mean_us": round(statistics.fmean(d), 3) if d else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
