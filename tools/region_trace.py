#!/usr/bin/env python3
"""Break the C2 timed region down from a rocprofv3 kernel trace of exactly the
driver's command (`bench.py --gpus 1 --steps 20 --warmup 5`):

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- \\
        python3 bench.py --gpus 1 --steps 20 --warmup 5
    python tools/region_trace.py D/run_kernel_trace.csv --warmup 5 --steps 20

bench.py's parse-kernel dispatches in order: W warm-up steps, the K timed
steps (the region), then the ungated re-run, the algorithmic-bytes parse, the
single-stream roofline pass and the variants.  For the region's K dispatches
this reports, on the device clock of the trace:
  * region: first start -> last end;
  * stagger: first dispatch start -> the other stream's first start, during
    which one stream runs alone;
  * tail: the other stream's last end -> the region's end (one stream alone);
  * gaps: per stream, next start - previous end (the dependent-launch
    boundary);
  * overlapped: the span where both streams have a dispatch running, and the
    time per batch inside it (the steady two-stream rate);
  * what the region would take at that steady rate with no solo stretches.
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
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--bytes-per-step", type=float, default=(64 + 16) * (1 << 20))
    ap.add_argument("--read-bytes-per-step", type=float, default=64 * (1 << 20))
    args = ap.parse_args()
    rows = [r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    reg = rows[args.warmup:args.warmup + args.steps]
    qkey = "Stream_Id" if "Stream_Id" in reg[0] else "Queue_Id"
    t0 = min(int(r["Start_Timestamp"]) for r in reg)
    d = [{"q": r[qkey], "start_us": (int(r["Start_Timestamp"]) - t0) / 1e3,
          "end_us": (int(r["End_Timestamp"]) - t0) / 1e3} for r in reg]
    for x in d:
        x["dur_us"] = x["end_us"] - x["start_us"]
    region = max(x["end_us"] for x in d)
    queues = sorted({x["q"] for x in d})
    per_q = {q: [x for x in d if x["q"] == q] for q in queues}
    firsts = sorted(min(x["start_us"] for x in v) for v in per_q.values())
    lasts = sorted(max(x["end_us"] for x in v) for v in per_q.values())
    stagger = firsts[1] - firsts[0] if len(firsts) > 1 else 0.0
    tail = lasts[-1] - lasts[-2] if len(lasts) > 1 else 0.0
    gaps = []
    for v in per_q.values():
        for a, b in zip(v, v[1:]):
            gaps.append(b["start_us"] - a["end_us"])
    # steady: the overlapped span [second stream's first start, first stream's last end]
    lo, hi = (firsts[-1], lasts[0]) if len(firsts) > 1 else (0.0, region)
    inside = [x for x in d if x["start_us"] >= lo and x["end_us"] <= hi]
    # batches completed per us inside the overlap, from dispatch time shares
    share = sum(max(0.0, min(x["end_us"], hi) - max(x["start_us"], lo)) / x["dur_us"] for x in d)
    steady_us = (hi - lo) / share if share > 0 else None
    out = {
        "dispatches": len(d),
        "streams": len(queues),
        "region_us": round(region, 3),
        "us_per_step": round(region / args.steps, 3),
        "read_frac": round(args.read_bytes_per_step * args.steps / (region * 1e-6) / 8e12, 4),
        "stagger_us": round(stagger, 3),
        "tail_us": round(tail, 3),
        "gap_us_median": round(statistics.median(gaps), 3) if gaps else None,
        "gap_us_sum": round(sum(gaps), 3),
        "dispatch_us_median": round(statistics.median(x["dur_us"] for x in d), 3),
        "first_dispatch_us": round(d[0]["dur_us"], 3),
        "last_dispatch_us": round(d[-1]["dur_us"], 3),
        "overlap_span_us": round(hi - lo, 3),
        "steady_us_per_step_in_overlap": round(steady_us, 3) if steady_us else None,
        "region_at_steady_rate_us": round(steady_us * args.steps, 3) if steady_us else None,
        "fixed_cost_us": round(region - steady_us * args.steps, 3) if steady_us else None,
        "dispatch_timeline": [{k: (round(v, 3) if isinstance(v, float) else v)
                               for k, v in x.items()} for x in d],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
