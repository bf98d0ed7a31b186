#!/usr/bin/env python3
"""Where a short timed region's time goes (C2, the driver's 20-step bench).

Times gated regions of K steps for K = 1 .. 2000 and fits T(K) = a + b*K
(a = the fixed cost per region, b = the steady per-step time), and times
20-step regions after different preparations: idle gaps before the region,
every arena copy touched first, one vs two streams.

    python tools/region_probe.py [--config c2] > gpurun_out/region_probe.json
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
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
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(R)]
    torch.cuda.synchronize()
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(3)]
    gate = bench.Gate(ingot_amd, ctx)

    def runner(ns, rec=16):
        return bench.Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs,
                            streams[:ns], rec)

    r2 = runner(2)
    r1 = runner(1)
    r2.run(50, gate)
    out = {"config": args.config, "copies": R}

    def med(f, reps=args.reps):
        v = [f() for _ in range(reps)]
        return round(statistics.median(v), 3), [round(x, 2) for x in v]

    # T(K) for 2 streams, back to back
    tk = {}
    for K in (1, 2, 4, 8, 20, 50, 200, 2000):
        m, _ = med(lambda: r2.run(K, gate)[0] * 1e3)
        tk[K] = m
    out["region_us_by_steps_2streams"] = tk
    ks = sorted(tk)
    xs, ys = ks, [tk[k] for k in ks]
    mx, my = statistics.fmean(xs), statistics.fmean(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    out["fit_2streams"] = {"fixed_us": round(my - b * mx, 2), "per_step_us": round(b, 3)}
    tk1 = {}
    for K in (1, 2, 4, 20, 200):
        tk1[K] = med(lambda: r1.run(K, gate)[0] * 1e3)[0]
    out["region_us_by_steps_1stream"] = tk1

    # 20-step regions after different preparations
    def after(prep):
        def f():
            prep()
            return r2.run(20, gate)[0] * 1e3 / 20
        return f

    def idle(s):
        return lambda: (torch.cuda.synchronize(), time.sleep(s))

    def warm(k):
        return lambda: (r2.run(k, gate), torch.cuda.synchronize())

    out["us_per_step_20"] = {
        "back_to_back": med(after(lambda: None)),
        "after_1ms_idle": med(after(idle(0.001))),
        "after_50ms_idle": med(after(idle(0.05))),
        "after_500ms_idle": med(after(idle(0.5))),
        "after_warm5": med(after(warm(5))),
        "after_warm8_all_copies": med(after(warm(R))),
        "after_warm64": med(after(warm(64))),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
