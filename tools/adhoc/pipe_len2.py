#!/usr/bin/env python3
"""Measurement tool: is it kernel LENGTH or kernel CONCURRENCY that sets the
C2 rate?  k_parse_pipe (the per-batch ring kernel, unchanged) over batches of
L M frames, L = 1, 2, 4, 8, 16, each batch its own arena copy, on one stream
or on two streams with stream 1 started half a launch late — µs per 1 M
frames in 10-launch regions after a warm-up.  Also the persistent ring
consumer (k_parse_ring) over 20 x 1 M batches on one and on two streams.

    python tools/pipe_len2.py [--out F]
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
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "pipe_len2.json"))
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    m = 1 << 20
    base, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, m, stride=64)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    res = {}
    for L in (1, 2, 4, 8, 16):
        n = L * m
        reps = max(2, 8 // L)  # arena copies: >= 512 MiB rotated, >= 2
        arenas = [base.repeat(L, 1).reshape(-1) if base.dim() == 2 else base.repeat(L)
                  for _ in range(reps)]
        outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(reps)]
        torch.cuda.synchronize()
        stag = 6.0 * L
        for ns in (1, 2):
            r = bench.Runner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, None, None, outs,
                             streams[:ns], 16)
            g = bench.Gate(ingot_amd, ctx, stag if ns == 2 else 0.0)
            vals = []
            for _ in range(args.reps):
                r.run(4, g)
                torch.cuda.synchronize()
                ms, _ = r.run(10, g)
                vals.append(ms * 1e3 / 10 / L)
            res[f"pipe_{L}M_s{ns}"] = round(statistics.median(vals), 3)
            print(f"pipe_{L}M_s{ns}", res[f"pipe_{L}M_s{ns}"], flush=True)
        del arenas, outs
        torch.cuda.empty_cache()
    # the persistent consumer over 20 x 1 M batches, one and two streams
    arenas = [base] + [base.clone() for _ in range(7)]
    outs = [torch.empty((m, 16), dtype=torch.uint8, device="cuda") for _ in range(20)]
    for ns in (1, 2):
        rr = bench.RingRunner(torch, lib, ctx, Chain.UdpParser, m, 64, arenas, outs, streams[:ns],
                              16, 20)
        g = bench.Gate(ingot_amd, ctx, 60.0 if ns == 2 else 0.0)
        vals = []
        for _ in range(args.reps):
            rr.warm(20, g)
            torch.cuda.synchronize()
            ms, _ = rr.run(20, g)
            vals.append(ms * 1e3 / 20)
        res[f"ring_20x1M_s{ns}"] = round(statistics.median(vals), 3)
        print(f"ring_20x1M_s{ns}", res[f"ring_20x1M_s{ns}"], flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps({"us_per_1M_frames": res}, indent=1))


if __name__ == "__main__":
    main()
