#!/usr/bin/env python3
"""Measurement tool: one pass over a long packed batch (C3: 16.7 M mixed
frames, GenericUlp; or C4 / C6) as ONE launch, against the same pass cut
into S sub-launches of n/S frames alternating over 2 (or 3) streams — each
sub-launch its slice of the descriptors and of the records, all inside one
region (the streams fork from one start event and the region ends at the
last end event).  Do two overlapping short launches beat one long one on the
gather-bound kernels as they do on the C2 ring?

    python tools/split_launch.py [--config c3] [--reps 5]
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    prof, n, stride, chain_name, _ = bench.CONFIGS[args.config]
    assert stride is None
    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    h, c = ctx._h, int(Chain[chain_name])
    ap_, op_, lp_, rp_ = arena.data_ptr(), off.data_ptr(), lens.data_ptr(), out.data_ptr()
    torch.cuda.synchronize()

    def run(S, ns):
        m = n // S
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(streams[0])
        for s in streams[1:ns]:
            s.wait_event(e0)
        for j in range(S):
            cnt = m if j < S - 1 else n - m * (S - 1)
            rc = lib.ingot_gpu_parse(h, ap_, op_ + 8 * m * j, lp_ + 2 * m * j, cnt, c,
                                     rp_ + 16 * m * j, streams[j % ns].cuda_stream)
            assert rc == 0, rc
        ends = []
        for s in streams[:ns]:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ends.append(e)
        torch.cuda.synchronize()
        return max(e0.elapsed_time(e) for e in ends) * 1e3

    variants = {"one_launch": (1, 1), "s2_x4": (4, 2), "s2_x8": (8, 2), "s2_x16": (16, 2),
                "s2_x32": (32, 2), "s3_x16": (16, 3), "s1_x16": (16, 1)}
    res = {k: [] for k in variants}
    ref = None
    for r in range(args.reps):
        for name, (S, ns) in variants.items():
            run(S, ns)
            res[name].append(run(S, ns))
            if ref is None:
                ref = out.clone()
            elif r == 0:
                assert torch.equal(out, ref), name  # every split writes the same records
        print(f"rep {r}: " + " ".join(f"{k}={v[-1]:.1f}" for k, v in res.items()), flush=True)
    summ = {k: round(statistics.median(v), 2) for k, v in res.items()}
    o = {"config": args.config, "frames": n, "us_per_pass_median": summ, "raw": res}
    p = Path(args.out or ROOT / "gpurun_out" / f"split_launch_{args.config}.json")
    p.parent.mkdir(parents=True, exist_ok=True)
    p.write_text(json.dumps(o, indent=1))
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
