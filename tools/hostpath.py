#!/usr/bin/env python3
"""Measurement tool: the host-inclusive rate.  The path starts and ends in host
memory (a NIC/loopback ring): pinned host arena -> hipMemcpyAsync H2D ->
parse -> records D2H into pinned host memory.  Steps are pipelined over S
streams (copy of batch k+1 overlaps the parse of batch k).  Reported in
DESIGN.md; never the bench `value` (which is device-resident).

    python tools/hostpath.py [--config c2|c3] [--streams 3] [--steps 200]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()

    import torch

    import bench
    import ingot_amd
    from ingot_amd import Chain, GenProfile

    prof, _, stride, chain_name, _ = bench.CONFIGS[args.config]
    n = args.frames
    chain = Chain[chain_name]
    ctx = ingot_amd.Context(0)
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, stride=stride)
    S = args.streams
    streams = [torch.cuda.Stream() for _ in range(S)]
    R = S + 1
    host_arena = [torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True) for _ in range(R)]
    for h in host_arena:
        h.copy_(arena)
    host_recs = [torch.empty((n, 16), dtype=torch.uint8, pin_memory=True) for _ in range(R)]
    dev_arena = [torch.empty_like(arena) for _ in range(S)]
    dev_recs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(S)]
    # descriptors live on the device (a ring's descriptor table would be
    # copied too: add 10 B/pkt; counted below)
    desc_bytes = 0 if stride else n * 10
    host_desc = None
    if off is not None:
        host_desc = (torch.empty(n, dtype=torch.int64, pin_memory=True),
                     torch.empty(n, dtype=torch.uint16, pin_memory=True))
        host_desc[0].copy_(off)
        host_desc[1].copy_(lens)
        dev_desc = [(torch.empty_like(off), torch.empty_like(lens)) for _ in range(S)]

    def step(k):
        s = streams[k % S]
        with torch.cuda.stream(s):
            dev_arena[k % S].copy_(host_arena[k % R], non_blocking=True)
            if host_desc is not None:
                o, ln = dev_desc[k % S]
                o.copy_(host_desc[0], non_blocking=True)
                ln.copy_(host_desc[1], non_blocking=True)
                ctx.parse(dev_arena[k % S], o, ln, chain, out=dev_recs[k % S], stream=s)
            else:
                ctx.parse_strided(dev_arena[k % S], stride, n, chain, out=dev_recs[k % S],
                                  stream=s)
            host_recs[k % R].copy_(dev_recs[k % S], non_blocking=True)

    for k in range(2 * S):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    h2d = arena.numel() + desc_bytes
    d2h = n * 16
    # raw copy ceilings for context
    t1 = time.perf_counter()
    for k in range(50):
        dev_arena[0].copy_(host_arena[k % R], non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbs = 50 * arena.numel() / (time.perf_counter() - t1) / 1e9
    res = {
        "config": args.config, "frames_per_batch": n, "streams": S, "steps": args.steps,
        "host_inclusive_Mpkt_s": round(n * args.steps / dt / 1e6, 1),
        "ms_per_batch": round(dt / args.steps * 1e3, 4),
        "bytes_h2d_per_batch": h2d, "bytes_d2h_per_batch": d2h,
        "pcie_GBps_effective": round((h2d + d2h) * args.steps / dt / 1e9, 2),
        "h2d_copy_only_GBps": round(h2d_gbs, 2),
    }
    print(json.dumps(res))
    out = ROOT / "gpurun_out" / f"hostpath_{args.config}.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
