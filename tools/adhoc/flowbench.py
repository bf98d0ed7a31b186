#!/usr/bin/env python3
"""Measurement tool: where does the flow-histogram step spend its time?
Interleaved in one process: parse only (compact records), flow_hist with
65,536 bins, with 2^24 bins (contention spread), on Zipf flows and on
uniform flows (MIXED)."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    n = int(os.environ.get("FB_N", str(1 << 23)))
    ctx = ingot_amd.Context(0)
    data = {p: ingot_amd.gen_frames(GenProfile[p], n) for p in ("FLOWS", "VLAN_V6EH")}
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    h16 = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    h24 = torch.zeros(1 << 24, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    variants = {}
    for p, (a, o, l) in data.items():
        variants[f"{p}:parse_rec8"] = lambda a=a, o=o, l=l: ctx.parse_compact(a, o, l,
                                                                              Chain.VlanUlp, out)
        variants[f"{p}:flow_2^16"] = lambda a=a, o=o, l=l: ctx.flow_hist(a, o, l, Chain.VlanUlp,
                                                                         h16)
        variants[f"{p}:flow_2^24"] = lambda a=a, o=o, l=l: ctx.flow_hist(a, o, l, Chain.VlanUlp,
                                                                         h24)
    res = {k: [] for k in variants}
    for _ in range(3):
        for k, fn in variants.items():
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 100)
    for k, v in res.items():
        print(f"{k:28s} {min(v):9.1f} us  {n / min(v) / 1e3:7.2f} Gpkt/s", flush=True)


if __name__ == "__main__":
    main()
