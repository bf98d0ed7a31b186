#!/usr/bin/env python3
"""Measurement tool: HBM fetch granularity on config-3 frames.  Per packet,
read NSEG aligned SEG-byte segments at its frame start (tools/stream_ceiling.hip
k_gather_seg), interleaved rounds in one process.  If time scales with SEG
down to 32/64 B, partial-line fetches are real and a parse that touches only
its header sectors moves fewer bytes than whole 128-B lines.

    python tools/segbench.py            # timing
    SEG_ONLY=1 rocprofv3 --pmc ... -- python3 tools/segbench.py   # counters
"""
import ctypes
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main():
    import torch

    import ingot_amd
    from ingot_amd import GenProfile
    from microbench import build_stream

    slib = build_stream()
    slib.seg_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64,
                                                                     ctypes.c_void_p]
    n = int(os.environ.get("SEG_N", str(1 << 24)))
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    names = {0: "32x1", 5: "32x2", 1: "64x1", 2: "64x2", 3: "128x1", 4: "128x2"}
    only = os.environ.get("SEG_ONLY")
    if only:
        names = {k: v for k, v in names.items() if v == only} or names
    steps = int(os.environ.get("SEG_STEPS", "10"))
    res = {v: [] for v in names.values()}
    for _ in range(int(os.environ.get("SEG_ROUNDS", "3"))):
        for w, v in names.items():
            slib.seg_run(w, arena.data_ptr(), off.data_ptr(), lens.data_ptr(), out.data_ptr(), n, sp)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(steps):
                slib.seg_run(w, arena.data_ptr(), off.data_ptr(), lens.data_ptr(), out.data_ptr(),
                             n, sp)
            e1.record(s)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / steps)
    for v, xs in res.items():
        us = min(xs)
        seg, k = (int(x) for x in v.split("x"))
        print(f"seg {v:6s} {us:9.1f} us  {n / us / 1e3:7.2f} Gpkt/s  requested "
              f"{n * (seg * k + 26) / us / 1e6:6.3f} TB/s", flush=True)


if __name__ == "__main__":
    main()
