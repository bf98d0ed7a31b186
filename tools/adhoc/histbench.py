#!/usr/bin/env python3
"""Measurement tool: cost of the per-flow histogram's flush on config-5 flow
ids (tools/stream_ceiling.hip k_h16): packed 16-bit LDS counters per block,
flushed as global atomics (mode 0, the product design), as plain stores into
per-block rows + a reduce pass (mode 1), or not at all (mode 2: counting
only); and the product's ingot_gpu_flow_hist histogram for reference."""
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
    from ingot_amd import Chain, GenProfile
    from microbench import build_stream

    slib = build_stream()
    slib.h16_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    n = 1 << 23
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n)
    ctx = ingot_amd.Context(0)
    hist = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hist=hist, n=n)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    rows = torch.empty((512, 32768), dtype=torch.int32, device="cuda")
    res = {}
    for g in (128, 256, 512):
        for mode in (0, 1, 2):
            def fn():
                slib.h16_run(mode, flow.data_ptr(), n, hist.data_ptr(), rows.data_ptr(), g,
                             s.cuda_stream)
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            res[(g, mode)] = e0.elapsed_time(e1) * 1e3 / 20
            print(f"g={g:4d} mode={mode} {res[(g, mode)]:8.1f} us", flush=True)
    # check mode 1 reproduces the histogram
    h1 = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    h0 = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    slib.h16_run(1, flow.data_ptr(), n, h1.data_ptr(), rows.data_ptr(), 256, s.cuda_stream)
    slib.h16_run(0, flow.data_ptr(), n, h0.data_ptr(), rows.data_ptr(), 256, s.cuda_stream)
    torch.cuda.synchronize()
    print("rows == atomics:", bool((h0 == h1).all()), flush=True)


if __name__ == "__main__":
    main()
