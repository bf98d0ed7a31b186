#!/usr/bin/env python3
"""Measurement tool: gather ceiling for config-3 frames vs the parse kernel
(indexed layout), one process, interleaved rounds."""
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
    slib.gather_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64,
                                                                        ctypes.c_void_p]
    n = int(os.environ.get("GB_N", str(1 << 24)))
    prof = GenProfile[os.environ.get("GB_PROFILE", "MIXED")]
    arena, off, lens = ingot_amd.gen_frames(prof, n)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    lib = ingot_amd.load_library()
    ctx = ingot_amd.Context(0)
    names = {0: "gather_reg5", 1: "gather_reg8", 2: "gather_reg9", 3: "gather_glds5",
             4: "gather_glds9", 9: "desc_only"}
    variants = {v: (lambda w=w: slib.gather_run(w, arena.data_ptr(), off.data_ptr(),
                                                 lens.data_ptr(), out.data_ptr(), n, sp))
                for w, v in names.items()}
    variants["parse"] = lambda: lib.ingot_gpu_parse(ctx._h, arena.data_ptr(), off.data_ptr(),
                                                    lens.data_ptr(), n, int(Chain.GenericUlp),
                                                    out.data_ptr(), sp)
    steps = int(os.environ.get("GB_STEPS", "20"))
    res = {k: [] for k in variants}
    for _ in range(3):
        for k, fn in variants.items():
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(steps):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / steps)
    for k, v in res.items():
        us = min(v)
        print(f"{k:14s} {us:9.1f} us  {n / us / 1e3:7.2f} Gpkt/s  "
              f"{n * 154 / us / 1e6:6.3f} TB/s@154B", flush=True)


if __name__ == "__main__":
    main()
