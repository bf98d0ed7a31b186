#!/usr/bin/env python3
"""Measurement tool: parse kernel vs the streaming ceiling at config-2 size.

Interleaves variants in rounds in one process (cdna_hip_programming.md §5.4
rule 24) and prints µs/step and effective TB/s (80 B per packet) for:
  stream_reg / stream_glds  — tools/stream_ceiling.hip (no parsing)
  parse[g]                  — the product kernel with grid capped at g blocks
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def build_stream():
    out = ROOT / "tools" / "build" / "libstream.so"
    out.parent.mkdir(exist_ok=True)
    src = ROOT / "tools" / "stream_ceiling.hip"
    if not out.exists() or out.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                        str(src), "-o", str(out)], check=True)
    lib = ctypes.CDLL(str(out))
    lib.stream_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_uint32, ctypes.c_void_p]
    return lib


def main():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    n = 1 << 20
    steps = int(os.environ.get("MB_STEPS", "400"))
    rounds = int(os.environ.get("MB_ROUNDS", "3"))
    grids = [int(g) for g in os.environ.get("MB_GRIDS", "1024,2048,4096,8192").split(",")]
    slib = build_stream()
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    reps = 8
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(reps)]
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    lib = ingot_amd.load_library()
    ctxs = {}
    for g in grids:
        os.environ["INGOT_GPU_MAX_BLOCKS"] = str(g)
        ctxs[g] = ingot_amd.Context(0)
    os.environ.pop("INGOT_GPU_MAX_BLOCKS", None)
    ctxs[0] = ingot_amd.Context(0)

    variants = {}
    for g in grids:
        variants[f"stream_reg[{g}]"] = (lambda k, g=g: slib.stream_run(
            0, arenas[k % reps].data_ptr(), outs[k % reps].data_ptr(), n, g, sp))
        variants[f"stream_glds[{g}]"] = (lambda k, g=g: slib.stream_run(
            1, arenas[k % reps].data_ptr(), outs[k % reps].data_ptr(), n, g, sp))
    for g in [0] + grids:
        h = ctxs[g]._h
        variants[f"parse[{g or 'auto'}]"] = (lambda k, h=h: lib.ingot_gpu_parse_strided(
            h, arenas[k % reps].data_ptr(), 64, None, n, int(Chain.UdpParser),
            outs[k % reps].data_ptr(), sp))
    h = ctxs[0]._h
    variants["parse_rec8"] = (lambda k: lib.ingot_gpu_parse_strided_compact(
        h, arenas[k % reps].data_ptr(), 64, None, n, int(Chain.UdpParser),
        outs[k % reps].data_ptr(), sp))
    # independent batches on S streams (consecutive kernels may overlap)
    streams = [s] + [torch.cuda.Stream() for _ in range(3)]
    for ns in (2, 4):
        variants[f"parse_{ns}streams"] = (lambda k, ns=ns: lib.ingot_gpu_parse_strided(
            h, arenas[k % reps].data_ptr(), 64, None, n, int(Chain.UdpParser),
            outs[k % reps].data_ptr(), streams[k % ns].cuda_stream))
        variants[f"parse_rec8_{ns}streams"] = (lambda k, ns=ns: lib.ingot_gpu_parse_strided_compact(
            h, arenas[k % reps].data_ptr(), 64, None, n, int(Chain.UdpParser),
            outs[k % reps].data_ptr(), streams[k % ns].cuda_stream))

    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, fn in variants.items():
            for k in range(20):
                fn(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for st in streams[1:]:
                st.wait_event(e0)
            for k in range(steps):
                fn(k)
            for st in streams[1:]:
                ev = torch.cuda.Event()
                ev.record(st)
                s.wait_event(ev)
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / steps)
    out = {}
    for name, v in res.items():
        us = min(v)
        out[name] = {"us_min": round(us, 3), "us_all": [round(x, 3) for x in v],
                     "TBps": round(n * 80 / us / 1e6, 3)}
        print(f"{name:22s} {us:8.3f} us/step  {n * 80 / us / 1e6:6.3f} TB/s  "
              f"{n / us / 1e3:8.2f} Gpkt/s", flush=True)
    Path(os.environ.get("MB_OUT", ROOT / "gpurun_out" / "microbench.json")).write_text(
        json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
