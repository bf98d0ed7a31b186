#!/usr/bin/env python3
"""Measurement tool: the parse kernel vs streaming ceilings at config-2 size
(1,048,576 x 64 B), interleaved in rounds in one process
(cdna_hip_programming.md §5.4 rule 24).

  stream_copy  64 B read + 16 B written per packet, no parsing
  stream_read  64 B read per packet, nothing written
  parse        the product kernel (16-B records), parse_rec8 (8-B records)
each on 1 and 2 streams (step k on stream k % S).  Prints µs/step and the
HBM rate for the bytes each variant moves.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
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
    steps = int(os.environ.get("MB_STEPS", "1000"))
    rounds = int(os.environ.get("MB_ROUNDS", "3"))
    slib = build_stream()
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    reps = 8
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(reps)]
    s = torch.cuda.current_stream()
    streams = [s, torch.cuda.Stream()]
    lib = ingot_amd.load_library()
    ctx = ingot_amd.Context(0)
    h = ctx._h
    bytes_per = {"stream_copy": 80, "stream_read": 64, "parse": 80, "parse_rec8": 72}

    def mk(kind, ns):
        def fn(k):
            sp = streams[k % ns].cuda_stream
            a, o = arenas[k % reps].data_ptr(), outs[k % reps].data_ptr()
            if kind == "stream_copy":
                return slib.stream_run(0, a, o, n, 4096, sp)
            if kind == "stream_read":
                return slib.stream_run(2, a, o, n, 4096, sp)
            if kind == "parse":
                return lib.ingot_gpu_parse_strided(h, a, 64, None, n, int(Chain.UdpParser), o, sp)
            return lib.ingot_gpu_parse_strided_compact(h, a, 64, None, n, int(Chain.UdpParser),
                                                       o, sp)
        return fn

    variants = {f"{k}_s{ns}": (mk(k, ns), ns, k) for k in bytes_per for ns in (1, 2)}
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, (fn, ns, _) in variants.items():
            for k in range(20):
                fn(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            streams[1].wait_event(e0)
            for k in range(steps):
                fn(k)
            ev = torch.cuda.Event()
            ev.record(streams[1])
            s.wait_event(ev)
            e1.record(s)
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / steps)
    out = {}
    for name, v in res.items():
        us = min(v)
        b = bytes_per[variants[name][2]]
        out[name] = {"us_min": round(us, 3), "TBps": round(n * b / us / 1e6, 3),
                     "Gpkt_s": round(n / us / 1e3, 2)}
        print(f"{name:18s} {us:8.3f} us/step  {n * b / us / 1e6:6.3f} TB/s ({b} B/pkt)  "
              f"{n / us / 1e3:7.2f} Gpkt/s", flush=True)
    Path(os.environ.get("MB_OUT", ROOT / "gpurun_out" / "microbench.json")).write_text(
        json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
