#!/usr/bin/env python3
"""Profiling driver: back-to-back launches of the single-batch ring kernel
(k_parse_pipe) and of the persistent ring consumer (k_parse_ring) over the
same C2 batches, one stream, no gate — a short program to run under
`rocprofv3 --pmc ...` so the two kernels' counters can be compared.

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 tools/ring_probe.py
"""
from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    n = 1 << 20
    arena, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)
    arenas = [arena] + [arena.clone() for _ in range(7)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device="cuda") for _ in range(20)]
    s = torch.cuda.current_stream()
    pipe = bench.Runner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, None, None, outs[:8],
                        [s], 16)
    ring1 = bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, outs, s, 16, 1)
    ring20 = bench.RingRunner(torch, lib, ctx, Chain.UdpParser, n, 64, arenas, outs, s, 16, 20)
    for r in (pipe, ring1, ring20):
        r.run(20)
    torch.cuda.synchronize()
    for name, r in (("pipe", pipe), ("ring_G1", ring1), ("ring_G20", ring20)):
        ms, _ = r.run(40)
        print(f"{name}: {ms * 1e3 / 40:.3f} us per batch", flush=True)


if __name__ == "__main__":
    main()
