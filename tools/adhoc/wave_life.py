#!/usr/bin/env python3
"""Measurement tool: long-lived vs short-lived waves on one long C2 launch.
k_parse_pipe over 16 M 64-B frames in one arena (1 GiB) and one launch, with
INGOT_TUNE_PIPELINE = tiles per wave: 0 = the default grid capped at 2
blocks per CU (each wave walks 64 tiles, persistent-like), or 8 / 16 / 32
tiles per wave (grid = tiles / (4 x tpw) blocks, the dispatcher refilling
CUs as blocks finish).  Records: one 256 MiB buffer, or 16 x 1 M records
rotated over 8 buffers by splitting the launch (footprint check).  µs per
1 M frames, single stream.

    python tools/wave_life.py
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, abi

    ctx = ingot_amd.Context(0)
    lib = ingot_amd.load_library()
    m, L = 1 << 20, 16
    base, _, _ = ingot_amd.gen_frames(GenProfile.V4UDP64, m, stride=64)
    base = base.reshape(-1)
    arenas = [base.repeat(L) for _ in range(2)]
    out = torch.empty((L * m, 16), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    h, c = ctx._h, int(Chain.UdpParser)
    s = torch.cuda.current_stream()

    def once(k):
        return lib.ingot_gpu_parse_strided(h, arenas[k % 2].data_ptr(), 64, None, L * m, c,
                                           out.data_ptr(), s.cuda_stream)

    res = {}
    for tpw in (0, 8, 16, 32, 64, 4):
        ctx.set_tuning(abi.TUNE_PIPELINE, tpw)
        vals = []
        for k in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            assert once(k) == 0
            e1.record(s)
            torch.cuda.synchronize()
            if k:
                vals.append(e0.elapsed_time(e1) * 1e3 / L)
        res[f"tpw{tpw}"] = round(statistics.median(vals), 3)
        print(f"tpw{tpw}", res[f"tpw{tpw}"], flush=True)
    ctx.set_tuning(abi.TUNE_PIPELINE, 0)
    Path(ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "wave_life.json").write_text(
        json.dumps({"us_per_1M_frames_single_launch_16M": res}, indent=1))


if __name__ == "__main__":
    main()
