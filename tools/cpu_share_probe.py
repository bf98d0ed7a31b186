#!/usr/bin/env python3
"""Measurement tool: the CPU baseline's run-to-run spread against its worker
count, on the host it runs on (no GPU needed).  1 M C2-shaped frames (64-B
Eth/IPv4/UDP slots) built on the host; bench.cpu_baseline with 4 / 8 / 12 /
15 workers, twice each, interleaved; per run the value, the CPU share the
workers obtained and the spread.  Tells host contention (share < 1 at every
count) from the cgroup quota (share < 1 only near the quota).

    python tools/cpu_share_probe.py [--out gpurun_out/cpu_share_probe.json]
"""
from __future__ import annotations

import argparse
import json
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def c2_frames(n: int) -> np.ndarray:
    """n 64-B slots: Eth (00.. / ff..) / IPv4 ihl 5 proto 17 TTL 0xf0 / UDP."""
    f = bytearray(64)
    f[6:12] = b"\xff" * 6
    f[12:14] = b"\x08\x00"
    f[14] = 0x45
    struct.pack_into(">H", f, 16, 50)
    f[22], f[23] = 0xF0, 17
    f[26:34] = bytes(range(8))
    struct.pack_into(">HHH", f, 34, 1234, 5678, 30)
    return np.tile(np.frombuffer(bytes(f), dtype=np.uint8), n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--workers", default="4,8,12,15")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "cpu_share_probe.json"))
    args = ap.parse_args()
    import bench
    from ingot_amd import Chain

    arena = c2_frames(args.frames)
    res = []
    for rep in range(2):
        for w in (int(x) for x in args.workers.split(",")):
            r = bench.cpu_baseline(arena, None, None, 64, args.frames, Chain.UdpParser,
                                   budget_s=1.5, workers=w)
            row = {"workers": r["cores"], "rep": rep, "value": r["value"],
                   "run_spread": r["run_spread"], "runs": r["runs"],
                   "runs_cpu_share": r["runs_cpu_share"],
                   "single_core_value": r["single_core_value"],
                   "per_worker": round(r["value"] / r["cores"], 2)}
            res.append(row)
            print(json.dumps(row), flush=True)
    info = {k: v for k, v in r.items() if k not in ("value", "runs", "runs_cpu_share", "sample")}
    out = {"what": __doc__.strip().splitlines()[0], "host": info, "rows": res}
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
