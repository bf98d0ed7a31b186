#!/usr/bin/env python3
"""Measurement tool: HBM bytes per dispatch of EVERY kernel of a command,
from rocprofv3 PMC counters, one counter per pass (MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE in separate --pmc passes, both KiB; FETCH_SIZE
doubled on gfx950).  Prints and writes {kernel: {fetch_bytes, write_bytes,
dispatches}} (medians over the kernel's dispatches).

    python tools/pmc_kernels.py --out gpurun_out/pmc.json -- python3 tools/c5_same_run.py --reps 3
(run on the GPU box; the profiled program goes directly after `--`).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def one_pass(counter: str, cmd: list, outdir: Path) -> dict:
    d = outdir / counter.lower()
    d.mkdir(parents=True, exist_ok=True)
    full = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", str(d), "-o", "run",
            "--", *cmd]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(full, cwd=str(ROOT), env=env, capture_output=True, text=True, timeout=240)
    (d / "rocprof.log").write_text(r.stdout + "\n" + r.stderr)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed ({r.returncode}); see {d}/rocprof.log")
    files = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {d}")
    per = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), name)
            per.setdefault(name, {}).setdefault(key, 0.0)
            per[name][key] += float(row.get("Counter_Value", 0) or 0)
    return {k: list(v.values()) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", default="ingot_gpu", help="keep kernels whose name has this")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    args = ap.parse_args()
    cmd = args.cmd[1:] if args.cmd and args.cmd[0] == "--" else args.cmd
    outdir = Path(args.out).with_suffix("")
    fetch = one_pass("FETCH_SIZE", cmd, outdir)
    write = one_pass("WRITE_SIZE", cmd, outdir)
    res = {}
    for name in sorted(set(fetch) | set(write)):
        if args.match not in name:
            continue
        f, w = fetch.get(name, []), write.get(name, [])
        res[name] = {
            "dispatches": [len(f), len(w)],
            "fetch_bytes": statistics.median(f) * 1024 * 2 if f else None,
            "write_bytes": statistics.median(w) * 1024 if w else None,
        }
    out = {"command": " ".join(cmd),
           "correction": "FETCH_SIZE KiB x 1024 x 2 on gfx950 (MI355X_MICROARCH.md §HBM); "
                         "WRITE_SIZE KiB x 1024",
           "kernels": res}
    Path(args.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
