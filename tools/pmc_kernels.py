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


SIZED = ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum",
         "TCC_EA0_RDREQ_sum"]


def one_pass(counter: str, cmd: list, outdir: Path, by_counter: bool = False) -> dict:
    """One rocprofv3 --pmc pass over `cmd` ("A B ..." = several counters of
    one pass).  {kernel: [value per dispatch]}; by_counter: {counter:
    {kernel: [...]}}."""
    d = outdir / counter.split()[0].lower()
    d.mkdir(parents=True, exist_ok=True)
    full = ["rocprofv3", "--pmc", *counter.split(), "--output-format", "csv", "-d", str(d),
            "-o", "run", "--", *cmd]
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
            cn = row.get("Counter_Name", counter) if by_counter else counter
            key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), name)
            per.setdefault(cn, {}).setdefault(name, {}).setdefault(key, 0.0)
            per[cn][name][key] += float(row.get("Counter_Value", 0) or 0)
    out = {c: {k: list(v.values()) for k, v in ks.items()} for c, ks in per.items()}
    return out if by_counter else out.get(counter, {})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--match", default="ingot_gpu", help="keep kernels whose name has this")
    ap.add_argument("--sized", action="store_true",
                    help="also a pass of the L2->EA read requests by size (TCC_EA0_RDREQ_32B / "
                         "_64B / _128B): read bytes = 32 n32 + 64 n64 + 128 n128, no x2 guess")
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
    if args.sized:
        sz = one_pass(" ".join(SIZED), cmd, outdir, by_counter=True)
        for name, r in res.items():
            n = {c: statistics.median(sz.get(c, {}).get(name, [0]) or [0]) for c in SIZED}
            r["read_requests"] = {"32B": n[SIZED[0]], "64B": n[SIZED[1]], "128B": n[SIZED[2]],
                                  "all": n[SIZED[3]]}
            r["read_bytes_sized"] = 32 * n[SIZED[0]] + 64 * n[SIZED[1]] + 128 * n[SIZED[2]]
    out = {"command": " ".join(cmd),
           "correction": "FETCH_SIZE KiB x 1024 x 2 on gfx950 (MI355X_MICROARCH.md §HBM); "
                         "WRITE_SIZE KiB x 1024",
           "kernels": res}
    Path(args.out).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
