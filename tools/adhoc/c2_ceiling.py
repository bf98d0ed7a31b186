#!/usr/bin/env python3
"""Why C2 with 16-B records cannot reach 0.70 of the 8 TB/s HBM *read*
roofline: measured HBM bytes per second (PMC) of the parse kernel with 16-
and 8-B records and of two no-parse streaming kernels over the same arenas
(tools/stream_ceiling.hip: read-only, and read 64 B + write 16 B).

Runs tools/microbench.py three times: once for the timings (1,000 steps,
3 interleaved rounds, 1 and 2 streams) and once under each of two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md's
recipe: separate passes, FETCH_SIZE x2 on gfx950).  Writes
profiles/<tag>_c2_ceiling.json.

    python tools/c2_ceiling.py --tag r02        (on the GPU box)
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

ROOT = Path(__file__).resolve().parents[2]
KERNELS = {"k_read": "stream_read", "k_reg": "stream_copy",
           "k_parse_pipe<4u, 2u, 0, 0>": "parse", "k_parse_pipe<4u, 2u, 0, 1>": "parse_rec8"}


def pmc_pass(counter: str, out: Path) -> dict:
    d = out / counter.lower()
    d.mkdir(parents=True, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp", MB_STEPS="20", MB_ROUNDS="1",
               MB_OUT=str(d / "mb.json"))
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", str(d), "-o", "run",
           "--", sys.executable, str(ROOT / "tools" / "microbench.py")]
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    (d / "rocprof.log").write_text(r.stdout + "\n" + r.stderr)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed; see {d}/rocprof.log")
    f = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") != counter:
            continue
        for k, v in KERNELS.items():
            if k in row["Kernel_Name"]:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                per.setdefault(v, {}).setdefault(key, 0.0)
                per[v][key] += float(row["Counter_Value"])
    return {v: statistics.median(x.values()) for v, x in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    args = ap.parse_args()
    out = ROOT / "gpurun_out" / "c2_ceiling"
    out.mkdir(parents=True, exist_ok=True)
    tj = out / "timing.json"
    subprocess.run([sys.executable, str(ROOT / "tools" / "microbench.py")], check=True,
                   env=dict(os.environ, MB_OUT=str(tj)), timeout=600)
    timing = json.loads(tj.read_text())
    fetch = pmc_pass("FETCH_SIZE", out)
    write = pmc_pass("WRITE_SIZE", out)
    res = {"what": __doc__.split("\n\n")[0], "kernels": {}}
    n = 1 << 20
    for v in ("stream_read", "stream_copy", "parse", "parse_rec8"):
        traffic = fetch[v] * 1024 * 2 + write[v] * 1024
        row = {"pmc_fetch_bytes": fetch[v] * 1024 * 2, "pmc_write_bytes": write[v] * 1024,
               "pmc_traffic_bytes": traffic}
        for ns in (1, 2):
            us = timing[f"{v}_s{ns}"]["us_min"]
            row[f"us_per_launch_s{ns}"] = us
            row[f"hbm_TBps_by_pmc_s{ns}"] = round(traffic / us / 1e6, 3)
            row[f"read_TBps_by_pmc_s{ns}"] = round(fetch[v] * 2048 / us / 1e6, 3)
            row[f"Gpkt_s_s{ns}"] = round(n / us / 1e3, 2)
        res["kernels"][v] = row
    rd = res["kernels"]["stream_read"]["hbm_TBps_by_pmc_s2"]
    res["conclusion"] = (
        f"the read-only stream sustains {rd} TB/s; a launch that also writes 16-B records "
        "moves 80 B per packet at about the same total rate, so its read share is at most "
        f"{rd} x 64/80 / 8 = {rd * 0.8 / 8:.3f} of the 8 TB/s peak")
    dst = ROOT / "profiles" / f"{args.tag}_c2_ceiling.json"
    dst.write_text(json.dumps(res, indent=1) + "\n")
    (out / dst.name).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
