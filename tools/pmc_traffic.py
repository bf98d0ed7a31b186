#!/usr/bin/env python3
"""Measure HBM traffic of the parse kernel from rocprofv3 PMC counters.

Recipe (MI355X_MICROARCH.md §HBM, §rocprofv3 PMC slots): FETCH_SIZE and
WRITE_SIZE in separate --pmc passes (they do not fit one pass); both are in
KiB; on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide
coalesced streaming read, so it is doubled.  Per-dispatch values of the
k_parse kernel are averaged and written to profiles/<tag>_pmc_<config>.json,
which bench.py reports as `roofline.traffic`.

    python tools/pmc_traffic.py --config c2 --tag r01
(run on the GPU box; it launches rocprofv3 itself, the profiled program is
python3 bench.py directly after `--`).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


SIZED = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")


def run_pass(counter: str, config: str, outdir: Path, steps: int, extra=()) -> list[float]:
    """One --pmc pass; `counter` may name several counters of one pass
    ("A B C"): then the values are {counter: [per dispatch]}."""
    many = counter.split()
    d = outdir / many[0].lower()
    d.mkdir(parents=True, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", *many, "--output-format", "csv", "-d", str(d), "-o", "run",
           "--", sys.executable, str(ROOT / "bench.py"), "--config", config, "--steps", str(steps),
           "--warmup", "2", "--streams", "1", "--no-cpu-baseline", "--no-variants", "--no-gate",
           "--no-host-path", "--no-sublines",
           *extra]
    env = dict(os.environ, TMPDIR="/tmp")
    r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=180)
    (d / "rocprof.log").write_text(r.stdout + "\n" + r.stderr)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed ({r.returncode}); see {d}/rocprof.log")
    files = glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {d}")
    vals = {c: {} for c in many}
    names = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            if not any(k in name for k in ("k_parse", "k_modify", "k_flows", "k_emit")):
                continue
            c = row.get("Counter_Name")
            if c not in vals:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals[c]))
            vals[c][key] = vals[c].get(key, 0.0) + float(row["Counter_Value"])
            names[key] = name
    # the timed launches: the most-dispatched parse kernel (the generator's
    # and the algorithmic-bytes pass's dispatches are a handful)
    count = {}
    for k in names.values():
        count[k] = count.get(k, 0) + 1
    top = max(count, key=count.get)
    KERNELS.add(top)
    out = {c: [v for k, v in vs.items() if names[k] == top] for c, vs in vals.items()}
    return out if len(many) > 1 else out[many[0]]


KERNELS: set = set()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--timing", default="launches", choices=("launches", "ring"),
                    help="ring: profile k_parse_ring launches of bench.ring_group(steps) "
                         "batches (bench.py --timing ring)")
    ap.add_argument("--tune", action="append", default=[],
                    help="bench.py --tune KEY=VALUE for a variant; its file is named "
                         "<tag>_pmc_<config>@<key>=<value>.json (never attached to a bench line)")
    args = ap.parse_args()
    extra = [x for kv in args.tune for x in ("--tune", kv)] + ["--timing", args.timing]
    suffix = ("_ring" if args.timing == "ring" else "") + "".join(f"@{kv}" for kv in args.tune)
    out = ROOT / "gpurun_out" / f"pmc_{args.config}{suffix}"
    fetch = run_pass("FETCH_SIZE", args.config, out, args.steps, extra)
    write = run_pass("WRITE_SIZE", args.config, out, args.steps, extra)
    # cross-check of the x2 correction: the L2 -> memory read requests by
    # size in a pass of their own (3 TCC counters)
    sized = run_pass(" ".join(SIZED), args.config, out, args.steps, extra)
    # the first dispatches include the generator's and the algorithmic-bytes
    # pass: keep the timed ones (all k_parse dispatches are the same launch)
    f_kib = sorted(fetch)[len(fetch) // 2]
    w_kib = sorted(write)[len(write) // 2]
    sys.path.insert(0, str(ROOT))
    import bench

    group = bench.ring_group(args.steps) if args.timing == "ring" else 1
    if len(KERNELS) != 1:
        raise RuntimeError(f"the two passes profiled different kernels: {sorted(KERNELS)}")
    res = {
        "config": args.config,
        "kernel": sorted(KERNELS)[0],
        "sources_sha": bench.kernel_sources_sha(),
        "frames_per_launch": bench.CONFIGS[args.config][1] * group,
        "batches_per_launch": group,
        "timing": args.timing,
        "dispatches": [len(fetch), len(write)],
        "FETCH_SIZE_KiB_median": f_kib,
        "WRITE_SIZE_KiB_median": w_kib,
        "fetch_bytes_corrected": f_kib * 1024 * 2,
        "write_bytes": w_kib * 1024,
        "traffic_bytes_per_launch": f_kib * 1024 * 2 + w_kib * 1024,
        "correction": "FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md:298)",
    }
    med = {c: sorted(v)[len(v) // 2] if v else 0.0 for c, v in sized.items()}
    res["read_requests_by_size"] = {"32B": med[SIZED[0]], "64B": med[SIZED[1]],
                                    "128B": med[SIZED[2]]}
    res["fetch_bytes_sized"] = 32 * med[SIZED[0]] + 64 * med[SIZED[1]] + 128 * med[SIZED[2]]
    res["sized_vs_corrected"] = (round(res["fetch_bytes_sized"] / res["fetch_bytes_corrected"], 4)
                                 if res["fetch_bytes_corrected"] else None)
    res["tune"] = args.tune
    prof = ROOT / "profiles" / f"{args.tag}_pmc_{args.config}{suffix}.json"
    prof.write_text(json.dumps(res, indent=1) + "\n")
    (ROOT / "gpurun_out" / prof.name).write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
