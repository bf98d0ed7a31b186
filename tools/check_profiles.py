#!/usr/bin/env python3
"""Tie every bench line's roofline to the committed rocprofv3 evidence.

For each config: the bench line (gpurun_out/bench_<cfg>.log, from
tools/profile_round.sh), the kernel-trace stats of a single-stream run of
the same config (profiles/<tag>_<cfg>_streams1_kernel_stats.csv) and the PMC
traffic file (profiles/<tag>_pmc_<cfg>.json).  Recomputes

    frac_profile = algorithmic bytes per launch / mean duration of the
                   step's kernels in the profile / 8 TB/s

(the step's kernels: the dominant one, plus the offset-scan kernels of the
lengths-only layout, whose launch bench.py times as one call) and checks it
against the `roofline.frac` of the profiled run's own line (<= 2 % apart;
gpurun_out/prof_<cfg>.log, single stream, the same process as the summary),
the headline line's frac against that one (<= 6 %: kernel tracing slows the
launches by 1.5-5 %), that the line attached the
PMC file of its own kernel, and that the PMC kernel is the profile's
dominant kernel.  Writes profiles/<tag>_bench_all_configs.json.

    python tools/check_profiles.py --tag r02 [--logs gpurun_out]
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CONFIGS = "c2 c2m c2r c3 c3p c3r c3s c4 c5 c6 c6e".split()
# kernels launched by one timed call besides the dominant one
EXTRA = {"c3p": ("k_tile_sums", "k_group_scan")}


def line_of(path: Path):
    lines = [x for x in path.read_text().splitlines() if x.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--logs", default=str(ROOT / "gpurun_out"))
    ap.add_argument("--configs", default=None,
                    help="comma list: check only these and merge them into the tag's existing "
                         "<tag>_bench_all_configs.json")
    args = ap.parse_args()
    out, bad = {}, []
    dst = ROOT / "profiles" / f"{args.tag}_bench_all_configs.json"
    only = args.configs.split(",") if args.configs else None
    if only and dst.exists():
        prev = json.loads(dst.read_text())
        out = {k: v for k, v in prev["configs"].items() if k not in only}
        bad = [b for b in prev["checks_failed"] if b.split(":")[0] not in only]
    for cfg in (only or CONFIGS):
        lp = Path(args.logs) / f"bench_{cfg}.log"
        sp = ROOT / "profiles" / f"{args.tag}_{cfg}_streams1_kernel_stats.csv"
        pp = ROOT / "profiles" / f"{args.tag}_pmc_{cfg}.json"
        if not (lp.exists() and sp.exists()):
            bad.append(f"{cfg}: missing {lp if not lp.exists() else sp}")
            continue
        line = line_of(lp)
        # the profiled run's own line (same process as the kernel-trace
        # summary); the headline line (default streams) is reported beside it
        pl = Path(args.logs) / f"prof_{cfg}.log"
        prof_line = line_of(pl) if pl.exists() else None
        if prof_line is None:
            bad.append(f"{cfg}: no line from the profiled run ({pl})")
            prof_line = line
        rows = list(csv.DictReader(open(sp)))
        parse = [r for r in rows if any(k in r["Name"] for k in ("k_parse", "k_modify", "k_flows",
                                                                   "k_emit"))]
        # the line names its kernel (and a C2 run's summary also holds the
        # C3 sub-line's k_parse): match it; else the most-called parse kernel
        kname = prof_line["roofline"].get("kernel") or ""
        # (the printed line names it without the "void ingot_gpu::(anon)::"
        # prefix and the argument list)
        named = [r for r in parse if r["Name"] == kname] or \
            [r for r in parse if kname and "<" in kname and kname in r["Name"]]
        dom = named[0] if named else max(parse, key=lambda r: int(r["Calls"]))
        mean_us = float(dom["AverageNs"]) / 1e3
        for extra in EXTRA.get(cfg, ()):
            mean_us += sum(float(r["AverageNs"]) / 1e3 for r in rows if extra in r["Name"])
        rl = line["roofline"]
        pr = prof_line["roofline"]
        # (lines printed before the field joined the compact form: achieved
        # GB/s x the launch mean gives the same bytes to ~1e-5)
        alg = pr.get("algorithmic_bytes_per_launch") or \
            pr["achieved"] * pr["launch_mean_us"] * 1e3
        frac_p = alg / (mean_us * 1e-6) / 1e9 / pr["peak"]
        rec = {"value": line["value"], "ms_per_step": line["ms_per_step"],
               "frac_line": rl["frac"], "frac_profiled_run_line": pr["frac"],
               "frac_profile": round(frac_p, 4),
               "launch_mean_us_line": rl["launch_mean_us"],
               "launch_mean_us_profiled_run": pr["launch_mean_us"],
               "profile_mean_us": round(mean_us, 3), "profile_kernel": dom["Name"],
               "traffic_ratio": (rl.get("traffic_detail") or {}).get("ratio_to_algorithmic",
                                                                     rl.get("traffic_ratio")),
               "line": line, "profiled_run_line": prof_line}
        if abs(frac_p - pr["frac"]) > 0.02 * pr["frac"]:
            bad.append(f"{cfg}: profiled run's frac {pr['frac']} vs its profile {frac_p:.4f}")
        # kernel tracing itself slows single-stream launches by 1.5-5 %
        if abs(rl["frac"] - pr["frac"]) > 0.06 * pr["frac"]:
            bad.append(f"{cfg}: headline frac {rl['frac']} vs profiled run's {pr['frac']}")
        if pp.exists():
            pk = json.loads(pp.read_text()).get("kernel")
            rec["pmc_kernel"] = pk
            if pk != dom["Name"]:
                bad.append(f"{cfg}: PMC kernel {pk} is not the profile's {dom['Name']}")
            if rl.get("traffic") is None:
                bad.append(f"{cfg}: the line did not attach {pp.name}")
        else:
            bad.append(f"{cfg}: no PMC file")
        out[cfg] = rec
        print(f"{cfg:4s} value {line['value']:10.1f}  frac line {rl['frac']:.4f} profiled-run "
              f"{pr['frac']:.4f} profile {frac_p:.4f}  mean {mean_us:9.2f} us (profiled-run "
              f"line {pr['launch_mean_us']})  traffic x{rec['traffic_ratio']}")
    dst.write_text(json.dumps({"checks_failed": bad, "configs": out}, indent=1) + "\n")
    for b in bad:
        print("FAIL", b)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
