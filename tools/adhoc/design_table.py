#!/usr/bin/env python3
"""Regenerate DESIGN.md §5's per-config table from
profiles/<tag>_bench_all_configs.json (tools/check_profiles.py output), so
the document quotes exactly the committed lines.

    python tools/design_table.py --tag r02
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
DESC = {
    "c2": "C2 1 M × 64 B slots, UdpParser", "c2m": "C2m parse-and-decr-v4 in place",
    "c2r": "C2r C2 frames as the reference's 4-chunk `parse_read`",
    "c3": "C3 16.7 M mixed 64–1500 B packed, GenericUlp",
    "c3p": "C3p same frames, lengths only", "c3r": "C3r same frames, header + payload chunks",
    "c3s": "C3s same frames in 2048-B slots", "c4": "C4 8.4 M VLAN/QinQ + v6-EH, VlanUlp",
    "c5": "C5 C4 framing + Toeplitz + histogram",
    "c6": "C6 8.4 M Geneve-over-IPv6 (OPTE inbound)"}
NOTES = {
    "c2": "ring kernel, 2 streams", "c2m": "whole 128-B lines read and rewritten (§1c)",
    "c2r": "§1b (round 1: 31.5); dense table {dense}", "c3": "line-completing window; line-gather bound (§4)",
    "c3p": "offsets scanned on the device (§1d)", "c3r": "§1b, chunk 0 line-completing (was 2.55×); dense table {dense}",
    "c3s": "3 streams", "c4": "",
    "c5": "frac: the flows kernel; step adds count + reduce (+ all-reduce at N>1)",
    "c6": "6–9-chunk line-completing window"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    args = ap.parse_args()
    d = json.loads((ROOT / "profiles" / f"{args.tag}_bench_all_configs.json").read_text())
    rows = []
    for c in DESC:
        r = d["configs"][c]
        ln = r["line"]
        cpu = ln.get("cpu_baseline") or {}
        dn = ln["variants"].get(f"streams{ln['config']['streams']}_dense_table", {}).get("value")
        note = NOTES[c].replace("{dense}", f"{dn / 1e3:.1f}" if dn else "–")
        v = ln["value"] / 1e3
        val = f"**{v:.1f}**" if c == "c2" else f"{v:.1f}"
        rows.append(f"| {DESC[c]} | {val} | {ln['ms_per_step'] * 1e3:,.2f} | "
                    f"{ln['roofline']['frac']:.3f} | {r['traffic_ratio']:.2f}× | "
                    f"{cpu.get('value', 0):,.0f} / {cpu.get('single_core_value', 0):.1f} | "
                    f"{note} |")
    p = ROOT / "DESIGN.md"
    s = p.read_text()
    start = s.index("| C2 1 M × 64 B slots, UdpParser |")
    end = s.index("| C4 strong, 64 M frames on 1 GPU")
    p.write_text(s[:start] + "\n".join(rows) + "\n" + s[end:])
    print("\n".join(rows))


if __name__ == "__main__":
    main()
