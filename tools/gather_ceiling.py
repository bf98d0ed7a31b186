#!/usr/bin/env python3
"""Measurement tool: the sparse 128-B line-gather ceiling under the C3 / C4
parse kernels.

On the same device-generated frames as the bench configs, times (HIP events,
launches back to back on one stream, medians of interleaved rounds):

  parse   the product kernel (ctx.parse, 16-B records, the config's chain);
  stage   its staging alone (tools/gather_ceiling.hip: k_stage — the same
          line-completing LDS-DMA window, then a 4-B store per frame);
  touch   one 4-B load per distinct 128-B line of each frame's header bytes
          [12, payload_off) (k_touch), the fewest instructions that make HBM
          deliver the lines the walk needs.

and reports the distinct lines each pattern touches (host-side count from
the offsets) as lines/s and GB/s.  If `touch` is not faster than `parse`,
the parse runs at the rate at which the chip delivers those lines.

    python tools/gather_ceiling.py --build          # here: hipcc -> tools/bin/
    python tools/gather_ceiling.py [--configs c3,c4] [--reps 10] [--out F]   # GPU box
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
SRC = ROOT / "tools" / "gather_ceiling.hip"
LIB = ROOT / "tools" / "bin" / "libgather_ceiling.so"

CONFIGS = {  # name: (GenProfile, frames, Chain)
    "c3": ("MIXED", 1 << 24, "GenericUlp"),
    "c4": ("VLAN_V6EH", 1 << 23, "VlanUlp"),
    "c5": ("FLOWS", 1 << 23, "VlanUlp"),  # + the flows kernel (flow ids, histogram off)
    "c6": ("GENEVE", 1 << 23, "GeneveOverV6Tunnel"),
}


def build():
    LIB.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared",
                    "-fPIC", "-o", str(LIB), str(SRC)], check=True)
    print("built", LIB)


def lines_touched(off, start, end):
    """Distinct 128-B lines of the byte ranges [off+start, off+end) (end > start)."""
    import numpy as np

    a = (off + start) >> 7
    b = (off + end - 1) >> 7
    cnt = (b - a + 1).astype(np.int64)
    # ranges of consecutive frames may share a line: count the union
    ids = np.repeat(a, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    return int(np.unique(ids).size)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "gather_ceiling.json"))
    args = ap.parse_args()
    if args.build:
        build()
        return

    import numpy as np
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    unknown = [c for c in args.configs.split(",") if c not in CONFIGS]
    if unknown:
        raise SystemExit(f"unknown configs {unknown}; known: {sorted(CONFIGS)}")
    if not LIB.exists():
        raise SystemExit(f"{LIB} missing: run with --build first (in the build container)")
    lib = ctypes.CDLL(str(LIB))
    for f in (lib.gc_touch, lib.gc_stage):
        f.restype = ctypes.c_int
    P = ctypes.c_void_p
    ctx = ingot_amd.Context(0)
    res = {"tool": "tools/gather_ceiling.py", "reps": args.reps, "launches": args.launches,
           "configs": {}}
    for name in args.configs.split(","):
        prof, n, chain = CONFIGS[name]
        arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, seed=ingot_amd.GEN_SEED)
        ch = Chain[chain]
        rec = torch.empty((n, 16), dtype=torch.uint8, device="cuda:0")
        ctx.parse(arena, off, lens, ch, out=rec)
        torch.cuda.synchronize()
        r = ingot_amd.records_to_numpy(rec)
        off_np = off.cpu().numpy().astype(np.int64)
        len_np = lens.cpu().numpy().astype(np.int64)
        # header bytes [12, payload_off), at least 1 byte, within the frame
        end = np.clip(r["payload_off"].astype(np.int64), 13, None)
        end = np.minimum(end, len_np)
        ok = end > 12
        span = torch.from_numpy(np.where(ok, end - 12, 0).astype(np.uint16)).to("cuda:0")
        out = torch.empty(n, dtype=torch.int32, device="cuda:0")
        s = torch.cuda.current_stream().cuda_stream
        a_p, o_p, l_p, sp_p, out_p = (P(arena.data_ptr()), P(off.data_ptr()), P(lens.data_ptr()),
                                      P(span.data_ptr()), P(out.data_ptr()))

        def run_parse():
            ctx.parse(arena, off, lens, ch, out=rec)

        def run_stage():
            lib.gc_stage(a_p, o_p, l_p, ctypes.c_uint64(n), out_p, P(s))

        def run_touch():
            lib.gc_touch(a_p, o_p, l_p, ctypes.c_uint64(n), ctypes.c_uint32(12), sp_p, out_p, P(s))

        runs = {"parse": run_parse, "stage": run_stage, "touch": run_touch}
        if name == "c3":
            # c3r: the same frames as [header chunk | payload chunk] through
            # ingot_gpu_parse_read_first with chunk bounds on demand (the c3r
            # line's path): the header chunk's lines are the touch lines
            import bench
            from ingot_amd import _lib, abi

            seg_off, seg_len, pkt_seg, _ = bench.read_chunks(torch, off, None, lens, r, "split2",
                                                             "cuda:0")
            first = ingot_amd.first_chunks(seg_off, seg_len, pkt_seg)
            ctx_r = ingot_amd.Context(0)
            ctx_r.set_tuning(abi.TUNE_READ_PLAN, 17)
            L = _lib.load()
            rec_r = torch.empty((n, 16), dtype=torch.uint8, device="cuda:0")
            rargs = (ctx_r._h, arena.data_ptr(), seg_off.data_ptr(), seg_len.data_ptr(),
                     pkt_seg.data_ptr(), first.data_ptr(), n, int(ch), rec_r.data_ptr(), None)

            def run_read_first():
                L.ingot_gpu_parse_read_first(*rargs, s)

            runs["parse_read_first (c3r)"] = run_read_first
        if name == "c5":
            def run_flows():
                ctx.flow_hist(arena, off, lens, ch, flow=out)

            runs["flows"] = run_flows
        for f in runs.values():  # warm
            for _ in range(3):
                f()
        torch.cuda.synchronize()
        us = {k: [] for k in runs}
        for _ in range(args.reps):
            for k, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.launches):
                    f()
                e1.record()
                torch.cuda.synchronize()
                us[k].append(e0.elapsed_time(e1) * 1e3 / args.launches)
        # lines: touch = the header lines; stage = the staged window's lines
        lt = lines_touched(off_np[ok], 12, end[ok])
        mis = arena.data_ptr() & 31
        sh = (off_np + 12 + mis) & 15
        base = off_np + 12 - sh
        lp = ((arena.data_ptr() + base) >> 4) & 7
        want = np.minimum(((lp + 2 + 7) & ~7) - lp, 5)
        take = np.minimum(len_np, 12 + 16 * want - sh)
        nch = np.clip((take - (12 - sh) + 15) // 16, 0, None)
        st_ok = nch > 0
        ls = lines_touched(base[st_ok], 0, 16 * nch[st_ok])
        med = {k: round(statistics.median(v), 2) for k, v in us.items()}
        rep = {"frames": n, "profile": prof, "chain": chain, "median_us": med,
               "us": {k: [round(x, 2) for x in v] for k, v in us.items()},
               "lines_header": lt, "lines_staged": ls,
               "lines_per_frame": {"header": round(lt / n, 3), "staged": round(ls / n, 3)}}
        rep["G_lines_per_s"] = {"touch (header lines)": round(lt / med["touch"] / 1e3, 2),
                                "stage (window lines)": round(ls / med["stage"] / 1e3, 2),
                                "parse (header lines)": round(lt / med["parse"] / 1e3, 2)}
        rep["parse_over_touch"] = round(med["parse"] / med["touch"], 3)
        if "parse_read_first (c3r)" in med:
            rep["c3r_over_touch"] = round(med["parse_read_first (c3r)"] / med["touch"], 3)
        if "flows" in med:
            rep["flows_over_touch"] = round(med["flows"] / med["touch"], 3)
            rep["flows_over_parse"] = round(med["flows"] / med["parse"], 3)
        rep["TB_per_s_of_lines"] = {k: round(v * 128 / 1e3, 3)
                                    for k, v in rep["G_lines_per_s"].items()}
        res["configs"][name] = rep
        print(name, json.dumps({k: rep[k] for k in ("median_us", "lines_per_frame",
                                                    "G_lines_per_s")}), flush=True)
        del arena, off, lens, rec, out, span
        torch.cuda.empty_cache()
    # reference: the same touch kernel over consecutive 128-B lines (one line
    # per lane, 2 GiB), i.e. the streaming line rate
    n = 1 << 24
    buf = torch.zeros(n * 128 + 256, dtype=torch.uint8, device="cuda:0")
    off = torch.arange(n, dtype=torch.int64, device="cuda:0") * 128
    lens = torch.full((n,), 128, dtype=torch.int16, device="cuda:0")
    span = torch.full((n,), 1, dtype=torch.int16, device="cuda:0")
    out = torch.empty(n, dtype=torch.int32, device="cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    args_t = (P(buf.data_ptr()), P(off.data_ptr()), P(lens.data_ptr()), ctypes.c_uint64(n),
              ctypes.c_uint32(0), P(span.data_ptr()), P(out.data_ptr()), P(s))
    for _ in range(3):
        lib.gc_touch(*args_t)
    torch.cuda.synchronize()
    us = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.launches):
            lib.gc_touch(*args_t)
        e1.record()
        torch.cuda.synchronize()
        us.append(e0.elapsed_time(e1) * 1e3 / args.launches)
    m = statistics.median(us)
    res["streaming_lines"] = {"lines": n, "median_us": round(m, 2),
                              "G_lines_per_s": round(n / m / 1e3, 2),
                              "TB_per_s_of_lines": round(n * 128 / m / 1e6, 3)}
    print("streaming", json.dumps(res["streaming_lines"]), flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
