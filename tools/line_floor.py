#!/usr/bin/env python3
"""Measurement tool: the 128-B line floor of a record-mode parse.

For the frames of a bench config (device-generated, parsed on the device for
their layer offsets), lists the frame bytes the record walk must read —
ethertype and VLAN tags' ethertypes, IPv4 ihl / protocol, the IPv6 next
header, every extension header's next_header / length bytes, TCP's data
offset (UDP and ICMP need only the frame length) — and the 16-B chunks the
kernel stages (W chunks from the one holding byte 12), and counts the
distinct 128-B lines they touch per 64-frame tile (one wave's frames: a line
two of them share is fetched once).  Descriptors (u64 offset + u16 length)
and the 16-B record add 10 + 16 B per frame.  The result is what a kernel
that fetches every touched line exactly once moves, to compare with the PMC
traffic per frame in profiles/<tag>_pmc_<config>.json.

    python tools/line_floor.py --config c4 [--frames 2097152] > out.json
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402

FRAG, HOP, DST, RT, MOB, HIP, SHIM, EXP1, EXP2 = 44, 0, 60, 43, 135, 139, 140, 253, 254
RFC6564 = (HOP, DST, RT, MOB, HIP, SHIM, EXP1, EXP2)


def needed_positions(buf, base, off, lens, rec, chain, flows=False):
    """Frame-relative positions the record walk reads, as a list of
    (positions, valid) arrays (absolute arena offsets)."""
    out = []
    n = len(off)
    l3 = rec["l3_off"].astype(np.int64)
    l4 = rec["l4_off"].astype(np.int64)
    l3k = rec["l3_kind"]
    l4k = rec["l4_kind"]
    nv = rec["n_vlan"].astype(np.int64)
    ne = rec["n_v6ext"].astype(np.int64)
    ok_len = lens.astype(np.int64)

    def add(rel, valid):
        rel = np.asarray(rel, dtype=np.int64)
        valid = valid & (rel < ok_len) & (rel >= 0)
        out.append((off + rel, valid))

    every = np.ones(n, bool)
    add(np.full(n, 12), every)
    add(np.full(n, 13), every)
    for j in range(2):
        has = nv > j
        add(14 + 4 * j + 2, has)
        add(14 + 4 * j + 3, has)
    v4 = l3k == 1
    v6 = l3k == 2
    add(l3, v4)
    add(l3 + 9, v4)
    add(l3 + 6, v6)
    # extension headers: walk them on the host from the frame bytes
    pos = l3 + 40
    nh = np.where(v6, buf[np.minimum(off + l3 + 6, len(buf) - 1)], 0).astype(np.int64)
    for k in range(int(ne.max()) if n else 0):
        has = ne > k
        add(pos, has)
        add(pos + 1, has)
        ab = np.minimum(off + pos, len(buf) - 2)
        nxt = buf[ab].astype(np.int64)
        ext = buf[ab + 1].astype(np.int64)
        ln = np.where(nh == FRAG, 8, (ext + 1) * 8)
        pos = np.where(has, pos + ln, pos)
        nh = np.where(has, nxt, nh)
    add(l4 + 12, l4k == 1)
    if flows:  # the 5-tuple the flow hash reads (addresses, then ports)
        for k in range(12, 20):
            add(l3 + k, v4)
        for k in range(8, 40):
            add(l3 + k, v6)
        for k in range(4):
            add(l4 + k, (l4k == 1) | (l4k == 2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--frames", type=int, default=1 << 21)
    ap.add_argument("--windows", default="2,3,5,8")
    ap.add_argument("--flows", action="store_true",
                    help="add the 5-tuple bytes (flow mode) and line-completing 4-5 chunk windows")
    args = ap.parse_args()
    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    prof, n, stride, chain_name, _ = bench.CONFIGS[args.config]
    if stride is not None or chain_name == "GeneveOverV6Tunnel":
        raise SystemExit("offset-addressed, non-tunnel configs only")
    chain = Chain[chain_name]
    m = min(n, args.frames)
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], m)
    ctx = ingot_amd.Context(0)
    recs = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, chain))
    torch.cuda.synchronize()
    base = arena.data_ptr() % 4096
    off_h = off.cpu().numpy().astype(np.int64)
    len_h = lens.cpu().numpy().astype(np.int64)
    buf = arena.cpu().numpy()
    tile = np.arange(m, dtype=np.int64) // 64

    def lines(groups):
        keys = []
        for pos, valid in groups:
            ln = (base + pos[valid]) >> 7
            keys.append((tile[valid] << 36) | ln)
        k = np.unique(np.concatenate(keys))
        per_tile = len(k) / m
        glob = len(np.unique(k & ((1 << 36) - 1))) / m
        return per_tile, glob

    need = needed_positions(buf, base, off_h, len_h, recs, chain, args.flows)
    res = {"config": args.config, "frames": m, "arena_base_mod_4096": int(base),
           "ok_fraction": float((recs["status"] == 0).mean())}
    lt, lg = lines(need)
    res["needed_only"] = {"lines_per_frame_tile": round(lt, 4), "lines_per_frame_global": round(lg, 4),
                          "read_bytes_per_frame": round(lt * 128 + 10, 2)}
    for w in [int(x) for x in args.windows.split(",")]:
        skip = 12  # record modes stage from the chunk holding byte 12
        a0 = ((base + off_h + skip) & ~15) - base  # arena offset of the first staged chunk
        groups = list(need)
        for c in range(w):
            cs = a0 + 16 * c
            groups.append((cs, cs < off_h + len_h))
        lt, lg = lines(groups)
        res[f"needed_plus_window{w}"] = {"lines_per_frame_tile": round(lt, 4),
                                         "lines_per_frame_global": round(lg, 4),
                                         "read_bytes_per_frame": round(lt * 128 + 10, 2)}
    # line-completing windows: from byte 12's chunk, at least m chunks, then
    # to the end of that line, at most k (INGOT_TUNE_WINDOW_INDEXED 1000+10m+k)
    for m_, k_ in ((2, 5), (4, 5)):
        a0 = ((base + off_h + 12) & ~15) - base
        lp = ((base + a0) >> 4) & 7
        want = np.minimum(((lp + m_ + 7) & ~7) - lp, k_)
        groups = list(need)
        for c in range(k_):
            cs = a0 + 16 * c
            groups.append((cs, (c < want) & (cs < off_h + len_h)))
        lt, lg = lines(groups)
        res[f"needed_plus_linewin{m_}_{k_}"] = {"lines_per_frame_tile": round(lt, 4),
                                              "read_bytes_per_frame": round(lt * 128 + 10, 2)}
    pmc = [ROOT / "history" / "profiles" / f"r02_pmc_{args.config}.json"]
    if pmc[-1].exists():
        p = json.loads(pmc[-1].read_text())
        res["pmc"] = {"file": pmc[-1].name, "kernel": p.get("kernel"),
                      "read_bytes_per_frame": round(p["fetch_bytes_corrected"] / p["frames_per_launch"], 2),
                      "write_bytes_per_frame": round(p["write_bytes"] / p["frames_per_launch"], 2)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
