#!/usr/bin/env python3
"""Validation tool: determinism soak of the pipelined kernels.  Thousands of
launches of the ring kernel (C2 slots, 2 streams), the flow kernels
(persistent grid with full hashes; one tile per wave with the 16-bit table,
2 streams), parse_read over the reference bench's one-chunk-per-header
shape (2 streams), the packed-layout parse and the batched emit (2 streams), each output compared on the
device with the first run's over the same arena (which the parity tests pin
to the oracle) — an intermittent race in LDS-image reuse or the persistent
grids would show up as a mismatch.  Writes gpurun_out/soak.json.

    python tools/soak.py [--iters 3000]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3000)
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    res, t0 = {}, time.time()
    s = [torch.cuda.current_stream(), torch.cuda.Stream()]

    # ring kernel: 4 arenas x 1 M x 64-B slots, steps alternating over 2 streams
    n = 1 << 20
    arenas = [ingot_amd.gen_frames(GenProfile.ADVERSARIAL if k % 2 else GenProfile.V4UDP64, n,
                                   seed=k, stride=64)[0] for k in range(4)]
    want = [ctx.parse_strided(a, 64, n, Chain.UdpParser) for a in arenas]
    outs = [torch.empty_like(w) for w in want]
    torch.cuda.synchronize()
    # mismatch counters on the device, one per stream (no host sync inside the
    # loop, so the two streams keep overlapping; outs[k] is rewritten 4 steps
    # later on the same stream, after its comparison)
    acc = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in s]
    for it in range(args.iters):
        k = it % 4
        st = s[it % 2]
        ctx.parse_strided(arenas[k], 64, n, Chain.UdpParser, out=outs[k], stream=st)
        with torch.cuda.stream(st):
            acc[it % 2] += (outs[k] != want[k]).any().to(torch.int64)
    torch.cuda.synchronize()
    bad = int(sum(a.item() for a in acc))
    res["ring_kernel_c2"] = {"launches": args.iters, "mismatching_launches": bad}
    del arenas, want, outs

    # flow kernel (persistent grid) on VLAN/v6 traffic
    m = 1 << 21
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, m, seed=3)
    h0 = torch.zeros(m, dtype=torch.int32, device="cuda")
    f0 = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hashes=h0)
    torch.cuda.synchronize()
    bad = 0
    for it in range(args.iters // 10):
        h = torch.zeros(m, dtype=torch.int32, device="cuda")
        f = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hashes=h)
        bad += int(not (torch.equal(f, f0) and torch.equal(h, h0)))
    torch.cuda.synchronize()
    res["flow_kernel"] = {"launches": args.iters // 10, "mismatching_launches": bad}

    # flow ids only (16-bit table, one tile per wave), steps over 2 streams
    g0 = ctx.flow_hist(arena, off, lens, Chain.VlanUlp)
    torch.cuda.synchronize()
    gout = [torch.empty_like(g0) for _ in range(4)]
    acc = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in s]
    for it in range(args.iters):
        k, st = it % 4, s[it % 2]
        ctx.flow_hist(arena, off, lens, Chain.VlanUlp, flow=gout[k], stream=st)
        with torch.cuda.stream(st):
            acc[it % 2] += (gout[k] != g0).any().to(torch.int64)
    torch.cuda.synchronize()
    res["flow_kernel_16bit"] = {"launches": args.iters,
                                "mismatching_launches": int(sum(a.item() for a in acc))}
    del gout

    # parse_read, one chunk per header (chunks cut from the C2 slots, staged
    # from chunk 0's window), steps over 2 streams
    import bench
    sl_arena = ingot_amd.gen_frames(GenProfile.V4UDP64, n, stride=64)[0]
    recs0 = ctx.parse_strided(sl_arena, 64, n, Chain.UdpParser)
    torch.cuda.synchronize()
    rl = torch.full((n,), 64, dtype=torch.int32, device="cuda")
    seg_off, seg_len, pkt_seg, _ = bench.read_chunks(
        torch, None, 64, rl, ingot_amd.records_to_numpy(recs0), "per_header", "cuda")
    r0, c0 = ctx.parse_read(sl_arena, seg_off, seg_len, pkt_seg, Chain.UdpParser)
    torch.cuda.synchronize()
    routs = [torch.empty_like(r0) for _ in range(4)]
    acc = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in s]
    for it in range(args.iters):
        k, st = it % 4, s[it % 2]
        ctx.parse_read(sl_arena, seg_off, seg_len, pkt_seg, Chain.UdpParser, out=routs[k],
                       stream=st)
        with torch.cuda.stream(st):
            acc[it % 2] += (routs[k] != r0).any().to(torch.int64)
    torch.cuda.synchronize()
    res["parse_read_per_header"] = {"launches": args.iters,
                                    "mismatching_launches": int(sum(a.item() for a in acc))}
    del routs, sl_arena

    # packed layout (tile scan + in-kernel prefix scan)
    want = ctx.parse(arena, off, lens, Chain.VlanUlp)
    bad = 0
    for it in range(args.iters // 10):
        got = ctx.parse_packed(arena, lens, Chain.VlanUlp)
        bad += int(not torch.equal(got, want))
    torch.cuda.synchronize()
    res["packed_layout"] = {"launches": args.iters // 10, "mismatching_launches": bad}

    # batched emit (sixteen waves sharing each 256-packet group's walk through
    # LDS), steps over 2 streams, every packet at a fresh misalignment
    import numpy as np
    hdr, sets = bench.emit_stack()
    ports, vnis = bench.emit_values(m)
    dsets = [sets[0], sets[1], (*sets[2], torch.from_numpy(ports.view(np.int16)).cuda()),
             (*sets[3], torch.from_numpy(vnis.view(np.int32)).cuda())]
    tot = lens.to(torch.int64) + len(hdr) + 3
    d_off = torch.cumsum(tot, 0) - tot
    size = int(tot.sum().item()) + 64
    # every launch writes into a buffer refilled with a sentinel first (gap
    # bytes included, which must stay untouched), so a launch that writes
    # nothing or only part of its output is a mismatch
    SENT = 0xEE
    e0 = torch.full((size,), SENT, dtype=torch.uint8, device="cuda")
    ctx.emit_packets(hdr, dsets, arena, off, lens, e0, d_off)
    torch.cuda.synchronize()
    eouts = [torch.empty(size, dtype=torch.uint8, device="cuda") for _ in range(4)]
    acc = [torch.zeros((), dtype=torch.int64, device="cuda") for _ in s]
    for it in range(args.iters // 5):
        k, st = it % 4, s[it % 2]
        with torch.cuda.stream(st):
            eouts[k].fill_(SENT)
        ctx.emit_packets(hdr, dsets, arena, off, lens, eouts[k], d_off, stream=st)
        with torch.cuda.stream(st):
            acc[it % 2] += (eouts[k] != e0).any().to(torch.int64)
    torch.cuda.synchronize()
    res["emit_packets"] = {"launches": args.iters // 5,
                           "mismatching_launches": int(sum(a.item() for a in acc))}
    del eouts, e0

    out = {"wall_s": round(time.time() - t0, 1), "checks": res,
           "all_zero": all(v["mismatching_launches"] == 0 for v in res.values())}
    print(json.dumps(out))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "soak.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
