#!/usr/bin/env python3
"""Measurement tool: the host-inclusive rate.  The path starts and ends in host
memory (a NIC/loopback ring): pinned host arena -> hipMemcpyAsync H2D ->
parse -> records D2H into pinned host memory.  Steps are pipelined over S
streams (copy of batch k+1 overlaps the parse of batch k).  Reported in
DESIGN.md; never the bench `value` (which is device-resident).

    python tools/hostpath.py [--config c2|c3] [--streams 3] [--steps 200] [--zero-copy]

--zero-copy: no copies at all.  The arena, its descriptors and the records
stay in pinned host memory mapped for the device (ingot_gpu_host_map); the
kernels read only the header bytes they touch across PCIe and write records
straight back.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def measure(torch, ingot_amd, ctx, arena, off, lens, stride, chain, n, streams=3, steps=200,
            zero_copy=False, rec8=False):
    """Host-inclusive rate of one batch shape (frames from the device arena
    `arena`, first n): returns the result dict.  Also used live by bench.py
    (its `host_inclusive` object)."""
    S = streams
    strm = [torch.cuda.Stream() for _ in range(S)]
    R = S + 1
    nbytes = arena.numel() if off is None else int(off[n - 1].item()) + int(lens[n - 1].item())
    if stride:
        nbytes = n * stride
    src = arena[:nbytes]
    if off is not None:
        off, lens = off[:n], lens[:n]
    elif lens is not None:
        lens = lens[:n]
    host_arena = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(R)]
    for h in host_arena:
        h.copy_(src)
    host_recs = [torch.empty((n, 16), dtype=torch.uint8, pin_memory=True) for _ in range(R)]
    dev_arena = [torch.empty(nbytes, dtype=torch.uint8, device=arena.device) for _ in range(S)]
    dev_recs = [torch.empty((n, 16), dtype=torch.uint8, device=arena.device) for _ in range(S)]
    # descriptors travel with the frames: 10 B/pkt (u64 off + u16 len) for
    # packed frames, 2 B/pkt (u16 len) for slots with a length table
    desc_bytes = (2 * n if lens is not None else 0) if stride else n * 10
    host_slot_lens = None
    if stride and lens is not None:
        host_slot_lens = torch.empty(n, dtype=torch.uint16, pin_memory=True)
        host_slot_lens.copy_(lens)
        dev_slot_lens = [torch.empty_like(lens) for _ in range(S)]
    host_desc = None
    if off is not None:
        host_desc = (torch.empty(n, dtype=torch.int64, pin_memory=True),
                     torch.empty(n, dtype=torch.uint16, pin_memory=True))
        host_desc[0].copy_(off)
        host_desc[1].copy_(lens)
        dev_desc = [(torch.empty_like(off), torch.empty_like(lens)) for _ in range(S)]

    lib = ingot_amd.load_library()
    if zero_copy:
        d_arena = [ctx.host_map(h) for h in host_arena]
        d_recs = [ctx.host_map(h) for h in host_recs]
        d_off = ctx.host_map(host_desc[0]) if host_desc is not None else None
        d_len = ctx.host_map(host_desc[1]) if host_desc is not None else None
        d_slot_lens = ctx.host_map(host_slot_lens) if host_slot_lens is not None else None

    def step_zc(k):
        s = strm[k % S].cuda_stream
        if host_desc is not None:
            fn = lib.ingot_gpu_parse_compact if rec8 else lib.ingot_gpu_parse
            rc = fn(ctx._h, d_arena[k % R], d_off, d_len, n, int(chain), d_recs[k % R], s)
        else:
            fn = lib.ingot_gpu_parse_strided_compact if rec8 else lib.ingot_gpu_parse_strided
            rc = fn(ctx._h, d_arena[k % R], stride, d_slot_lens, n, int(chain), d_recs[k % R], s)
        assert rc == 0

    def step(k):
        if zero_copy:
            return step_zc(k)
        s = strm[k % S]
        with torch.cuda.stream(s):
            dev_arena[k % S].copy_(host_arena[k % R], non_blocking=True)
            if host_desc is not None:
                o, ln = dev_desc[k % S]
                o.copy_(host_desc[0], non_blocking=True)
                ln.copy_(host_desc[1], non_blocking=True)
                ctx.parse(dev_arena[k % S], o, ln, chain, out=dev_recs[k % S], stream=s)
            else:
                sl = None
                if host_slot_lens is not None:
                    sl = dev_slot_lens[k % S]
                    sl.copy_(host_slot_lens, non_blocking=True)
                ctx.parse_strided(dev_arena[k % S], stride, n, chain, lens=sl,
                                  out=dev_recs[k % S], stream=s)
            host_recs[k % R].copy_(dev_recs[k % S], non_blocking=True)

    for k in range(2 * S):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if zero_copy:
        for h in host_arena + host_recs + [x for x in (host_desc or ()) ] + \
                ([host_slot_lens] if host_slot_lens is not None else []):
            ctx.host_unmap(h)
    h2d = nbytes + desc_bytes
    d2h = n * (8 if rec8 else 16)
    res = {
        "mode": "zero-copy" if zero_copy else "memcpy",
        "record_bytes": 8 if rec8 else 16,
        "frames_per_batch": n, "streams": S, "steps": steps,
        "host_inclusive_Mpkt_s": round(n * steps / dt / 1e6, 1),
        "ms_per_batch": round(dt / steps * 1e3, 4),
        "bytes_h2d_per_batch": h2d, "bytes_d2h_per_batch": d2h,
        "pcie_GBps_effective": round((h2d + d2h) * steps / dt / 1e9, 2),
    }
    if zero_copy:
        res["note"] = ("zero-copy: nothing is copied; bytes_h2d/pcie_GBps_effective count what "
                       "the memcpy path would move for the same batch")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--zero-copy", action="store_true")
    ap.add_argument("--win", type=int, default=0, help="staged window (INGOT_TUNE_WINDOW_*)")
    ap.add_argument("--rec8", action="store_true", help="8-B records (zero-copy mode)")
    args = ap.parse_args()

    import torch

    import bench
    import ingot_amd
    from ingot_amd import Chain, GenProfile

    prof, _, stride, chain_name, _ = bench.CONFIGS[args.config]
    n = args.frames
    chain = Chain[chain_name]
    ctx = ingot_amd.Context(0)
    if args.win:
        from ingot_amd.abi import TUNE_WINDOW_INDEXED, TUNE_WINDOW_STRIDED
        ctx.set_tuning(TUNE_WINDOW_STRIDED if stride else TUNE_WINDOW_INDEXED, args.win)
    arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, stride=stride)
    res = measure(torch, ingot_amd, ctx, arena, off, lens, stride, chain, n, args.streams,
                  args.steps, args.zero_copy, args.rec8)
    res.update(config=args.config, window=args.win or "default")
    print(json.dumps(res))
    tag = ("_zc" if args.zero_copy else "") + ("_rec8" if args.rec8 else "")
    out = ROOT / "gpurun_out" / f"hostpath_{args.config}{tag}.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
