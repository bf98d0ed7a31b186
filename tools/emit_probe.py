#!/usr/bin/env python3
"""Measurement tool: the batched Emit kernels against the copy ceiling.

On 8,388,608 generator frames (MIXED, 64-1500 B; BASELINE C4's per-GPU count)
encapsulated as OPTE's outbound path does (outer Ethernet / IPv6 / UDP /
Geneve + one option = 74 B, lengths filled in per packet, a per-packet
flow-entropy UDP source port and VNI), times with HIP events (median of
interleaved rounds):

  packets   ingot_gpu_emit_packets into a packed destination arena;
  headers   ingot_gpu_emit_headers into 80-B slots (two-chunk packets);
  copy      torch's device-to-device copy of the same source bytes (the
            plain-copy ceiling for the packets' payload bytes);

and reports algorithmic GB/s: packets = read sum(len) + 24 B/packet of
descriptors and set values, write sum(74 + len); headers = read 8 B/packet
(len + values), write 74 B/packet.

    python tools/emit_probe.py [--frames N] [--reps 10] [--rounds 3] [--out F]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 23)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--hdr-strides", default="",
                    help="also time header blocks into slots of these strides (comma list)")
    ap.add_argument("--hdr-pad", type=int, default=0,
                    help="header blocks: also time the block zero-padded by this many bytes "
                         "(a slot whose padding is the caller's to overwrite)")
    ap.add_argument("--only", default="", help="time only these runs (comma list)")
    ap.add_argument("--lib", default=None, help="tools/variants/<name>/libingot_gpu.so instead")
    args = ap.parse_args()
    if args.lib:
        from ingot_amd import _lib as L

        L.LIB_PATH = ROOT / "tools" / "variants" / args.lib / "libingot_gpu.so"

    import numpy as np
    import torch

    import ingot_amd
    from ingot_amd import EmitSource, Field, GenProfile
    from ingot_amd import emit as E

    ctx = ingot_amd.Context(0)
    n = args.frames
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n)
    hdr = (E.ethernet(bytes(6), bytes(6), 0x86DD) + E.ipv6(bytes(16), bytes(16), 17, hop_limit=64)
           + E.udp(0, 6081) + E.geneve(0, options=E.geneve_opt(0x0129, 0)))
    H = len(hdr)
    g = torch.Generator(device="cuda").manual_seed(1)
    ports = torch.randint(0, 1 << 15, (n,), dtype=torch.int16, device="cuda", generator=g)
    vnis = torch.randint(0, 1 << 24, (n,), dtype=torch.int32, device="cuda", generator=g)
    sets = [(14, Field.V6_PAYLOAD_LEN, EmitSource.LENGTH, -40),
            (54, Field.UDP_LENGTH, EmitSource.LENGTH, 0),
            (54, Field.UDP_SOURCE, EmitSource.U16, 0, ports),
            (62, Field.GENEVE_VNI, EmitSource.U32, 0, vnis)]
    ln = lens.to(torch.int64)
    dst_off = torch.cumsum(ln + H, 0) - (ln + H)
    total = int((ln + H).sum().item())
    payload = int(ln.sum().item())
    dst = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    stride = (H + 15) // 16 * 16
    slots = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    copy_dst = torch.empty(payload, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()

    runs = {
        "packets": lambda: ctx.emit_packets(hdr, sets, arena, off, lens, dst, dst_off),
        "headers": lambda: ctx.emit_header_blocks(hdr, sets, lens, slots, stride=stride),
        "copy": lambda: copy_dst.copy_(arena[:payload]),
    }
    algo = {"packets": payload + 24 * n + total, "headers": 8 * n + H * n, "copy": 2 * payload}
    if args.hdr_pad:
        hp = hdr + bytes(args.hdr_pad)
        stp = (len(hp) + 15) // 16 * 16
        slp = torch.empty(n * stp + 64, dtype=torch.uint8, device="cuda")
        runs[f"headers_padded{len(hp)}_stride{stp}"] = (
            lambda: ctx.emit_header_blocks(hp, sets, lens, slp, stride=stp))
        algo[f"headers_padded{len(hp)}_stride{stp}"] = 8 * n + H * n
    for st in [int(x) for x in args.hdr_strides.split(",") if x]:
        sl = torch.empty(n * st + 64, dtype=torch.uint8, device="cuda")
        runs[f"headers_stride{st}"] = (lambda sl=sl, st=st:
                                       ctx.emit_header_blocks(hdr, sets, lens, sl, stride=st))
        algo[f"headers_stride{st}"] = 8 * n + H * n
    if args.only:
        runs = {k: f for k, f in runs.items() if k in args.only.split(",")}
    for f in runs.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in runs}
    for _ in range(args.rounds):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                f()
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    # position-weighted checksum of the emitted packets (variants must agree)
    csum = None
    if "packets" in runs:
        csum, step = 0, 1 << 27
        for a0 in range(0, total, step):
            b0 = min(total, a0 + step)
            w = torch.arange(a0, b0, device="cuda", dtype=torch.int64) % 65521 + 1
            csum += int((dst[a0:b0].to(torch.int64) * w).sum().item())
    out = {"what": __doc__.split("\n\n")[0], "lib": args.lib or "in-tree", "frames": n,
           "packets_checksum": csum,
           "hdr_len": H,
           "payload_bytes": payload, "emitted_bytes": total, "runs": {}}
    for k, v in res.items():
        us = statistics.median(v)
        out["runs"][k] = {"us": round(us, 1), "rounds": [round(x, 1) for x in v],
                          "algorithmic_bytes": algo[k],
                          "GB_s": round(algo[k] / us / 1e3, 1),
                          "frac_of_8TBs": round(algo[k] / us / 1e3 / 8000, 3),
                          "Mpkt_s": round(n / us, 1) if k != "copy" else None}
    print(json.dumps(out), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
