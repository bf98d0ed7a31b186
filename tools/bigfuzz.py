#!/usr/bin/env python3
"""Validation tool: a large one-off differential run, device vs oracle, beyond
the sizes the pytest suite uses.  For every chain: records and every getter
over N adversarial frames (every truncation / ihl / data_offset / EH / Geneve
defect path), in the packed layout and in 256-B slots; flow ids and hashes
for the VLAN chain.  Prints one JSON line with the mismatch counts (all must
be 0) and writes it to gpurun_out/bigfuzz.json.  Also parse_read over random
4-chunk splits (every staging plan kept, parse_read_first, lazy bounds),
flow bins from k_flows_bits and from k_parse's flows mode, and the slot ring.

    python tools/bigfuzz.py [--frames 4000000] [--seed 1234]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4_000_000)
    ap.add_argument("--seed", type=int, default=1234)
    args = ap.parse_args()

    import torch

    import ingot_amd
    import oracle
    from ingot_amd import Chain, GenProfile

    ctx = ingot_amd.Context(0)
    n, res, t0 = args.frames, {}, time.time()
    for chain in Chain:
        prof = (GenProfile.GENEVE_ADVERSARIAL if chain == Chain.GeneveOverV6Tunnel
                else GenProfile.ADVERSARIAL)
        for layout in ("packed", "slots256"):
            stride = 256 if layout == "slots256" else None
            arena, off, lens = ingot_amd.gen_frames(prof, n, seed=args.seed + int(chain),
                                                    stride=stride)
            if stride:
                recs = ctx.parse_strided(arena, stride, n, chain, lens=lens)
            else:
                recs = ctx.parse(arena, off, lens, chain)
            if chain == Chain.GeneveOverV6Tunnel:
                flds = ctx.geneve_fields(arena, off, lens, stride=stride or 0, n=n)
            else:
                flds = ctx.fields(arena, off, lens, chain, stride=stride or 0, n=n)
            torch.cuda.synchronize()
            a = arena.cpu().numpy()
            o = None if off is None else off.cpu().numpy()
            ln = None if lens is None else lens.cpu().numpy()
            w_rec = oracle.parse_batch(a, o, ln, chain, stride=stride or 0, n=n, nthreads=16)
            if chain == Chain.GeneveOverV6Tunnel:
                w_fld = oracle.geneve_fields_batch(a, o, ln, stride=stride or 0, n=n)
            else:
                _, w_fld = oracle.parse_batch(a, o, ln, chain, stride=stride or 0, n=n,
                                              fields=True, nthreads=16)
            g_rec = recs.cpu().numpy().reshape(n, -1)
            g_fld = flds.cpu().numpy().reshape(n, -1)
            bad_r = int((g_rec != w_rec.view(np.uint8).reshape(n, -1)).any(axis=1).sum())
            bad_f = int((g_fld != w_fld.view(np.uint8).reshape(n, -1)).any(axis=1).sum())
            st = g_rec[:, 0]
            res[f"{chain.name}/{layout}"] = {"record_mismatches": bad_r, "field_mismatches": bad_f,
                                            "ok_fraction": round(float((st == 0).mean()), 4)}
            print(chain.name, layout, res[f"{chain.name}/{layout}"], flush=True)
            del arena, off, lens, recs, flds
            torch.cuda.empty_cache()
    # parse_read over random chunk splits with every staging plan
    from ingot_amd.abi import TUNE_READ_PLAN

    for chain in Chain:
        prof = (GenProfile.GENEVE_ADVERSARIAL if chain == Chain.GeneveOverV6Tunnel
                else GenProfile.ADVERSARIAL)
        arena, off, lens = ingot_amd.gen_frames(prof, n, seed=args.seed + 10 + int(chain))
        a, o, ln = arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy()
        # 4 chunks per packet at 3 sorted random cuts (empty chunks included)
        rng = np.random.default_rng(args.seed + int(chain))
        cuts = np.sort(rng.integers(0, ln.astype(np.int64)[:, None] + 1, size=(n, 3)), axis=1)
        bounds = np.concatenate([np.zeros((n, 1), np.int64), cuts,
                                 ln.astype(np.int64)[:, None]], axis=1)
        seg_off = (o.astype(np.int64)[:, None] + bounds[:, :4]).reshape(-1)
        seg_len = (bounds[:, 1:] - bounds[:, :4]).reshape(-1).astype(np.uint16)
        pkt_seg = (np.arange(n + 1, dtype=np.int64) * 4).astype(np.uint32)
        w_r, _, w_ch = oracle.parse_read_batch(a, seg_off.view(np.uint64), seg_len, pkt_seg,
                                                chain, nthreads=16)
        d_so = torch.from_numpy(seg_off).cuda()
        d_sl = torch.from_numpy(seg_len.view(np.int16)).cuda()
        d_ps = torch.from_numpy(pkt_seg.view(np.int32)).cuda()
        for plan in (0, 1):
            c2 = ingot_amd.Context(0)
            c2.set_tuning(TUNE_READ_PLAN, plan)
            r, ch = c2.parse_read(arena, d_so, d_sl, d_ps, chain)
            torch.cuda.synchronize()
            bad = int((r.cpu().numpy().reshape(n, -1) != w_r.view(np.uint8).reshape(n, -1))
                      .any(axis=1).sum())
            badc = int((ch.cpu().numpy().view(np.uint16) != w_ch).sum())
            res[f"{chain.name}/parse_read_plan{plan}"] = {"record_mismatches": bad,
                                                          "chunk_mismatches": badc}
            print(chain.name, f"parse_read plan {plan}", res[f"{chain.name}/parse_read_plan{plan}"],
                  flush=True)
        # round 3/4: chunk 0 per packet (parse_read_first), bounds per tile or
        # on demand (READ_PLAN 17)
        first = ingot_amd.first_chunks(d_so, d_sl, d_ps)
        for plan in (0, 17):
            c2 = ingot_amd.Context(0)
            c2.set_tuning(TUNE_READ_PLAN, plan)
            r, ch = c2.parse_read(arena, d_so, d_sl, d_ps, chain, first=first)
            torch.cuda.synchronize()
            bad = int((r.cpu().numpy().reshape(n, -1) != w_r.view(np.uint8).reshape(n, -1))
                      .any(axis=1).sum())
            badc = int((ch.cpu().numpy().view(np.uint16) != w_ch).sum())
            key = f"{chain.name}/parse_read_first" + ("_lazy" if plan else "")
            res[key] = {"record_mismatches": bad, "chunk_mismatches": badc}
            print(chain.name, key, res[key], flush=True)
        del arena, off, lens, d_so, d_sl, d_ps, first
        torch.cuda.empty_cache()
    # flows on the VLAN chain
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=args.seed)
    flow16 = ctx.flow_hist(arena, off, lens, Chain.VlanUlp)  # no hashes: the 16-bit table
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hashes=hashes)
    torch.cuda.synchronize()
    _, w_hash = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                                 Chain.VlanUlp)
    w_flow = oracle.flow_hist.last_flows
    res["flows/VlanUlp"] = {
        "hash_mismatches": int((hashes.cpu().numpy().view(np.uint32) != w_hash).sum()),
        "flow_mismatches": int((flow.cpu().numpy().view(np.uint32) != w_flow).sum()),
        "flow16_mismatches": int((flow16.cpu().numpy().view(np.uint32) != w_flow).sum())}
    print("flows", res["flows/VlanUlp"], flush=True)
    # k_parse's flows mode (explicit windows) beside the default k_flows_bits,
    # on the FLOWS frames and on adversarial frames
    from ingot_amd.abi import TUNE_WINDOW_INDEXED

    for fk in (0, 1025, 1056):  # 0: k_flows_bits; else k_parse flows with that window
        c4 = ingot_amd.Context(0)
        c4.set_tuning(TUNE_WINDOW_INDEXED, fk)
        f4 = c4.flow_hist(arena, off, lens, Chain.VlanUlp)
        torch.cuda.synchronize()
        res[f"flows/VlanUlp/win{fk}"] = {
            "flow_mismatches": int((f4.cpu().numpy().view(np.uint32) != w_flow).sum())}
        print("flows", fk, res[f"flows/VlanUlp/win{fk}"], flush=True)
    del arena, off, lens
    torch.cuda.empty_cache()
    for chain in (Chain.GenericUlp, Chain.VlanUlp):
        arena, off, lens = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, n,
                                                seed=args.seed + 40 + int(chain))
        oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(), chain)
        w_adv = oracle.flow_hist.last_flows
        for fk in (0, 1025, 1056):
            c4 = ingot_amd.Context(0)
            c4.set_tuning(TUNE_WINDOW_INDEXED, fk)
            f4 = c4.flow_hist(arena, off, lens, chain)
            torch.cuda.synchronize()
            key = f"flows_adversarial/{chain.name}/win{fk}"
            res[key] = {"flow_mismatches": int((f4.cpu().numpy().view(np.uint32) != w_adv).sum())}
            print(key, res[key], flush=True)
        del arena, off, lens
        torch.cuda.empty_cache()
    # the C2 slot-ring kernel (64-B slots, no lengths) over adversarial
    # bytes, 16- and 8-B records
    for chain in (Chain.UdpParser, Chain.GenericUlp, Chain.VlanUlp):
        arena, _, _ = ingot_amd.gen_frames(GenProfile.ADVERSARIAL, n, seed=args.seed + 20 +
                                           int(chain), stride=64)
        w_rec = oracle.parse_batch(arena.cpu().numpy(), None, None, chain, stride=64, n=n,
                                   nthreads=16)
        g16 = ctx.parse_strided(arena, 64, n, chain)
        g8 = ctx.parse_strided_compact(arena, 64, n, chain)
        torch.cuda.synchronize()
        bad16 = int((g16.cpu().numpy().reshape(n, -1) != w_rec.view(np.uint8).reshape(n, -1))
                    .any(axis=1).sum())
        from ingot_amd.abi import rec16_to_rec8

        w8 = rec16_to_rec8(w_rec)
        r = {"record_mismatches": bad16,
             "rec8_mismatches": int((g8.cpu().numpy().reshape(n, -1) !=
                                     w8.view(np.uint8).reshape(n, -1)).any(axis=1).sum())}
        res[f"{chain.name}/ring64"] = r
        print(chain.name, "ring64", r, flush=True)
        del arena, g16, g8
        torch.cuda.empty_cache()
    # batched Emit (ingot_gpu_emit_packets / _headers): random header blocks
    # (1-256 B) with random setters over generator frames, destinations packed
    # with random gaps (the bytes between packets must stay untouched)
    from ingot_amd import EmitSource, Field

    for case in range(3):
        rng = np.random.default_rng(args.seed + 50 + case)
        prof = (GenProfile.MIXED, GenProfile.ADVERSARIAL, GenProfile.GENEVE)[case]
        arena, off, lens = ingot_amd.gen_frames(prof, n, seed=args.seed + 60 + case)
        H = int(rng.integers(1, 257))
        hdr = rng.integers(0, 256, H, dtype=np.uint8).tobytes()
        u16 = rng.integers(0, 1 << 16, n, dtype=np.uint64).astype(np.uint16)
        u32 = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        host_sets, dev_sets = [], []
        fields = [f for f in Field]
        for _ in range(int(rng.integers(0, 9))):
            f = fields[int(rng.integers(0, len(fields)))]
            at = int(rng.integers(0, max(1, H - 3)))
            src = EmitSource(int(rng.integers(0, 4)))
            add = int(rng.integers(-(1 << 31), 1 << 31))
            vals = u16 if src == EmitSource.U16 else u32 if src == EmitSource.U32 else None
            host_sets.append((at, f, src, add) + ((vals,) if vals is not None else ()))
            dev_sets.append((at, f, src, add) + (
                (torch.from_numpy(vals.view(np.int16 if vals.dtype == np.uint16 else np.int32))
                 .cuda(),) if vals is not None else ()))
        # drop setters whose field would not lie inside the header block
        keep = []
        for hs, ds in zip(host_sets, dev_sets):
            try:
                oracle.emit_batch(hdr, [hs[:4] + hs[4:5]], np.zeros(16, np.uint8), [0], [0],
                                  np.zeros(H + 16, np.uint8), [0])
                keep.append((hs, ds))
            except ValueError:
                pass
        host_sets = [k[0] for k in keep]
        dev_sets = [k[1] for k in keep]
        ln = lens.cpu().numpy()
        tot = H + ln.astype(np.int64)
        gaps = rng.integers(0, 33, n)
        dst_off = np.cumsum(np.r_[0, (tot + gaps)[:-1]]) + int(rng.integers(0, 16))
        fill = rng.integers(0, 256, int(dst_off[-1] + tot[-1] + 64), dtype=np.uint8)
        dst = torch.from_numpy(fill).cuda()
        ctx.emit_packets(hdr, dev_sets, arena, off, lens, dst,
                         torch.from_numpy(dst_off.astype(np.int64)).cuda())
        # header blocks into each frame's headroom of a second copy
        hfill = rng.integers(0, 256, int(dst_off[-1] + tot[-1] + 64), dtype=np.uint8)
        hdst = torch.from_numpy(hfill).cuda()
        ctx.emit_header_blocks(hdr, dev_sets, lens, hdst,
                               out_off=torch.from_numpy(dst_off.astype(np.int64)).cuda())
        torch.cuda.synchronize()
        want = fill.copy()
        a = arena.cpu().numpy()
        oracle.emit_batch(hdr, host_sets, a, off.cpu().numpy(), ln, want, dst_off, nthreads=16)
        hwant = hfill.copy()
        oracle.emit_batch(hdr, host_sets, None, None, ln, hwant, dst_off, copy=False, nthreads=16)
        key = f"emit/{prof.name}/H{H}/sets{len(host_sets)}"
        res[key] = {"packet_byte_mismatches": int((dst.cpu().numpy() != want).sum()),
                    "header_block_byte_mismatches": int((hdst.cpu().numpy() != hwant).sum())}
        print(key, res[key], flush=True)
        del arena, off, lens, dst, hdst
        torch.cuda.empty_cache()
    out = {"frames_per_case": n, "seed": args.seed, "wall_s": round(time.time() - t0, 1),
           "cases": res,
           "all_zero": all(v == 0 for c in res.values() for k, v in c.items() if "mismatch" in k)}
    print(json.dumps(out))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "bigfuzz.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
