#!/usr/bin/env python3
"""Validation tool: a large one-off differential run, device vs oracle, beyond
the sizes the pytest suite uses.  For every chain: records and every getter
over N adversarial frames (every truncation / ihl / data_offset / EH / Geneve
defect path), in the packed layout and in 256-B slots; flow ids and hashes
for the VLAN chain.  Prints one JSON line with the mismatch counts (all must
be 0) and writes it to gpurun_out/bigfuzz.json.

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
    # flows on the VLAN chain
    arena, off, lens = ingot_amd.gen_frames(GenProfile.FLOWS, n, seed=args.seed)
    hashes = torch.zeros(n, dtype=torch.int32, device="cuda")
    flow = ctx.flow_hist(arena, off, lens, Chain.VlanUlp, hashes=hashes)
    torch.cuda.synchronize()
    _, w_hash = oracle.flow_hist(arena.cpu().numpy(), off.cpu().numpy(), lens.cpu().numpy(),
                                 Chain.VlanUlp)
    w_flow = oracle.flow_hist.last_flows
    res["flows/VlanUlp"] = {
        "hash_mismatches": int((hashes.cpu().numpy().view(np.uint32) != w_hash).sum()),
        "flow_mismatches": int((flow.cpu().numpy().view(np.uint32) != w_flow).sum())}
    print("flows", res["flows/VlanUlp"], flush=True)
    out = {"frames_per_case": n, "seed": args.seed, "wall_s": round(time.time() - t0, 1),
           "cases": res,
           "all_zero": all(v == 0 for c in res.values() for k, v in c.items() if "mismatch" in k)}
    print(json.dumps(out))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "bigfuzz.json").write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
