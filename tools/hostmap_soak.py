#!/usr/bin/env python3
"""Soak of the host-mapping API (ingot_gpu_host_map / _unmap) in one process,
the state round 5's fault followed: many map / parse / unmap / free cycles of
pageable buffers (some pairs sharing a page, some mapped twice or by a
sub-range), torch-pinned (hipHostMalloc) buffers mapped and unmapped, and
pageable D2H copies of assorted sizes between them.  Every parse result and
every copy is checked; the run stops at the first mismatch.

    python tools/hostmap_soak.py [--iters 300] [--seed 1]
-> one JSON line (also gpurun_out/hostmap_soak.json)
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
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    lib = ingot_amd.load_library()
    ctx = ingot_amd.Context(0)
    rng = np.random.default_rng(args.seed)
    n = 8192
    arena, off, lens = ingot_amd.gen_frames(GenProfile.MIXED, n, seed=args.seed)
    want = ctx.parse(arena, off, lens, Chain.GenericUlp).cpu().numpy()
    a_np = arena.cpu().numpy()
    nbytes = a_np.nbytes
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    counts = {"pageable_maps": 0, "shared_page_pairs": 0, "double_maps": 0, "pinned_maps": 0,
              "d2h_copies": 0, "parses": 0}
    t0 = time.time()
    bad = None

    def parse(d_arena, d_out):
        rc = lib.ingot_gpu_parse(ctx._h, d_arena, off.data_ptr(), lens.data_ptr(), n,
                                 int(Chain.GenericUlp), d_out, None)
        torch.cuda.synchronize()
        counts["parses"] += 1
        return rc

    for it in range(args.iters):
        kind = it % 4
        if kind == 0:  # pageable frames, records in the page right after
            raw = np.zeros(nbytes + n * 16 + 4 * 4096, np.uint8)
            s = int(rng.integers(0, 4096)) // 16 * 16
            fr = raw[s:s + nbytes]
            fr[:] = a_np
            r0 = s + (nbytes + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
            rec = raw[r0:r0 + n * 16]
            d_f, d_r = ctx.host_map(fr), ctx.host_map(rec)
            counts["pageable_maps"] += 2
            counts["shared_page_pairs"] += int((fr.ctypes.data + nbytes - 1) // 4096 ==
                                                rec.ctypes.data // 4096)
            rec[:] = 0xEE
            if parse(d_f, d_r) != 0 or rec.tobytes() != want.tobytes():
                bad = f"iter {it}: pageable pair"
            ctx.host_unmap(rec)
            ctx.host_unmap(fr)
            del raw, fr, rec
        elif kind == 1:  # one buffer mapped twice and by a sub-range
            raw = np.empty(nbytes + 4096, np.uint8)
            fr = raw[:nbytes]
            fr[:] = a_np
            d1 = ctx.host_map(fr)
            d2 = ctx.host_map(fr[4096:])
            counts["double_maps"] += 1
            ctx.host_unmap(fr)  # d2's mapping keeps the registration
            out.fill_(0)
            if d2 != d1 + 4096 or parse(d1, out.data_ptr()) != 0 or \
                    out.cpu().numpy().tobytes() != want.tobytes():
                bad = f"iter {it}: double map"
            ctx.host_unmap(fr[4096:])
            del raw, fr
        elif kind == 2:  # hipHostMalloc (torch pinned): map / unmap never unregisters
            h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            h.copy_(arena)
            d = ctx.host_map(h)
            counts["pinned_maps"] += 1
            ctx.host_unmap(h)
            d = ctx.host_map(h)
            out.fill_(0)
            if parse(d, out.data_ptr()) != 0 or out.cpu().numpy().tobytes() != want.tobytes():
                bad = f"iter {it}: pinned"
            ctx.host_unmap(h)
            back = torch.empty_like(arena)
            back.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            if not torch.equal(back, arena):
                bad = f"iter {it}: pinned copy back"
            del h, back
        else:  # pageable D2H copies of assorted sizes (1.6 MB records, arenas)
            for sz in (int(rng.integers(1, 64)) << 16, 1_600_000, nbytes):
                dev = torch.randint(0, 255, (sz,), dtype=torch.uint8, device="cuda")
                chk = int(dev[:: max(1, sz // 997)].to(torch.int64).sum().item())
                host = dev.cpu().numpy()
                counts["d2h_copies"] += 1
                if int(host[:: max(1, sz // 997)].astype(np.int64).sum()) != chk:
                    bad = f"iter {it}: D2H copy of {sz} B"
                del dev, host
        if bad:
            break
    torch.cuda.synchronize()
    res = {"iters": it + 1, "wall_s": round(time.time() - t0, 1), "counts": counts,
           "first_failure": bad, "ok": bad is None}
    print(json.dumps(res))
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "hostmap_soak.json").write_text(json.dumps(res, indent=1))
    sys.exit(0 if bad is None else 1)


if __name__ == "__main__":
    main()
