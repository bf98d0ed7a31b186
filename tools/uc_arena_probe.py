#!/usr/bin/env python3
"""Probe: does an arena in uncached / fine-grained device memory cut the
line over-fetch of the gather configs?

In default (coarse-grained) device memory the L2 fills whole 128-B lines, so a
C3 header touching 1.375 lines costs 176 B/frame of HBM reads.
Memory allocated with hipExtMallocWithFlags(hipDeviceMallocUncached /
hipDeviceMallocFinegrained) is mapped with another MTYPE; if the L2 then
passes the accesses through at their own size, the gather moves fewer bytes.
This times ctx.parse's kernel on the same frames in the three kinds of memory
(records compared byte for byte), median of interleaved rounds.  C2 (64-B
slots, the slot-ring kernel) rotates 8 copies of its arena per kind.

    python tools/uc_arena_probe.py [--configs c3,c4] [--reps 10] [--rounds 3] [--out F]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

CONFIGS = {"c2": ("V4UDP64", 1 << 20, "UdpParser"),  # 64-B slots, 8 rotated copies
           "c3": ("MIXED", 1 << 24, "GenericUlp"), "c4": ("VLAN_V6EH", 1 << 23, "VlanUlp"),
           "c6": ("GENEVE", 1 << 23, "GeneveOverV6Tunnel")}
KINDS = {"coarse": None, "finegrained": 0x1, "uncached": 0x3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import ingot_amd
    from ingot_amd import Chain, GenProfile, _lib

    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                          ctypes.c_uint]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    ctx = ingot_amd.Context(0)
    lib = _lib.load()
    s = torch.cuda.current_stream()
    out = {"what": __doc__.split("\n\n")[0], "configs": {}}
    for name in args.configs.split(","):
        prof, n, chain = CONFIGS[name]
        chain = Chain[chain]
        stride = 64 if name == "c2" else None
        copies = 8 if name == "c2" else 1  # C2: 512 MiB of arenas, past the Infinity Cache
        arena, off, lens = ingot_amd.gen_frames(GenProfile[prof], n, stride=stride)
        want = (ctx.parse_strided(arena, stride, n, chain) if stride
                else ctx.parse(arena, off, lens, chain))
        torch.cuda.synchronize()
        nbytes = arena.numel()
        ptrs = {}
        owned = []
        for kind, flags in KINDS.items():
            ptrs[kind] = []
            for _ in range(copies):
                if flags is None:
                    t = torch.empty_like(arena)
                    t.copy_(arena)
                    owned.append(t)
                    ptrs[kind].append(t.data_ptr())
                    continue
                p = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
                assert rc == 0 and p.value, (kind, rc)
                assert hip.hipMemcpy(p, arena.data_ptr(), nbytes, 3) == 0
                ptrs[kind].append(p.value)
                owned.append(p)
        if copies == 1:  # the generator's own arena beside its copies
            ptrs["generated"] = [arena.data_ptr()]
        torch.cuda.synchronize()
        recs = torch.empty_like(want)
        k = [0]

        def launch(ps):
            ptr = ps[k[0] % len(ps)]
            k[0] += 1
            if stride:
                rc = lib.ingot_gpu_parse_strided(ctx._h, ptr, stride, None, n, int(chain),
                                                 recs.data_ptr(), s.cuda_stream)
            else:
                rc = lib.ingot_gpu_parse(ctx._h, ptr, off.data_ptr(), lens.data_ptr(), n,
                                         int(chain), recs.data_ptr(), s.cuda_stream)
            assert rc == 0, rc

        res = {k: [] for k in ptrs}
        exact = {}
        for kind, ps in ptrs.items():  # parity (every copy) + warm-up
            ok = True
            for _ in ps:
                recs.zero_()
                launch(ps)
                torch.cuda.synchronize()
                ok = ok and bool(torch.equal(recs, want))
            exact[kind] = ok
        for _ in range(args.rounds):
            for kind, ptr in ptrs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(args.reps):
                    launch(ptr)
                e1.record(s)
                torch.cuda.synchronize()
                res[kind].append(e0.elapsed_time(e1) * 1e3 / args.reps)
        med = {k: round(statistics.median(v), 1) for k, v in res.items()}
        out["configs"][name] = {"frames": n, "chain": chain.name, "arena_bytes": nbytes,
                                "us_per_launch_median": med,
                                "rounds": {k: [round(x, 1) for x in v] for k, v in res.items()},
                                "records_bit_exact": exact,
                                "vs_coarse": {k: round(v / med["coarse"], 3)
                                              for k, v in med.items()}}
        print(name, json.dumps(out["configs"][name]), flush=True)
        for p in owned:
            if isinstance(p, ctypes.c_void_p):
                hip.hipFree(p)
        del arena, off, lens, want, recs
        torch.cuda.empty_cache()
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
