#!/usr/bin/env python3
"""bench.py — device-resident L2/L3/L4 parse throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c2m|c3|c3r|c3s|c4|c5|c6]
                    [--streams S] [--record 16|8]

A *step* is one launch of the parse path over one batch of synthetic frames
already resident in HBM.  At N=1 the default workload is BASELINE.json
configs[1] (C2): 1,048,576 x 64-B Eth/IPv4/UDP frames in 64-B slots, parsed as
ingot's `UdpParser`, 16-B records.  N>1 (torchrun, one rank per GPU): every
rank parses its own shard of the same size (weak scaling; packets are
independent, so there is no data-path collective).  Rank 0 prints one JSON
line.

Pipelining: consecutive batches are independent, so step k is launched on
stream k % S (default S=2, a double-buffered pipeline like a NIC-ring
consumer): the next batch's kernel ramps up while the previous one drains,
hiding the ~1.5 us dependent-launch boundary.  Every step is still exactly
one launch over one 1M-frame batch; `variants` reports S=1 and 8-B records.

To measure HBM and not the 256 MiB Infinity Cache, step k reads arena copy
k % R and writes record buffer k % R (R copies >= 512 MiB in total, R >= 4
so concurrent launches on up to 4 streams never share data).

`roofline.achieved` = algorithmic bytes per launch (R_i =
min(len,128) + max(0, H_i-128) + D, W_i = record bytes) / (timed region / K),
i.e. the HBM rate the device sustains on this path, from HIP events on the
launch streams.  `cpu_baseline` = the C restatement of ingot's parse
(oracle/, "port") on the host cores, rank 0, N=1.
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mpkt/s device-resident L2/L3/L4 parse, 64–1500 B frames; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md:36 (spec)
HBM_MEASURED_GBS = 6290.0  # MI355X_MICROARCH.md:36 (measured float4 copy)

CONFIGS = {
    # name: (profile, frames per GPU, slot stride or None (packed), chain, description)
    "c2": ("V4UDP64", 1 << 20, 64, "UdpParser",
           "C2: 1,048,576 x 64 B Eth/IPv4/UDP per GPU, 64-B slots, UdpParser"),
    "c3": ("MIXED", 1 << 24, None, "GenericUlp",
           "C3: 16,777,216 mixed 64-1500 B v4/v6 x TCP/UDP per GPU, packed, GenericUlp"),
    "c3s": ("MIXED", 1 << 22, 2048, "GenericUlp",
            "C3 frames in 2048-B ring slots (NIC-ring layout): 4,194,304 per GPU, GenericUlp"),
    "c4": ("VLAN_V6EH", 1 << 23, None, "VlanUlp",
           "C4: 8,388,608 VLAN/QinQ + IPv6-EH mixed frames per GPU (64M over 8), packed, "
           "VlanUlp"),
    "c5": ("FLOWS", 1 << 23, None, "VlanUlp",
           "C5: C4 framing, 65,536 Zipf(1.1) flows; parse + RSS Toeplitz 5-tuple hash + "
           "per-flow histogram (65,536 x u32) + RCCL all-reduce per step, 8,388,608 per GPU"),
    "c6": ("GENEVE", 1 << 23, None, "GeneveOverV6Tunnel",
           "C6 (SURVEY 8f-1): 8,388,608 Geneve-over-IPv6 tunnel frames per GPU (OPTE inbound: "
           "outer Eth/IPv6/UDP/Geneve+options, inner 64-1500 B Eth/v4|v6/TCP|UDP|ICMP, 2% ARP), "
           "packed, GeneveOverV6Tunnel"),
    "c2m": ("V4UDP64", 1 << 20, 64, "UdpParser",
            "C2 as the reference's parse-and-decr-v4 (ingot-examples/benches/packet.rs:139-145):"
            " 1,048,576 x 64 B, parse UdpParser + l4.destination -= 1 in place (SURVEY 8f-4)"),
    "c3r": ("MIXED", 1 << 24, None, "GenericUlp",
            "C3 frames as 2-chunk packets (header chunk + payload chunk, mblk-style), "
            "parse_read over chunk lists (SURVEY 8f-3), 16,777,216 per GPU, GenericUlp"),
    "c3p": ("MIXED", 1 << 24, None, "GenericUlp",
            "C3 frames back to back with only a length array (capture-buffer layout): "
            "offsets scanned on the device, 16,777,216 per GPU, GenericUlp"),
}
# configs that time something other than the batched parse_slice records
MODES = {"c5": "flows", "c2m": "modify", "c3r": "read", "c3p": "packed"}
# Streams the steps alternate over, measured per config (tools/abtune.py,
# DESIGN.md §5): short launches overlap their ramp-up/drain on 2 (C2 12.3 vs
# 15.2 us, C2m 20.5 vs 25.0) or 3 (C3s 112.5 vs 115.1); long gather-bound
# launches gain nothing (C3 606 / 618, C4 324 / 324, C6 392 / 393 us on 1 / 2).
STREAMS = {"c2": 2, "c2m": 2, "c3": 1, "c3p": 1, "c3r": 2, "c3s": 3, "c4": 1, "c5": 2,
           "c6": 1}
FLOW_BINS = 1 << 16


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(recs_np, lens_np, stride, descriptor_bytes, record_bytes):
    """R_i = min(len_i,128) + max(0, H_i-128) + D ; W_i = record.
    H_i = the header span the parse consumed (payload_off)."""
    lens = lens_np.astype(np.int64) if lens_np is not None else np.full(len(recs_np), stride)
    h = recs_np["payload_off"].astype(np.int64)
    r = np.minimum(lens, 128) + np.maximum(0, h - 128) + descriptor_bytes
    return int(r.sum()), record_bytes * len(recs_np)


def host_inclusive(config: str):
    """The host-inclusive rates of this config (frames start and end in host
    memory), from the committed tools/hostpath.py measurement — reported
    beside `value`, never as it."""
    f = sorted(ROOT.glob("profiles/*_hostpath.json"))
    if not f:
        return None
    d = json.loads(f[-1].read_text())
    if config not in d:
        return None
    out = {"memcpy_Mpkt_s": d[config]["host_inclusive_Mpkt_s"],
           "source": f"{f[-1].relative_to(ROOT)} (tools/hostpath.py, 1 M frames per batch)"}
    if f"{config}_zc" in d:
        out["zero_copy_Mpkt_s"] = d[f"{config}_zc"]["host_inclusive_Mpkt_s"]
    return out


def cpu_baseline(arena_np, off_np, lens_np, stride, n, chain, budget_s=1.5, mode="parse",
                 segs=None):
    """Time the oracle on the host cores over the same frames (bounded).
    mode "read": parse_read over `segs` = (seg_off, seg_len, pkt_seg);
    "modify": parse + the same setter in place on the sample."""
    import oracle
    from ingot_amd import EditOp, Field

    try:  # -march=native build for this host, into a scratch dir
        d = Path(os.environ.get("TMPDIR", "/tmp")) / f"ingot_oracle_native_{os.getpid()}"
        lib = oracle.load(oracle.build(out_dir=d, native=True))
        arch = "native"
    except Exception as e:  # noqa: BLE001
        log(f"[bench] native oracle build failed ({e}); using the prebuilt x86-64-v3 one")
        lib = oracle.load()
        arch = "x86-64-v3"

    def one_pass(t):
        if mode == "read":
            oracle.parse_read_batch(arena_np, *segs, chain, lib=lib, nthreads=t)
        elif mode == "modify":
            oracle.parse_modify_batch(arena_np, off_np, lens_np, chain,
                                      [(2, Field.UDP_DESTINATION, EditOp.SUB, 1)], stride=stride,
                                      n=n, lib=lib, nthreads=t)
        else:
            oracle.parse_batch(arena_np, off_np, lens_np, chain, stride=stride, n=n,
                               nthreads=t, lib=lib)

    threads = max(1, min(16, os.cpu_count() or 1))
    res = {}
    for t in sorted({1, threads}):
        one_pass(t)
        reps, t0 = 0, time.perf_counter()
        while True:
            one_pass(t)
            reps += 1
            el = time.perf_counter() - t0
            if el > (budget_s if t > 1 else budget_s / 2):
                break
        res[t] = (reps * n / el / 1e6, reps, el)
    mp, reps, el = res[threads]
    what = {"parse": "parse_slice", "read": "parse_read", "modify": "parse + set_destination"}
    return {
        "value": round(mp, 3), "unit": "Mpkt/s", "cores": threads, "kind": "port",
        "sample": f"{reps} passes x {n} frames of the benchmark batch (same bytes), "
                  f"{el:.2f} s wall on {threads} threads; C restatement of ingot "
                  f"{what.get(mode, mode)} (oracle/), -march={arch}",
        "single_core_value": round(res[1][0], 3),
        "cpu_model": _cpu_model(),
        "host_cpus": os.cpu_count(),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class Runner:
    """Launches step k (arena k % R -> records k % R) on stream k % S."""

    def __init__(self, torch, lib, ctx, chain, n, stride, arenas, off, lens, outs, streams,
                 record_bytes):
        self.torch, self.streams = torch, streams
        reps = len(arenas)
        h = ctx._h
        optr = off.data_ptr() if off is not None else None
        lptr = lens.data_ptr() if lens is not None else None
        aptrs = [a.data_ptr() for a in arenas]
        outptrs = [o.data_ptr() for o in outs]
        sps = [s.cuda_stream for s in streams]
        ns = len(sps)
        c = int(chain)
        if stride is not None:
            fn = lib.ingot_gpu_parse_strided if record_bytes == 16 else \
                lib.ingot_gpu_parse_strided_compact
            self.launch = lambda k: fn(h, aptrs[k % reps], stride, lptr, n, c,
                                       outptrs[k % reps], sps[k % ns])
        else:
            fn = lib.ingot_gpu_parse if record_bytes == 16 else lib.ingot_gpu_parse_compact
            self.launch = lambda k: fn(h, aptrs[k % reps], optr, lptr, n, c,
                                       outptrs[k % reps], sps[k % ns])

    def run(self, steps):
        """Time `steps` launches: fork all streams from streams[0], join back."""
        return _timed(self.torch, self.streams, self.launch, steps)


class PackedRunner:
    """Lengths-only packed frames: ingot_gpu_parse_packed (tile-sum scan +
    parse) on arena k % R, a workspace per stream."""

    def __init__(self, torch, lib, ctx, chain, n, arenas, lens, outs, streams):
        self.torch, self.streams = torch, streams
        reps, h, c = len(arenas), ctx._h, int(chain)
        aptrs = [a.data_ptr() for a in arenas]
        outptrs = [o.data_ptr() for o in outs]
        lptr = lens.data_ptr()
        wb = lib.ingot_gpu_packed_workspace_size(n)
        self.work = [torch.empty(wb, dtype=torch.uint8, device=lens.device) for _ in streams]
        wptrs = [w.data_ptr() for w in self.work]
        sps = [s.cuda_stream for s in streams]
        ns = len(sps)
        self.launch = lambda k: lib.ingot_gpu_parse_packed(h, aptrs[k % reps], lptr, n, c,
                                                           outptrs[k % reps], None,
                                                           wptrs[k % ns], wb, sps[k % ns])

    def run(self, steps):
        return _timed(self.torch, self.streams, self.launch, steps)


class ModifyRunner:
    """parse-and-decr: parse + `l4.set_destination(l4.destination() - 1)` in
    place on arena k % R, no records (the reference bench keeps none)."""

    def __init__(self, torch, lib, ctx, chain, n, stride, arenas, off, lens, streams):
        import ingot_amd

        self.torch, self.streams = torch, streams
        reps, h, c = len(arenas), ctx._h, int(chain)
        self._edits = ingot_amd.edits_array([(2, ingot_amd.Field.UDP_DESTINATION,
                                              ingot_amd.EditOp.SUB, 1)])
        eptr = self._edits.ctypes.data
        aptrs = [a.data_ptr() for a in arenas]
        optr = off.data_ptr() if off is not None else None
        lptr = lens.data_ptr() if lens is not None else None
        sps = [s.cuda_stream for s in streams]
        ns = len(sps)
        self.launch = lambda k: lib.ingot_gpu_parse_modify(h, aptrs[k % reps], optr, lptr,
                                                           stride or 0, n, c, eptr, 1, None,
                                                           sps[k % ns])

    def run(self, steps):
        return _timed(self.torch, self.streams, self.launch, steps)


class ReadRunner:
    """parse_read over chunk lists: arena k % R with the shared segment tables."""

    def __init__(self, torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg, outs,
                 streams):
        self.torch, self.streams = torch, streams
        reps, h, c = len(arenas), ctx._h, int(chain)
        aptrs = [a.data_ptr() for a in arenas]
        outptrs = [o.data_ptr() for o in outs]
        so, sl, ps = seg_off.data_ptr(), seg_len.data_ptr(), pkt_seg.data_ptr()
        sps = [s.cuda_stream for s in streams]
        ns = len(sps)
        self.launch = lambda k: lib.ingot_gpu_parse_read(h, aptrs[k % reps], so, sl, ps, n, c,
                                                         outptrs[k % reps], None, sps[k % ns])

    def run(self, steps):
        return _timed(self.torch, self.streams, self.launch, steps)


class FlowRunner:
    """Config 5 step: zero the histogram, parse + hash + histogram kernels,
    then the RCCL all-reduce of that step's histogram.  Step k runs on stream
    k % S with its own histogram workspace, so the next step's flow kernel
    fills the CUs the histogram passes leave idle; the all-reduce runs on
    RCCL's stream and overlaps later steps.  Histograms rotate over the arena
    copies: a step's buffer is reused `reps` steps later, after its reduce has
    been waited for on the reusing step's stream; the timed region ends after
    every reduce has completed."""

    def __init__(self, torch, lib, ctx, chain, n, arenas, off, lens, hists, flows, streams,
                 reduce_fn):
        self.torch, self.streams = torch, list(streams)
        reps, S = len(arenas), len(self.streams)
        assert reps >= 4
        h, c = ctx._h, int(chain)
        optr, lptr = off.data_ptr(), lens.data_ptr()
        aptrs = [a.data_ptr() for a in arenas]
        works = {}

        # caller-owned workspaces (one per stream): the atomics-free histogram pass
        wbytes = lib.ingot_gpu_flow_hist_workspace_size(n, hists[0].numel())
        self.work = [torch.empty(max(1, wbytes), dtype=torch.uint8, device=hists[0].device)
                     for _ in range(S)]

        def launch(k):
            st = self.streams[k % S]
            hist = hists[k % reps]
            with torch.cuda.stream(st):
                w = works.pop(k - reps, None)  # the last reduce of this buffer
                if w is not None:
                    w.wait()
                hist.zero_()
                rc = lib.ingot_gpu_flow_hist_ws(h, aptrs[k % reps], optr, lptr, 0, n, c, None,
                                                hist.numel(), flows[k % reps].data_ptr(), None,
                                                hist.data_ptr(), self.work[k % S].data_ptr(),
                                                wbytes, st.cuda_stream)
                w = reduce_fn(hist)
            if w is not None:
                works[k] = w
            return rc

        def finish():
            with torch.cuda.stream(self.streams[0]):
                for k in sorted(works):
                    works.pop(k).wait()

        self.launch, self.finish = launch, finish

    def run(self, steps):
        return _timed(self.torch, self.streams, self.launch, steps, self.finish)


def _timed(torch, streams, launch, steps, finish=None):
    """Run `steps` launches between two HIP events on streams[0]; the other
    streams fork from the start event and join before the end event (as does
    `finish`'s outstanding work)."""
    s0 = streams[0]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    e0.record(s0)
    for s in streams[1:]:
        s.wait_event(e0)
    for k in range(steps):
        rc = launch(k)
        if rc:
            raise RuntimeError(f"launch failed: {rc}")
    if finish is not None:
        finish()
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        s0.wait_event(ev)
    e1.record(s0)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), time.perf_counter() - w0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--streams", type=int, default=0,
                    help="streams the steps alternate over (0 = the config's measured best)")
    ap.add_argument("--record", type=int, default=16, choices=(16, 8))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=1.5)
    ap.add_argument("--rotate-mib", type=int, default=512,
                    help="minimum bytes of distinct arenas rotated across steps")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N>1 on one GPU")
    args = ap.parse_args()
    if args.streams <= 0:
        args.streams = STREAMS.get(args.config, 2)

    import torch
    import torch.distributed as dist

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    from ingot_amd import dist as idist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; a --dist-backend gloo rehearsal may fold ranks onto
    # fewer GPUs (e.g. the 1-GPU test box)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    prof_name, n, stride, chain_name, desc = CONFIGS[args.config]
    profile, chain = GenProfile[prof_name], Chain[chain_name]
    ctx = ingot_amd.Context(local)
    lib = ingot_amd.load_library()

    # --- data: this rank's shard (pure in (seed, index)) + R copies ---
    first, n = idist.shard(rank, world, n)
    arena, off, lens = ingot_amd.gen_frames(profile, n, first=first, stride=stride,
                                            device=local)
    # >= 512 MiB of distinct arenas (the 256 MiB MALL cannot serve a step from
    # the previous one), and >= 4 copies so that launches in flight on up to 4
    # streams never read the same bytes (no cross-step cache sharing)
    reps = max(4, -(-(args.rotate_mib << 20) // arena.numel()))
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device=dev) for _ in range(reps)]
    torch.cuda.synchronize(dev)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                  for _ in range(max(3, args.streams - 1))]

    mode = MODES.get(args.config, "parse")
    flows = mode == "flows"
    if flows:
        hists = [torch.zeros(FLOW_BINS, dtype=torch.int32, device=dev) for _ in range(reps)]
        flow_ids = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(reps)]
    if mode == "read":
        # mblk-style packets: chunk 0 = the header span (payload_off of a
        # parse_slice pass), chunk 1 = the payload; both in the same arena
        poff = ingot_amd.records_to_numpy(ctx.parse(arena, off, lens, chain))["payload_off"]
        poff = torch.from_numpy(poff.astype(np.int64)).to(dev)
        len64 = lens.to(torch.int64)
        seg_off = torch.stack([off, off + poff], 1).reshape(-1).contiguous()
        seg_len = torch.stack([poff, len64 - poff], 1).reshape(-1).to(torch.int32) \
            .to(torch.uint16).contiguous()
        pkt_seg = torch.arange(0, 2 * n + 1, 2, dtype=torch.int32, device=dev)
        del poff, len64

    def runner(nstreams, record):
        if flows:
            return FlowRunner(torch, lib, ctx, chain, n, arenas, off, lens, hists, flow_ids,
                              streams[:nstreams], idist.reduce_histogram_async)
        if mode == "modify":
            return ModifyRunner(torch, lib, ctx, chain, n, stride, arenas, off, lens,
                                streams[:nstreams])
        if mode == "packed":
            return PackedRunner(torch, lib, ctx, chain, n, arenas, lens, outs,
                                streams[:nstreams])
        if mode == "read":
            return ReadRunner(torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg,
                              outs, streams[:nstreams])
        return Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs,
                      streams[:nstreams], record)

    if flows:
        args.no_variants = True
    if mode in ("modify", "read", "packed") and args.record == 8:
        ap.error("8-B records are not offered for this config")
    if chain == Chain.GeneveOverV6Tunnel and args.record == 8:
        ap.error("8-B records are not offered for the tunnel chain (include/ingot_gpu.h)")
    main_run = runner(args.streams, args.record)
    main_run.run(args.warmup)

    # --- timed region: K steps, barrier + sync on both sides ---
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ms_region, wall = main_run.run(args.steps)
    if world > 1:
        dist.barrier()
    t_sec = idist.max_over_ranks(ms_region / 1e3, device=dev)
    value = n * args.steps * world / t_sec / 1e6
    ms_step = t_sec * 1e3 / args.steps

    # --- algorithmic bytes from this batch's records (16-B form) ---
    recs = ctx.parse_strided(arenas[0], stride, n, chain, lens=lens) \
        if stride is not None else ctx.parse(arenas[0], off, lens, chain)
    torch.cuda.synchronize(dev)
    recs_np = ingot_amd.records_to_numpy(recs)
    lens_np = lens.cpu().numpy() if lens is not None else None
    if mode == "read":
        # chunk 0 read like a frame of the header span's length; descriptors:
        # pkt_seg (4 B) + chunk 0's (u64 off, u16 len) = 14 B
        rd, wr = algorithmic_bytes(recs_np, recs_np["payload_off"], 0, 14, 16)
    elif mode == "packed":
        # descriptors: the u16 length, read by the parse and once more by the
        # tile-sum pass; tile sums and bases: 12 B per 64 packets
        rd, wr = algorithmic_bytes(recs_np, lens_np, 0, 2, args.record)
        rd += 2 * n + 12 * ((n + 63) // 64)
    else:
        rd, wr = algorithmic_bytes(recs_np, lens_np, stride or 0, 0 if stride else 10,
                                   args.record)
    if flows:  # per-packet flow id (4 B) written, read once by the histogram pass
        wr = 4 * n + FLOW_BINS * 4
        rd += 4 * n
    if mode == "modify":  # no records; the 2 rewritten bytes per packet
        wr = 2 * n
    bytes_launch = rd + wr
    pipelined_gbs = bytes_launch / (ms_region / args.steps / 1e3) / 1e9
    # Roofline of the kernel itself: a single-stream pass (launches back to
    # back, so region/K = one launch incl. the dependent-launch boundary; this
    # is what rocprofv3's per-dispatch mean measures).  In the pipelined
    # schedule two launches overlap, so per-dispatch durations are not per-step.
    iso = runner(1, args.record)
    iso.run(min(args.warmup, 50))
    iso_steps = min(args.steps, 1000)
    ms_iso, _ = iso.run(iso_steps)
    launch_ms = ms_iso / iso_steps
    achieved = bytes_launch / (launch_ms / 1e3) / 1e9
    ok_frac = float((recs_np["status"] == 0).mean())
    # the multi-tile ring kernel serves slot rings without a length array
    # (launch_parse in parse.hip); everything else is the one-tile k_parse
    ring = (mode == "parse" and stride is not None and stride >= 64 and lens is None
            and chain != Chain.GeneveOverV6Tunnel)
    traffic = None
    pmc = sorted(ROOT.glob(f"profiles/*_pmc_{args.config}.json"))
    if pmc and args.record == 16:
        t = json.loads(pmc[-1].read_text())
        traffic = {"bytes_per_launch": t["traffic_bytes_per_launch"],
                   "ratio_to_algorithmic": round(t["traffic_bytes_per_launch"] / bytes_launch, 4),
                   "source": f"{pmc[-1].relative_to(ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + "
                             "WRITE_SIZE, separate passes)"}

    # --- variants (outside the timed region; same data) ---
    variants = {}
    if not args.no_variants:
        vsteps = min(args.steps, 1000)
        for ns, rb in ((1, 16), (2, 8), (1, 8), (4, 16)):
            if (ns, rb) == (args.streams, args.record):
                continue
            if rb == 8 and (chain == Chain.GeneveOverV6Tunnel or mode != "parse"):
                continue
            r = runner(ns, rb)
            r.run(min(args.warmup, 50))
            ms, _ = r.run(vsteps)
            bpl = rd + (rb * n if mode != "modify" else wr)
            variants[f"streams{ns}_rec{rb}"] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3),
                "hbm_GBps": round(bpl / (ms / vsteps / 1e3) / 1e9, 1),
            }

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            m = min(n, 1 << 20)  # bounded sample: the first 1M frames of the batch
            if off is not None:
                o_np = off[:m].cpu().numpy()
                end = int(o_np[-1]) + int(lens_np[m - 1])
                a_np = arenas[0][:end + 64].cpu().numpy()
            else:
                o_np, a_np = None, arenas[0][:m * stride].cpu().numpy()
            l_np = lens_np[:m] if lens_np is not None else None
            segs = None
            if mode == "read":
                segs = (seg_off[:2 * m].cpu().numpy().view(np.uint64),
                        seg_len[:2 * m].to(torch.int32).cpu().numpy().astype(np.uint16),
                        pkt_seg[:m + 1].cpu().numpy().view(np.uint32))
            cpu = cpu_baseline(a_np, o_np, l_np, stride or 0, m, chain, args.cpu_budget,
                               mode="parse" if flows else mode, segs=segs)
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-generated, seed 20250808)",
            "config": {
                "workload": desc,
                "frames_per_gpu": n,
                "chain": chain_name,
                "layout": f"strided {stride} B" if stride else "packed, u64 offsets + u16 lengths",
                "record_bytes": args.record,
                "streams": args.streams,
                "arena_copies_rotated": reps,
                "parallelism": (f"shard per GPU x{world}; RCCL all-reduce (sum) of the "
                                f"{FLOW_BINS} x u32 flow histogram every step" if flows else
                                f"shard per GPU x{world} (no data-path collective)"),
                "ok_fraction": round(ok_frac, 6),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "traffic_detail": traffic,
                "kernel": ("k_parse_pipe" if ring else "k_parse") + " (ingot_amd/csrc/parse.hip)" + {
                    "modify": ", OUT_MODIFY", "read": ", LAYOUT_SEGMENTED",
                    "packed": ", LAYOUT_PACKED + k_tile_sums/k_tile_scan",
                    "flows": ", OUT_FLOWS + k_flow_count16/k_flow_reduce16"}.get(mode, ""),
                "launch_mean_us": round(launch_ms * 1e3, 3),
                "launch_timing": "single-stream pass, HIP events, region/K",
                "pipelined_GBps": round(pipelined_gbs, 1),
                "pipelined_frac": round(pipelined_gbs / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": bytes_launch,
                "read_bytes_per_launch": rd,
                "write_bytes_per_launch": wr,
                "read_frac": round(rd / (launch_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "frac_of_measured_copy_ceiling": round(achieved / HBM_MEASURED_GBS, 4),
            },
            "variants": variants,
            "cpu_baseline": cpu,
            "wall_s_timed_region": round(wall, 4),
            "host_inclusive": host_inclusive(args.config),
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
