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
    "c2r": ("V4UDP64", 1 << 20, 64, "UdpParser",
            "C2 frames as the reference's parse-read-v4 chunk chain (ingot-examples/benches/"
            "packet.rs:130-134, 152-156): one chunk per header, 14 / 20 / 8 B + payload, "
            "parse_read over chunk lists, 1,048,576 per GPU, UdpParser"),
}
# configs that time something other than the batched parse_slice records
MODES = {"c5": "flows", "c2m": "modify", "c3r": "read", "c3p": "packed", "c2r": "read"}
# parse_read chunking: "split2" = header span | payload; "per_header" = one
# chunk per parsed header, then the payload (the reference bench's shape)
READ_CHUNKS = {"c3r": "split2", "c2r": "per_header"}
# Strong scaling (--scaling strong): the whole job's frames, split over the
# ranks (BASELINE.json configs[3]: 64 M frames over 8 GPUs); other configs
# split their single-GPU batch.
STRONG_TOTAL = {"c4": 1 << 26, "c5": 1 << 26}
# Arena copies rotated across steps are capped at this many bytes per GPU.
ROTATE_CAP_BYTES = 64 << 30
# Streams the steps alternate over, measured per config (tools/abtune.py,
# DESIGN.md §5): short launches overlap their ramp-up/drain on 2 (C2 12.3 vs
# 15.2 us, C2m 20.5 vs 25.0) or 3 (C3s 112.5 vs 115.1); long gather-bound
# launches gain nothing (C3 606 / 618, C4 324 / 324, C6 392 / 393 us on 1 / 2).
STREAMS = {"c2": 2, "c2m": 2, "c3": 1, "c3p": 1, "c3r": 1, "c3s": 3, "c4": 1, "c5": 2,
           "c6": 1, "c2r": 2}
# Staggered streams (gated regions with >= 2 streams): stream i starts
# i * STAGGER_US behind stream 0 (ingot_gpu_stream_delay), so the streams'
# launches do not ramp up and drain in lockstep.  0 = start together.
# Measured (tools/stagger_ab.py, interleaved, 20-step regions after a 5-step
# warm-up as the driver runs them; profiles/r02_stagger_ab.json): C2 12.32-12.38
# -> 12.18-12.20 us/step at 5-7 us, 12.5 at 12 us; 200-step regions unchanged.
STAGGER_US = {"c2": 6.0}
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


def host_inclusive_live(torch, ingot_amd, ctx, arena, off, lens, stride, chain, n, steps=30):
    """The path as it starts and ends in host memory, measured in this run
    on the first min(n, 1 M) frames of the batch (tools/hostpath.py:measure):
    a pinned host ring -> hipMemcpyAsync H2D -> parse -> records D2H, and the
    zero-copy form (ring and records mapped for the device, the kernels read
    only the header bytes across PCIe).  Reported beside `value`, never as it."""
    sys.path.insert(0, str(ROOT / "tools"))
    import hostpath

    m = min(n, 1 << 20)
    out = {"frames_per_batch": m, "streams": 3}
    for zc in (False, True):
        r = hostpath.measure(torch, ingot_amd, ctx, arena, off, lens, stride, chain, m,
                             streams=3, steps=steps, zero_copy=zc)
        key = "zero_copy" if zc else "memcpy"
        out[f"{key}_Mpkt_s"] = r["host_inclusive_Mpkt_s"]
        out[f"{key}_ms_per_batch"] = r["ms_per_batch"]
    out["source"] = "measured in this run (tools/hostpath.py: measure)"
    return out


def cpu_baseline(arena_np, off_np, lens_np, stride, n, chain, budget_s=1.5, mode="parse",
                 segs=None):
    """Time the oracle (the C restatement of ingot's parse) on the host's
    cores over the same frames, bounded: all os.cpu_count() threads (the
    figure reported) and 1 thread.  Each worker repeats its contiguous share
    of the sample `passes` times per call, so thread start-up (one pthread
    per CPU per call) is amortised; a share is then cache-resident after the
    first pass — generous to the CPU.  mode "read": parse_read over `segs` =
    (seg_off, seg_len, pkt_seg); "modify": parse + the same setter in place."""
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

    def one_call(t):
        if mode == "read":
            oracle.parse_read_batch(arena_np, *segs, chain, lib=lib, nthreads=t)
        elif mode == "modify":
            oracle.parse_modify_batch(arena_np, off_np, lens_np, chain,
                                      [(2, Field.UDP_DESTINATION, EditOp.SUB, 1)], stride=stride,
                                      n=n, lib=lib, nthreads=t)
        else:
            oracle.parse_batch(arena_np, off_np, lens_np, chain, stride=stride, n=n,
                               nthreads=t, lib=lib)

    host = os.cpu_count() or 1
    res = {}
    for t, budget in ((1, budget_s / 2), (host, budget_s)):
        lib.oracle_set_passes(1)
        one_call(t)  # warm (page faults, thread stacks)
        t0 = time.perf_counter()
        one_call(t)
        once = max(time.perf_counter() - t0, 1e-6)
        passes = max(1, min(10000, int(budget / 4 / once)))
        lib.oracle_set_passes(passes)
        calls, t0 = 0, time.perf_counter()
        while True:
            one_call(t)
            calls += 1
            el = time.perf_counter() - t0
            if el > budget:
                break
        res[t] = (calls * passes * n / el / 1e6, calls * passes, el)
    lib.oracle_set_passes(1)
    mp, reps, el = res[host]
    what = {"parse": "parse_slice", "read": "parse_read", "modify": "parse + set_destination"}
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = host
    return {
        "value": round(mp, 3), "unit": "Mpkt/s", "cores": host, "kind": "port",
        "sample": f"{reps} passes x {n} frames of the benchmark batch (same bytes), "
                  f"{el:.2f} s wall on {host} threads (every host CPU; each thread repeats "
                  f"its share, cache-resident after the first pass); C restatement of ingot "
                  f"{what.get(mode, mode)} (oracle/), -march={arch}",
        "single_core_value": round(res[1][0], 3),
        "cpu_model": _cpu_model(),
        "host_cpus": host,
        "affinity_cpus": affinity,
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

    def run(self, steps, gate=None):
        """Time `steps` launches (see _timed)."""
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


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

    def run(self, steps, gate=None):
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


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

    def run(self, steps, gate=None):
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


class ReadRunner:
    """parse_read over chunk lists: arena k % R with the shared segment tables
    (dense: one (offset << 16) | length entry per chunk,
    ingot_gpu_parse_read_dense)."""

    def __init__(self, torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg, outs,
                 streams, dense=False):
        self.torch, self.streams = torch, streams
        reps, h, c = len(arenas), ctx._h, int(chain)
        aptrs = [a.data_ptr() for a in arenas]
        outptrs = [o.data_ptr() for o in outs]
        so, sl, ps = seg_off.data_ptr(), seg_len.data_ptr(), pkt_seg.data_ptr()
        sps = [s.cuda_stream for s in streams]
        ns = len(sps)
        if dense:
            self.seg = ((seg_off << 16) | (seg_len.to(torch.int32) & 0xFFFF).to(torch.int64))
            sd = self.seg.data_ptr()
            self.launch = lambda k: lib.ingot_gpu_parse_read_dense(
                h, aptrs[k % reps], sd, ps, n, c, 0, outptrs[k % reps], None, sps[k % ns])
            return
        self.launch = lambda k: lib.ingot_gpu_parse_read(h, aptrs[k % reps], so, sl, ps, n, c,
                                                         outptrs[k % reps], None, sps[k % ns])

    def run(self, steps, gate=None):
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


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
                 reduce_fn, flows_only=False):
        """flows_only: launch the parse + hash kernel alone (no histogram, no
        reduce) — the dominant kernel, timed for `roofline`."""
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
            if flows_only:
                return lib.ingot_gpu_flow_hist_ws(h, aptrs[k % reps], optr, lptr, 0, n, c, None,
                                                  hist.numel(), flows[k % reps].data_ptr(), None,
                                                  None, None, 0, st.cuda_stream)
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

    def run(self, steps, gate=None):
        return _timed(self.torch, self.streams, self.launch, steps, self.finish, gate=gate)


class Gate:
    """Holds the first launches of a timed region behind a doorbell
    (ingot_gpu_doorbell_wait on every stream), the way a ring consumer
    enqueues its next batches before they arrive: the region then starts when
    the GPU starts the first step, not when the host has finished submitting
    it (ctypes + hipLaunchKernel + event records cost tens of us of host time
    while the start event has already been stamped).  Every launch still runs
    inside the region.  Only the first HOLD launches wait (a bounded number of
    queued packets); a watchdog thread rings the doorbell after WATCHDOG_S
    whatever happens, so a stream can never be left waiting."""

    HOLD = 64
    WATCHDOG_S = 20.0

    def __init__(self, ingot_amd, ctx, stagger_us=0.0):
        import threading

        self.db = ingot_amd.Doorbell(ctx)
        self.ctx = ctx
        self.stagger_ns = int(round(stagger_us * 1000))
        self.seq = 0
        self._threading = threading

    def arm(self, streams):
        self.seq += 1
        for i, s in enumerate(streams):
            self.db.wait(self.seq, s)
            if i and self.stagger_ns:
                self.ctx.stream_delay(i * self.stagger_ns, s)
        seq, db = self.seq, self.db
        self._timer = self._threading.Timer(self.WATCHDOG_S, lambda: db.ring(seq))
        self._timer.daemon = True
        self._timer.start()

    def open(self):
        self.db.ring(self.seq)
        self._timer.cancel()


def _timed(torch, streams, launch, steps, finish=None, gate=None):
    """Run `steps` launches; returns (ms, wall s).  Every stream stamps a
    start event before its first launch and an end event after its last one;
    the region is the earliest start to the latest end (all on the device
    clock).  Ungated, the other streams fork from streams[0]'s start event;
    gated, every stream waits on the doorbell instead.  No stream joins
    another at the end: a cross-stream event wait costs ~7 us of device time
    that would land inside the region (tools/region_probe.py)."""
    s0 = streams[0]
    w0 = time.perf_counter()
    if gate is not None:
        gate.arm(streams)
    starts, ends = [], []
    try:
        if gate is None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            starts.append(e0)
            for s in streams[1:]:
                s.wait_event(e0)
        else:
            for s in streams:
                e = torch.cuda.Event(enable_timing=True)
                e.record(s)
                starts.append(e)
        for k in range(steps):
            rc = launch(k)
            if rc:
                raise RuntimeError(f"launch failed: {rc}")
            if gate is not None and k + 1 == Gate.HOLD:
                gate.open()
        if finish is not None:
            finish()
        for s in streams:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ends.append(e)
    finally:
        if gate is not None:
            gate.open()
    torch.cuda.synchronize()
    ms = max(a.elapsed_time(b) for a in starts for b in ends)
    return ms, time.perf_counter() - w0


def kernel_sources_sha() -> str:
    """Digest of every source the library's kernels are built from: a PMC
    profile in profiles/ is attached to a bench line only when it was taken
    on these exact sources (tools/pmc_traffic.py records the same digest)."""
    import hashlib

    h = hashlib.sha256()
    files = sorted((ROOT / "ingot_amd" / "csrc").glob("*")) + sorted((ROOT / "include").glob("*.h"))
    for f in files:
        if f.suffix in (".hip", ".h", ".cpp"):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:16]


def kernel_family(mode: str, ring: bool) -> str:
    """The dominant kernel this config launches (parse.hip's dispatch)."""
    if mode == "read":
        return "k_parse_read"
    if mode == "modify":
        return "k_modify_pipe" if ring else "k_parse"
    return "k_parse_pipe" if ring else "k_parse"


def pmc_for(config: str, family: str, sha: str, n: int):
    """The newest profiles/*_pmc_<config>.json taken on these kernel sources,
    over launches of n frames, whose profiled kernel is `family`; None
    otherwise."""
    for f in sorted(ROOT.glob(f"profiles/*_pmc_{config}.json"), reverse=True):
        t = json.loads(f.read_text())
        k = t.get("kernel") or (t.get("kernels") or [""])[0]
        if t.get("sources_sha") != sha or t.get("frames_per_launch") != n:
            continue
        if f"::{family}<" not in k and not k.startswith(f"{family}<"):
            continue
        return t, f
    return None, None


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list) -> int:
    """`--gpus N` without a launcher: start N child processes of this script,
    one per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun sets
    them), before anything in this process touches a GPU.  Rank 0's JSON
    line goes to the shared stdout.  If a rank fails, the others (exact PIDs
    started here) are terminated; returns the first failing exit code."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + argv,
                                      env=env))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def frames_for_rank(config: str, scaling: str, rank: int, world: int):
    """(first, n, total): this rank's contiguous share of the job's frames."""
    from ingot_amd import dist as idist

    n = CONFIGS[config][1]
    if scaling == "strong":
        total = STRONG_TOTAL.get(config, n)
        first, cnt = idist.split(total, rank, world)
        return first, cnt, total
    first, cnt = idist.shard(rank, world, n)
    return first, cnt, n * world


def read_chunks(torch, off, stride, lens, recs_np, kind, dev):
    """parse_read chunk tables for the read configs (all chunks inside the
    packet's own bytes of the arena, mblk-style): "split2" = [header span |
    payload], "per_header" = one chunk per parsed header, then the payload
    (cuts at l3_off, l4_off, payload_off: no header straddles a cut, so the
    records equal parse_slice's).  Returns (seg_off u64, seg_len u16,
    pkt_seg u32 as int32, chunks covering the header span per packet)."""
    n = len(recs_np)
    L = lens.to(torch.int64)
    poff = torch.from_numpy(recs_np["payload_off"].astype(np.int64)).to(dev)
    if kind == "split2":
        cuts = poff[:, None]
    else:
        cuts = torch.stack([torch.from_numpy(recs_np[k].astype(np.int64)).to(dev)
                            for k in ("l3_off", "l4_off", "payload_off")], 1)
    # keep a cut when it is past every earlier cut and inside the frame
    prev = torch.zeros(n, dtype=torch.int64, device=dev)
    keep = []
    for k in range(cuts.shape[1]):
        c = cuts[:, k]
        m = (c > prev) & (c < L)
        keep.append(m)
        prev = torch.where(m, c, prev)
    keep = torch.stack(keep, 1)
    bounds = torch.cat([torch.zeros(n, 1, dtype=torch.int64, device=dev), cuts, L[:, None]], 1)
    valid = torch.cat([torch.ones(n, 1, dtype=torch.bool, device=dev), keep], 1)
    nchunks = valid.sum(1)
    starts = bounds[:, :-1][valid]                        # row-major: packet by packet
    # each chunk ends at the next kept boundary (or the frame end)
    nxt = torch.full_like(bounds[:, :-1], -1)
    run = L.clone()
    for k in range(valid.shape[1] - 1, -1, -1):
        nxt[:, k] = run
        run = torch.where(valid[:, k], bounds[:, k], run)
    ends = nxt[valid]
    base = off if off is not None else torch.arange(n, dtype=torch.int64, device=dev) * stride
    seg_off = (base.repeat_interleave(nchunks) + starts).contiguous()
    seg_len = (ends - starts).to(torch.int32).to(torch.uint16).contiguous()
    pkt_seg = torch.zeros(n + 1, dtype=torch.int32, device=dev)
    pkt_seg[1:] = nchunks.cumsum(0).to(torch.int32)
    # chunks covering [0, payload_off): every kept chunk that starts below it
    head = ((bounds[:, :-1] < poff[:, None]) & valid).sum(1)
    return seg_off, seg_len, pkt_seg, head


def plan(args, world, rank):
    """--plan: the distributed plumbing without a GPU (gloo): every rank
    computes its share, rank 0 gathers them and prints one JSON line."""
    import torch.distributed as dist

    first, n, total = frames_for_rank(args.config, args.scaling, rank, world)
    shards = [(first, n)]
    if world > 1:
        dist.init_process_group("gloo")
        shards = [None] * world
        dist.all_gather_object(shards, (first, n))
    if rank == 0:
        print(json.dumps({"plan": True, "n_gpus": world, "scaling": args.scaling,
                          "config": args.config, "total_frames": total,
                          "shards": [list(s) for s in shards]}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak: every rank parses a full batch; strong: the job's frames "
                         "(STRONG_TOTAL, e.g. 64 M for c4) are split over the ranks")
    ap.add_argument("--streams", type=int, default=0,
                    help="streams the steps alternate over (0 = the config's measured best)")
    ap.add_argument("--record", type=int, default=16, choices=(16, 8))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the live host-inclusive (PCIe) measurement")
    ap.add_argument("--no-gate", action="store_true",
                    help="time from host submission (no doorbell-held first launches)")
    ap.add_argument("--stagger-us", type=float, default=None,
                    help="gated, >= 2 streams: stream i starts i * this many us behind "
                         "stream 0 (default: the config's STAGGER_US, else 0)")
    ap.add_argument("--plan", action="store_true",
                    help="print the ranks' shares and exit without touching a GPU")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="INGOT_TUNE_* knob for this run, e.g. slow_path=1 (A/B and "
                         "profiling of variants; results never depend on it)")
    ap.add_argument("--cpu-budget", type=float, default=1.5)
    ap.add_argument("--rotate-mib", type=int, default=512,
                    help="minimum bytes of distinct arenas rotated across steps")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N>1 on one GPU")
    args = ap.parse_args()
    if args.streams <= 0:
        args.streams = STREAMS.get(args.config, 2)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    # --- one process per GPU: under a launcher (WORLD_SIZE set) its world
    # must be --gpus; without one, start the ranks here (nothing has touched
    # a GPU yet in this process) ---
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
        world, rank, local = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
            sys.exit(2)
    if args.plan:
        plan(args, world, rank)
        return

    import torch
    import torch.distributed as dist

    import ingot_amd
    from ingot_amd import Chain, GenProfile

    from ingot_amd import dist as idist

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

    prof_name, _, stride, chain_name, desc = CONFIGS[args.config]
    profile, chain = GenProfile[prof_name], Chain[chain_name]
    ctx = ingot_amd.Context(local)
    from ingot_amd import abi

    for kv in args.tune:
        k, v = kv.split("=")
        ctx.set_tuning(getattr(abi, f"TUNE_{k.upper()}"), int(v))
    lib = ingot_amd.load_library()
    mode = MODES.get(args.config, "parse")
    flows = mode == "flows"

    # --- data: this rank's share (pure in (seed, index)) + R copies ---
    first, n, n_total = frames_for_rank(args.config, args.scaling, rank, world)
    arena, off, lens = ingot_amd.gen_frames(profile, n, first=first, stride=stride,
                                            device=local)
    if flows:
        args.no_variants = True
    # >= 512 MiB of distinct arenas (the 256 MiB MALL cannot serve a step from
    # the previous one), and a copy per stream in flight (launches running
    # together never read the same bytes) — up to ROTATE_CAP_BYTES; above it
    # (a 50 GB strong-scaling arena is far past every cache) one copy, and
    # only single-stream variants
    need = max(1, -(-(args.rotate_mib << 20) // arena.numel()))
    # (config 5's runner rotates its histograms with the arenas: >= 4)
    reps = max(need, args.streams, 4 if flows or not args.no_variants else 1)
    multi_stream_variants = True
    if arena.numel() * reps > ROTATE_CAP_BYTES:
        reps = max(need, args.streams)
        multi_stream_variants = False
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device=dev) for _ in range(reps)]
    torch.cuda.synchronize(dev)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                  for _ in range(max(3, args.streams - 1))]

    if flows:
        hists = [torch.zeros(FLOW_BINS, dtype=torch.int32, device=dev) for _ in range(reps)]
        flow_ids = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(reps)]
    recs0 = None
    if mode == "read":
        # mblk-style packets over the same frames (chunks inside each frame)
        recs0 = ingot_amd.records_to_numpy(
            ctx.parse_strided(arena, stride, n, chain) if stride is not None else
            ctx.parse(arena, off, lens, chain))
        rlens = lens if lens is not None else torch.full((n,), stride, dtype=torch.int32,
                                                         device=dev).to(torch.uint16)
        seg_off, seg_len, pkt_seg, head_chunks = read_chunks(
            torch, off, stride, rlens.to(torch.int32), recs0, READ_CHUNKS[args.config], dev)

    def runner(nstreams, record, flows_only=False, dense=False):
        if flows:
            return FlowRunner(torch, lib, ctx, chain, n, arenas, off, lens, hists, flow_ids,
                              streams[:nstreams], idist.reduce_histogram_async, flows_only)
        if mode == "modify":
            return ModifyRunner(torch, lib, ctx, chain, n, stride, arenas, off, lens,
                                streams[:nstreams])
        if mode == "packed":
            return PackedRunner(torch, lib, ctx, chain, n, arenas, lens, outs,
                                streams[:nstreams])
        if mode == "read":
            return ReadRunner(torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg,
                              outs, streams[:nstreams], dense)
        return Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs,
                      streams[:nstreams], record)

    if mode in ("modify", "read", "packed") and args.record == 8:
        ap.error("8-B records are not offered for this config")
    if chain == Chain.GeneveOverV6Tunnel and args.record == 8:
        ap.error("8-B records are not offered for the tunnel chain (include/ingot_gpu.h)")
    # the doorbell gate needs every launch of the region to be asynchronous:
    # the gloo rehearsal's histogram reduce copies through the host
    gate = None
    gate_note = "off (--no-gate)"
    if not args.no_gate and not (flows and world > 1 and args.dist_backend == "gloo"):
        try:
            stagger = (args.stagger_us if args.stagger_us is not None
                       else STAGGER_US.get(args.config, 0.0))
            gate = Gate(ingot_amd, ctx, stagger)
            gate_note = (f"first {Gate.HOLD} launches held behind a doorbell "
                         "(ingot_gpu_doorbell_wait); region from the first step's start")
            if stagger and args.streams > 1:
                gate_note += (f"; stream i starts i x {stagger:g} us behind stream 0 "
                              "(ingot_gpu_stream_delay), inside the region")
        except RuntimeError as e:
            gate_note = f"unavailable ({e}); region from host submission"
    main_run = runner(args.streams, args.record)
    main_run.run(args.warmup, gate)

    # --- timed region: K steps, barrier + sync on both sides ---
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ms_region, wall = main_run.run(args.steps, gate)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_sec = idist.max_over_ranks(ms_region / 1e3, device=dev)
    # every rank's frames: weak = n per rank; strong = the job's total
    frames_all = n_total
    value = frames_all * args.steps / t_sec / 1e6
    ms_step = t_sec * 1e3 / args.steps
    ungated = None
    if gate is not None:  # the same region timed from host submission, for reference
        ms_u, _ = main_run.run(args.steps)
        ungated = round(idist.max_over_ranks(ms_u / 1e3, device=dev) * 1e3 / args.steps, 5)

    # --- algorithmic bytes from this batch's records (16-B form) ---
    recs = ctx.parse_strided(arenas[0], stride, n, chain, lens=lens) \
        if stride is not None else ctx.parse(arenas[0], off, lens, chain)
    torch.cuda.synchronize(dev)
    recs_np = ingot_amd.records_to_numpy(recs)
    lens_np = lens.cpu().numpy() if lens is not None else None
    if mode == "read":
        # the header chunks read like a frame of the header span's length;
        # descriptors: pkt_seg (4 B) + (u64 off, u16 len) per header chunk
        hc = head_chunks.cpu().numpy().astype(np.int64)
        rd, wr = algorithmic_bytes(recs_np, recs_np["payload_off"], 0, 4 + 10 * hc, 16)
    elif mode == "packed":
        # descriptors: the u16 length, read by the parse and once more by the
        # tile-sum pass; tile sums and bases: 12 B per 64 packets
        rd, wr = algorithmic_bytes(recs_np, lens_np, 0, 2, args.record)
        rd += 2 * n + 12 * ((n + 63) // 64)
    else:
        rd, wr = algorithmic_bytes(recs_np, lens_np, stride or 0, 0 if stride else 10,
                                   args.record)
    step_rd, step_wr = rd, wr
    if flows:
        # the dominant kernel (parse + hash): the frames in, a 4-B flow id per
        # packet out; the whole step adds the histogram pass (flow ids read
        # once, 65,536 x u32 written)
        wr = 4 * n
        step_rd, step_wr = rd + 4 * n, 4 * n + FLOW_BINS * 4
    if mode == "modify":  # no records; the 2 rewritten bytes per packet
        wr = step_wr = 2 * n
    bytes_launch = rd + wr
    pipelined_gbs = (step_rd + step_wr) / (ms_step / 1e3) / 1e9
    # Roofline of the kernel itself: a single-stream pass (launches back to
    # back, so region/K = one launch incl. the dependent-launch boundary; this
    # is what rocprofv3's per-dispatch mean measures).  In the pipelined
    # schedule two launches overlap, so per-dispatch durations are not per-step.
    # Its own floor of warm-up and launches, so that a short run (--steps 1
    # --warmup 0) does not report a cold single launch as the kernel's rate.
    iso = runner(1, args.record, flows_only=True)
    iso.run(max(10, min(args.warmup, 50)))
    iso_steps = max(20, min(args.steps, 1000))
    ms_iso, _ = iso.run(iso_steps, gate)
    launch_ms = ms_iso / iso_steps
    achieved = bytes_launch / (launch_ms / 1e3) / 1e9
    ok_frac = float((recs_np["status"] == 0).mean())
    # the multi-tile ring kernels serve slot rings without a length array
    # (launch_parse / launch_modify in parse.hip); everything else is k_parse
    ring = (mode in ("parse", "modify") and stride is not None and stride >= 64
            and lens is None and chain != Chain.GeneveOverV6Tunnel)
    family = kernel_family(mode, ring)
    sha = kernel_sources_sha()
    traffic = None
    t, pf = (pmc_for(args.config, family, sha, n) if args.record == 16 and not args.tune
             else (None, None))
    if t is not None:
        traffic = {"bytes_per_launch": t["traffic_bytes_per_launch"],
                   "ratio_to_algorithmic": round(t["traffic_bytes_per_launch"] / bytes_launch, 4),
                   "source": f"{pf.relative_to(ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + "
                             "WRITE_SIZE, separate passes, same kernel sources)",
                   "kernel": t.get("kernel")}

    # --- variants (outside the timed region; same data) ---
    variants = {}
    if not args.no_variants:
        vsteps = min(args.steps, 1000)
        for ns, rb in ((1, 16), (2, 8), (1, 8), (4, 16)):
            if (ns, rb) == (args.streams, args.record):
                continue
            if ns > 1 and not multi_stream_variants:
                continue
            if rb == 8 and (chain == Chain.GeneveOverV6Tunnel or mode != "parse"):
                continue
            r = runner(ns, rb)
            r.run(min(args.warmup, 50))
            ms, _ = r.run(vsteps, gate)
            bpl = rd + (rb * n if mode != "modify" else wr)
            variants[f"streams{ns}_rec{rb}"] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3),
                "hbm_GBps": round(bpl / (ms / vsteps / 1e3) / 1e9, 1),
            }
        if mode == "read":  # the same chunks as one dense 8-B entry each
            r = runner(args.streams, 16, dense=True)
            r.run(min(args.warmup, 50))
            ms, _ = r.run(vsteps, gate)
            variants[f"streams{args.streams}_dense_table"] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3)}

    host_path = None
    if (world == 1 and mode == "parse" and args.record == 16 and not args.no_host_path
            and not args.tune):
        host_path = host_inclusive_live(torch, ingot_amd, ctx, arenas[0], off, lens, stride,
                                        chain, n)

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
                ps = pkt_seg[:m + 1].cpu().numpy().view(np.uint32)
                ns_ = int(ps[-1])
                segs = (seg_off[:ns_].cpu().numpy().view(np.uint64),
                        seg_len[:ns_].to(torch.int32).cpu().numpy().astype(np.uint16), ps)
            cpu = cpu_baseline(a_np, o_np, l_np, stride or 0, m, chain, args.cpu_budget,
                               mode="parse" if flows else mode, segs=segs)
        kname = {"modify": ", parse + setters",
                 "read": ", LAYOUT_SEGMENTED (parse_read)",
                 "packed": ", LAYOUT_PACKED + k_tile_sums/k_group_scan",
                 "flows": ", OUT_FLOWS16 (parse + Toeplitz hash; the step adds "
                          "k_flow_count16 / k_flow_reduce16)"}.get(mode, "")
        result = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 5),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-generated, seed 20250808)",
            "config": {
                "workload": desc,
                "frames_per_gpu": n,
                "frames_total": n_total,
                "chain": chain_name,
                "layout": f"strided {stride} B" if stride else "packed, u64 offsets + u16 lengths",
                "record_bytes": args.record,
                "streams": args.streams,
                "arena_copies_rotated": reps,
                "parallelism": (f"{args.scaling} scaling, contiguous share per GPU x{world}" +
                                (f"; {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} "
                                 f"all-reduce (sum) of the {FLOW_BINS} x u32 flow "
                                 "histogram every step" if flows else
                                 " (no data-path collective)")),
                "ok_fraction": round(ok_frac, 6),
                "timing": gate_note,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic["bytes_per_launch"] if traffic else None,
                "traffic_detail": traffic,
                "kernel": (traffic or {}).get("kernel") or
                          f"{family} (ingot_amd/csrc/parse.hip){kname}",
                "kernel_sources_sha": sha,
                "launch_mean_us": round(launch_ms * 1e3, 3),
                "launch_timing": "single-stream pass, HIP events, region/K",
                "pipelined_GBps": round(pipelined_gbs, 1),
                "pipelined_frac": round(pipelined_gbs / HBM_PEAK_GBS, 4),
                "pipelined_read_frac": round(step_rd / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": bytes_launch,
                "read_bytes_per_launch": rd,
                "write_bytes_per_launch": wr,
                "read_frac": round(rd / (launch_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "frac_of_measured_copy_ceiling": round(achieved / HBM_MEASURED_GBS, 4),
                "read_frac_of_measured_copy_ceiling": round(
                    rd / (launch_ms / 1e3) / 1e9 / HBM_MEASURED_GBS, 4),
            },
            "ms_per_step_ungated": ungated,
            "variants": variants,
            "cpu_baseline": cpu,
            "wall_s_timed_region": round(wall, 4),
            "host_inclusive": host_path,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
