#!/usr/bin/env python3
"""bench.py — device-resident L2/L3/L4 parse throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--config c2|c2m|c2r|c3|c3p|c3r|c3s|c4|c5|c6|c6e] [--streams S] [--record 16|8]

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
(oracle/, "port") on the host cores, rank 0, N=1.  C6e (not a parse config:
ingot's Emit batched, OPTE's outbound encapsulation) reports its own metric:
algorithmic bytes = the payload read + 24 B/packet of descriptors and setter
values, the 74-B outer stack + payload written.
"""
from __future__ import annotations

import argparse
import ctypes
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
    "c6e": ("MIXED", 1 << 23, None, "GenericUlp",
            "C6e (SURVEY 8f-4, ingot's Emit): OPTE outbound encapsulation, 8,388,608 inner "
            "64-1500 B frames per GPU each emitted behind an owned outer Eth / IPv6 / UDP / "
            "Geneve + 1 option stack (74 B) with per-packet setters (IPv6 payload_len, UDP "
            "length, flow-entropy UDP source port, VNI) into a packed destination arena"),
}
# configs that time something other than the batched parse_slice records
MODES = {"c5": "flows", "c2m": "modify", "c3r": "read", "c3p": "packed", "c2r": "read",
         "c6e": "emit"}
EMIT_METRIC = "Mpkt/s device-resident batched Emit (Geneve encapsulation), 64-1500 B inner frames"
# per packet the emit kernel reads: u64 source offset, u16 length, u64
# destination offset, the u16 source port and the u32 VNI of its setters
EMIT_DESC_BYTES = 8 + 2 + 8 + 2 + 4
# parse_read chunking: "split2" = header span | payload; "per_header" = one
# chunk per parsed header, then the payload (the reference bench's shape)
READ_CHUNKS = {"c3r": "split2", "c2r": "per_header"}
# parse_read configs timed with chunk 0's descriptor per packet (the mblk
# chain's head, which a packet ring carries: ingot_gpu_parse_read_first).
# c3r: 604 -> 567 us per step (round 4); c2r (one chunk per header, widened
# into chunk 0's window) gains nothing from it (18.2 vs 18.8 us, round 3), so
# it times the chunk table.
READ_FIRST = {"c3r"}
# ... and with the chunk bounds loaded only by walks that leave chunk 0 or
# fail in it (INGOT_TUNE_READ_PLAN 17, the header-split shape: every header
# in the mblk head): c3r 562.4 -> 548.7 us per launch, PMC read 176 B per
# packet (profiles/r04_c3r_lazy_bounds_ab.json).
READ_LAZY = {"c3r"}
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
           "c6": 1, "c2r": 2, "c6e": 1}
# Staggered streams (gated regions with >= 2 streams): stream i starts
# i * STAGGER_US behind stream 0 (ingot_gpu_stream_delay), so the streams'
# launches do not ramp up and drain in lockstep.  0 = start together.
# Measured (tools/stagger_ab.py, interleaved, 20-step regions after a 5-step
# warm-up as the driver runs them; history/profiles/r02_stagger_ab.json): C2 12.32-12.38
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


def _read(path):
    try:
        return Path(path).read_text().strip()
    except OSError:
        return None


def host_cpu_share():
    """The CPUs this process may really use: its affinity mask, capped by the
    tightest CPU quota of its cgroup or any ancestor (cgroup v2 `cpu.max`,
    v1 `cpu.cfs_quota_us / cpu.cfs_period_us`).  os.cpu_count() on the GPU
    box reports the whole machine; its share is a quota.  Returns (cpus to
    pin one worker each to, description)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        list(range(os.cpu_count() or 1))
    quota, where = None, None
    paths = {}
    for line in (_read("/proc/self/cgroup") or "").splitlines():
        hid, ctrls, path = line.split(":", 2)
        if hid == "0":
            paths["v2"] = path
        elif "cpu" in ctrls.split(","):
            paths["v1"] = path

    def ancestors(root, path):
        parts = [x for x in path.split("/") if x]
        for k in range(len(parts), -1, -1):
            yield Path(root, *parts[:k])

    cands = []
    if "v2" in paths:
        for d in ancestors("/sys/fs/cgroup", paths["v2"]):
            v = _read(d / "cpu.max")
            if v and not v.startswith("max"):
                q, per = v.split()
                cands.append((int(q) / int(per), str(d / "cpu.max")))
    for root in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        for d in ancestors(root, paths.get("v1", "/")):
            q, per = _read(d / "cpu.cfs_quota_us"), _read(d / "cpu.cfs_period_us")
            if q and per and int(q) > 0:
                cands.append((int(q) / int(per), str(d / "cpu.cfs_quota_us")))
    if cands:
        quota, where = min(cands)
    n = len(aff) if quota is None else max(1, min(len(aff), int(quota)))
    eff = None
    if "v2" in paths:
        eff = _read(Path("/sys/fs/cgroup", *[x for x in paths["v2"].split("/") if x],
                         "cpuset.cpus.effective"))
    return aff[:n], {"host_cpus": os.cpu_count(), "affinity_cpus": len(aff),
                     "cpu_quota": None if quota is None else round(quota, 3),
                     "cpu_quota_source": where, "cpuset_cpus_effective": eff,
                     "effective_cpus": n}


def physical_core_pick(cpus, want):
    """One CPU per physical core among `cpus` (SMT siblings dropped: a
    sibling shares its core's pipelines), all in ONE socket (the package of
    the first allowed CPU, or the one with the most cores if that has fewer
    than `want`: the sample's memory is then local to every worker), spread
    round-robin over that socket's L3 domains (CCDs) so that workers do not
    crowd one CCD's cache, up to `want`.  Returns (picked cpus,
    description).  Falls back to `cpus` in order when sysfs has no
    topology."""
    def rd(c, rel):
        return _read(f"/sys/devices/system/cpu/cpu{c}/{rel}")

    cores, order = {}, []
    for c in cpus:
        pkg, core = rd(c, "topology/physical_package_id"), rd(c, "topology/core_id")
        if pkg is None or core is None:
            return list(cpus[:want]), {"topology": "unavailable"}
        key = (pkg, rd(c, "topology/die_id"), core)
        if key not in cores:
            cores[key] = (c, rd(c, "cache/index3/id") or pkg)
            order.append(key)
    per_pkg = {}
    for key in order:
        per_pkg.setdefault(key[0], []).append(key)
    pkg = order[0][0]
    if len(per_pkg[pkg]) < want:
        pkg = max(per_pkg, key=lambda k: len(per_pkg[k]))
    order = per_pkg[pkg]
    by_l3 = {}
    for key in order:
        c, l3 = cores[key]
        by_l3.setdefault(l3, []).append(c)
    picked, queues = [], [list(v) for v in by_l3.values()]
    while len(picked) < want and any(queues):
        for q in queues:
            if q and len(picked) < want:
                picked.append(q.pop(0))
    used_l3 = {cores[k][1] for k in order if cores[k][0] in picked}
    return picked, {"topology": "sysfs", "socket": pkg, "sockets_available": len(per_pkg),
                    "physical_cores_available": len(cores),
                    "physical_cores_in_socket": len(order),
                    "physical_cores_used": len(picked), "l3_domains_used": len(used_l3),
                    "smt_siblings_skipped": len(cpus) - len(cores)}


def _cgroup_cpu_stat():
    """cgroup v2 cpu.stat of this process's cgroup: usage_usec (every process
    in it), nr_throttled, throttled_usec ({} when unavailable)."""
    paths = []
    for line in (_read("/proc/self/cgroup") or "").splitlines():
        hid, _, path = line.split(":", 2)
        if hid == "0":
            paths.append(Path("/sys/fs/cgroup", *[x for x in path.split("/") if x], "cpu.stat"))
    paths.append(Path("/sys/fs/cgroup/cpu.stat"))
    for p in paths:
        st = _read(p)
        if st:
            out = {}
            for kv in st.splitlines():
                k, _, v = kv.partition(" ")
                if k in ("usage_usec", "nr_throttled", "throttled_usec") and v.isdigit():
                    out[k] = int(v)
            if out:
                return out
    return {}


CPU_WORKERS = 0  # bench.py --cpu-workers: workers of the all-core baseline (0 = quota - 1)
CLEAN_SHARE = 0.9  # a run is clean when its workers got >= this share of their cores
RUNS_PER_PLACEMENT = 5  # up to this many runs per placement, until 3 are clean


def cpu_baseline(arena_np, off_np, lens_np, stride, n, chain, budget_s=1.5, mode="parse",
                 segs=None, workers=None):
    """Time the oracle (the C restatement of ingot's parse) on the host's
    cores over a bounded sample of the workload, bounded in time.  Each
    worker repeats its contiguous share of the sample `passes` times per
    call, so thread start-up is amortised; a share is then cache-resident
    after the first pass — generous to the CPU.

    Placements (name the cause of a low CPU share, compare 8
    workers with 15): W workers = one per physical core of the allowed set,
    one short of the cgroup CPU quota (host_cpu_share: not os.cpu_count(),
    which on the GPU box counts the whole machine) either pinned one per
    physical core of one socket ("pinned") or left to the scheduler within
    the process's affinity mask ("free"), and 8 pinned workers.  Each
    placement runs until 3 of its runs are clean (the workers got >=
    CLEAN_SHARE of their cores' time) or RUNS_PER_PLACEMENT runs.  Every run
    records the CPU the whole cgroup used (cpu.stat usage_usec: this
    process's workers plus anything else charged to the quota) and its
    throttled time, which name the cause of a low share.  The value is the
    median of the clean runs of the placement with the highest such median;
    with no placement clean 3 times, the median of all runs of the W-worker
    pinned placement, labelled contended.
    mode "read": parse_read over `segs` = (seg_off, seg_len, pkt_seg);
    "modify": parse + the same setter in place."""
    import ctypes
    import resource

    import oracle
    from ingot_amd import EditOp, Field

    lib, arch = _native_oracle(oracle)

    def one_call(t):
        if mode == "read":
            oracle.parse_read_batch(arena_np, *segs, chain, lib=lib, nthreads=t)
        elif mode == "modify":
            oracle.parse_modify_batch(arena_np, off_np, lens_np, chain,
                                      [(2, Field.UDP_DESTINATION, EditOp.SUB, 1)], stride=stride,
                                      n=n, lib=lib, nthreads=t)
        elif mode == "emit":
            hdr, sets, dst_np, dst_off = emit_args
            oracle.emit_batch(hdr, sets, arena_np, off_np, lens_np[:n], dst_np, dst_off,
                              nthreads=t, lib=lib)
        else:
            oracle.parse_batch(arena_np, off_np, lens_np, chain, stride=stride, n=n,
                               nthreads=t, lib=lib)

    allowed, share = host_cpu_share()
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else allowed
    want = len(allowed)
    if share["cpu_quota"] is not None and share["cpu_quota"] < len(aff):
        want = max(1, min(len(allowed), int(share["cpu_quota"]) - 1))
    workers = CPU_WORKERS if workers is None else workers
    if workers:
        want = max(1, min(want, int(workers)))
    cpus, topo = physical_core_pick(aff, want)
    cpus8, _ = physical_core_pick(aff, min(8, want))
    main_aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    # the sample's pages first-touched by this thread on the pinned socket
    if main_aff is not None:
        os.sched_setaffinity(0, cpus)
    arena_np = np.array(arena_np, copy=True)
    off_np = None if off_np is None else np.array(off_np, copy=True)
    lens_np = None if lens_np is None else np.array(lens_np, copy=True)
    if segs is not None:
        segs = tuple(np.array(x, copy=True) for x in segs)
    emit_args = None
    if mode == "emit":  # C6e's stack and setters; the packed destination (first-touched here)
        hdr, sets = emit_stack()
        ports, vnis = emit_values(n)
        sets = [sets[0], sets[1], (*sets[2], ports), (*sets[3], vnis)]
        ln = lens_np[:n].astype(np.int64) + len(hdr)
        dst_off = np.cumsum(ln) - ln
        emit_args = (hdr, sets, np.zeros(int(ln.sum()) + 64, np.uint8), dst_off)

    def place(pin):
        """pin: CPUs to pin worker t to (t mod len), or None = free within
        the process's affinity mask."""
        if pin is None:
            lib.oracle_set_affinity(None, 0)
            if main_aff is not None:
                os.sched_setaffinity(0, main_aff)
        else:
            arr = (ctypes.c_int * len(pin))(*pin)
            lib.oracle_set_affinity(ctypes.cast(arr, ctypes.c_void_p), len(pin))
            if main_aff is not None:
                os.sched_setaffinity(0, pin)

    def measure(t, budget):
        lib.oracle_set_passes(1)
        one_call(t)  # warm (page faults, thread stacks)
        t0 = time.perf_counter()
        one_call(t)
        once = max(time.perf_counter() - t0, 1e-6)
        passes = max(1, min(10000, int(budget / 4 / once)))
        lib.oracle_set_passes(passes)
        ru0, cg0 = resource.getrusage(resource.RUSAGE_SELF), _cgroup_cpu_stat()
        calls, t0 = 0, time.perf_counter()
        while True:
            one_call(t)
            calls += 1
            el = time.perf_counter() - t0
            if el > budget:
                break
        ru1, cg1 = resource.getrusage(resource.RUSAGE_SELF), _cgroup_cpu_stat()
        own = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        d = {k: cg1[k] - cg0[k] for k in cg1 if k in cg0}
        cg = d.get("usage_usec")
        return {"mpkt_s": calls * passes * n / el / 1e6, "passes": calls * passes, "wall_s": el,
                # CPU time the workers obtained per wall second and worker
                # (< 1: descheduled — other load on their cores, or the quota)
                "share": round(own / (el * t), 3),
                "cgroup_cpus": None if cg is None else round(cg / 1e6 / el, 2),
                "others_cpus": None if cg is None else round((cg / 1e6 - own) / el, 2),
                "throttled_ms": (round(d["throttled_usec"] / 1e3, 1)
                                 if "throttled_usec" in d else None),
                "nr_throttled": d.get("nr_throttled")}

    placements = [("pinned", len(cpus), cpus), ("free", len(cpus), None)]
    if len(cpus8) < len(cpus):
        placements.append(("pinned", len(cpus8), cpus8))
    results = []
    try:
        place(cpus)
        single = measure(1, budget_s / 3)
        for name, t, pin in placements:
            place(pin)
            runs = []
            while len(runs) < RUNS_PER_PLACEMENT:
                runs.append(measure(t, budget_s / 3))
                if sum(1 for r in runs if r["share"] >= CLEAN_SHARE) >= 3:
                    break
            results.append((name, t, runs))
    finally:
        lib.oracle_set_passes(1)
        lib.oracle_set_affinity(None, 0)
        if main_aff is not None:
            os.sched_setaffinity(0, main_aff)

    def med(xs):
        xs = sorted(xs)
        return xs[len(xs) // 2] if xs else None

    table = []
    for name, t, runs in results:
        clean = [r["mpkt_s"] for r in runs if r["share"] >= CLEAN_SHARE]
        table.append({"placement": f"{t} {name}", "workers": t, "runs": len(runs),
                      "clean": len(clean), "clean_median": med(clean),
                      "median_all": med([r["mpkt_s"] for r in runs]),
                      "share_median": med([r["share"] for r in runs]),
                      "others_cpus_median": med([r["others_cpus"] for r in runs
                                                 if r["others_cpus"] is not None]),
                      "throttled_ms": sum(r["throttled_ms"] or 0 for r in runs)})
    ok = [row for row in table if row["clean"] >= 3]
    if ok:
        pick = max(ok, key=lambda row: row["clean_median"])
        value, label = pick["clean_median"], (f"clean: median of {pick['clean']} clean runs of "
                                             f"{pick['runs']}, {pick['placement']} workers")
    else:
        pick = table[0]
        value, label = pick["median_all"], (f"contended: median of all {pick['runs']} runs, "
                                           f"0-2 clean, {pick['placement']} workers")
    # the measured cause of a low share: charged to the quota by others in
    # the cgroup (throttling), or the cores shared with load outside it
    thr = sum(row["throttled_ms"] for row in table)
    others = med([row["others_cpus_median"] for row in table
                  if row["others_cpus_median"] is not None])
    lows = [row for row in table if (row["share_median"] or 0) < CLEAN_SHARE]
    if not lows:
        cause = "none: every placement's workers got their cores"
    elif thr > 0:
        cause = (f"cgroup quota throttling ({thr:.0f} ms throttled; others in the cgroup "
                 f"used {others} CPUs)")
    elif others is not None:
        cause = (f"load outside this cgroup on the same cores: not throttled, others in the "
                 f"cgroup used {others} CPUs, workers got {lows[0]['share_median']} of theirs")
    else:
        cause = "unmeasured (no cgroup cpu.stat)"
    what = {"parse": "parse_slice", "read": "parse_read", "modify": "parse + set_destination",
            "emit": "Emit of the outer stack + payload copy"}
    return {
        "value": round(value, 3), "unit": "Mpkt/s", "cores": pick["workers"], "kind": "port",
        "sample": (f"{label}; {n} frames of the workload, C port of ingot "
                   f"{what.get(mode, mode)} (oracle/, -march={arch})"),
        "single_core_value": round(single["mpkt_s"], 3),
        "contention": cause,
        "placements": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}
                       for row in table],
        "detail": {
            "clean_share_threshold": CLEAN_SHARE,
            "runs": {row["placement"]: [{k: (round(v, 3) if isinstance(v, float) else v)
                                         for k, v in r.items()} for r in runs]
                     for row, (_, _, runs) in zip(table, results)},
            "single_core_share": single["share"], "cpu_model": _cpu_model(), **share, **topo,
            "passes_note": "each worker repeats its share of the sample; cache-resident after "
                           "the first pass"},
    }


_NATIVE_ORACLE = []


def _native_oracle(oracle):
    """The oracle built -march=native for this host (once per process, into a
    scratch dir), or the prebuilt x86-64-v3 one if that build fails."""
    if not _NATIVE_ORACLE:
        try:
            d = Path(os.environ.get("TMPDIR", "/tmp")) / f"ingot_oracle_native_{os.getpid()}"
            _NATIVE_ORACLE.append((oracle.load(oracle.build(out_dir=d, native=True)), "native"))
        except Exception as e:  # noqa: BLE001
            log(f"[bench] native oracle build failed ({e}); using the prebuilt x86-64-v3 one")
            _NATIVE_ORACLE.append((oracle.load(), "x86-64-v3"))
    return _NATIVE_ORACLE[0]


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class Runner:
    """Launches step k (arena k % R -> records k % len(outs)) on stream k % S."""

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
                                       outptrs[k % len(outptrs)], sps[k % ns])
        else:
            fn = lib.ingot_gpu_parse if record_bytes == 16 else lib.ingot_gpu_parse_compact
            self.launch = lambda k: fn(h, aptrs[k % reps], optr, lptr, n, c,
                                       outptrs[k % len(outptrs)], sps[k % ns])

    def run(self, steps, gate=None):
        """Time `steps` launches (see _timed)."""
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


def ring_group(steps: int, cap: int = 64) -> int:
    """Batches per ring launch: the largest divisor of `steps` up to `cap`
    (INGOT_RING_MAX_BATCHES), so every launch of a run covers the same
    number of batches and rocprofv3's per-dispatch mean of k_parse_ring is
    the launch the line's roofline divides by (20 steps: one launch of 20)."""
    steps = max(1, int(steps))
    return max(d for d in range(1, min(cap, steps) + 1) if steps % d == 0)


class HalfOffsetRunner:
    """Per-batch launches over two streams without a stagger wait: stream 0
    parses batches 0, 2, 4, ...; stream 1 opens with the first half of batch
    1, parses 3, 5, ..., and closes with batch 1's second half.  Both streams
    start at once yet run half a launch apart (stream 1's first kernel is half
    as long), and both end together (each carries 10 batches of a 20-step
    region) — no stretch where one stream runs alone, which the staggered
    start pays at both ends of the region.  Every step is still one batch's
    full pass (batch 1's as two half launches); batch k reads arena k % R and
    writes record buffer k % R."""

    def __init__(self, torch, lib, ctx, chain, n, stride, arenas, outs, streams, record_bytes):
        self.torch, self.streams = torch, list(streams[:2])
        assert len(self.streams) == 2
        self.reps = len(arenas)
        h, c = ctx._h, int(chain)
        fn = lib.ingot_gpu_parse_strided if record_bytes == 16 else \
            lib.ingot_gpu_parse_strided_compact
        aptrs = [a.data_ptr() for a in arenas]
        optrs = [o.data_ptr() for o in outs]
        sps = [st.cuda_stream for st in self.streams]
        half = n // 2
        self._go = lambda s, b, lo, cnt: fn(h, aptrs[b % self.reps] + lo * stride, stride, None,
                                             cnt, c, optrs[b % self.reps] + lo * record_bytes,
                                             sps[s])
        self.n, self.half = n, half

    def plan(self, steps):
        """[(stream, batch, first frame, frames)] in enqueue order."""
        if steps < 2:
            return [(0, b, 0, self.n) for b in range(steps)]
        even = list(range(0, steps, 2))
        odd = list(range(3, steps, 2))
        s1 = [(1, 1, 0, self.half)] + [(1, b, 0, self.n) for b in odd] + \
            [(1, 1, self.half, self.n - self.half)]
        s0 = [(0, b, 0, self.n) for b in even]
        out = []
        for i in range(max(len(s0), len(s1))):
            if i < len(s1):
                out.append(s1[i])
            if i < len(s0):
                out.append(s0[i])
        return out

    def run(self, steps, gate=None):
        pl = self.plan(steps)
        return _timed(self.torch, self.streams, lambda i: self._go(*pl[i]), len(pl), gate=gate)


class RingRunner:
    """The persistent ring consumer (ingot_gpu_parse_ring): steps k .. k+G-1
    are one launch per stream, stream s taking batches k+s, k+s+S, ... of the
    group; batch k reads arena k % R and writes its own record buffer
    k % len(outs) (every batch's records are stored inside the region)."""

    def __init__(self, torch, lib, ctx, chain, n, stride, arenas, outs, streams, record_bytes,
                 group):
        import ctypes

        import ingot_amd

        if not isinstance(streams, (list, tuple)):
            streams = [streams]
        self.torch, self.streams, self.group = torch, list(streams), group
        reps, nout = len(arenas), len(outs)
        h, c = ctx._h, int(chain)
        sps = [st.cuda_stream for st in self.streams]
        S = len(sps)
        aptrs = [a.data_ptr() for a in arenas]
        optrs = [o.data_ptr() for o in outs]
        tables = {}

        def table(first, m):
            """batches first, first+S, ... below the group's end"""
            key = (first % (reps * nout), m)
            if key not in tables:
                t = (ingot_amd.RingBatch * m)()
                for j in range(m):
                    b = first + j * S
                    t[j].d_arena, t[j].d_out = aptrs[b % reps], optrs[b % nout]
                tables[key] = t
            return tables[key]

        def launch(k, m=1):
            for s in range(min(S, m)):
                cnt = len(range(s, m, S))
                rc = lib.ingot_gpu_parse_ring(h, ctypes.cast(table(k + s, cnt), ctypes.c_void_p),
                                              cnt, stride, n, c, record_bytes, None, 0, 0, None,
                                              sps[s])
                if rc:
                    return rc
            return 0

        self.launch = launch

    def run(self, steps, gate=None):
        """Time `steps` batches as launches of `group` batches."""
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate, group=self.group)

    def warm(self, steps, gate=None):
        """Untimed: `steps` rounded up to whole groups (every launch of the
        run the same size)."""
        g = self.group
        return self.run(max(g, -(-steps // g) * g), gate)


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


def emit_stack():
    """C6e's owned outer stack (host serialiser, ingot_amd.emit) and setters:
    OPTE's outbound Geneve encapsulation (ingot-examples/src/packets.rs:27-40)."""
    from ingot_amd import EmitSource, Field
    from ingot_amd import emit as E

    hdr = (E.ethernet(bytes.fromhex("a84025777776"), bytes.fromhex("a84025777777"), 0x86DD)
           + E.ipv6(bytes.fromhex("fd00000000f7010100000000000000" + "02"),
                    bytes.fromhex("fd00000000f7010100000000000000" + "01"), 17, hop_limit=64)
           + E.udp(0, 6081) + E.geneve(0, options=E.geneve_opt(0x0129, 0)))
    sets = [(14, Field.V6_PAYLOAD_LEN, EmitSource.LENGTH, -40),
            (54, Field.UDP_LENGTH, EmitSource.LENGTH, 0),
            (54, Field.UDP_SOURCE, EmitSource.U16, 0),
            (62, Field.GENEVE_VNI, EmitSource.U32, 0)]
    return hdr, sets


def emit_values(n: int, first: int = 0):
    """Per-packet flow-entropy source ports and VNIs (pure in the index)."""
    i = np.arange(first, first + n, dtype=np.uint64)
    h = (i * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(32)
    return ((h & np.uint64(0x3FFF)) | np.uint64(0xC000)).astype(np.uint16), \
        (h >> np.uint64(8) & np.uint64(0xFFFFFF)).astype(np.uint32)


class EmitRunner:
    """C6e: ingot_gpu_emit_packets per step — arena k % R's frames emitted
    behind the owned outer stack into a packed destination arena."""

    def __init__(self, torch, lib, ctx, n, arenas, off, lens, first, streams):
        import ingot_amd

        self.torch, self.streams = torch, streams
        hdr, sets = emit_stack()
        ports, vnis = emit_values(n, first)
        dev = arenas[0].device
        self._vals = [torch.from_numpy(ports.view(np.int16)).to(dev),
                      torch.from_numpy(vnis.view(np.int32)).to(dev)]
        rows = [sets[0], sets[1], (*sets[2], self._vals[0].data_ptr()),
                (*sets[3], self._vals[1].data_ptr())]
        self._sets = ingot_amd.emit_sets_array(rows)
        self._hdr = (ctypes.c_uint8 * len(hdr)).from_buffer_copy(hdr)
        ln = lens.to(torch.int64)
        self.dst_off = torch.cumsum(ln + len(hdr), 0) - (ln + len(hdr))
        # one destination per stream: launches running together never write
        # the same bytes (as the parse runners' record buffers)
        size = int((ln + len(hdr)).sum().item()) + 64
        self.dst = [torch.empty(size, dtype=torch.uint8, device=dev) for _ in streams]
        h, reps = ctx._h, len(arenas)
        aptrs = [a.data_ptr() for a in arenas]
        sp, hp, H = self._sets.ctypes.data, ctypes.addressof(self._hdr), len(hdr)
        optr, lptr = off.data_ptr(), lens.data_ptr()
        dptrs, doptr = [d.data_ptr() for d in self.dst], self.dst_off.data_ptr()
        sps = [s.cuda_stream for s in streams]
        self.launch = lambda k: lib.ingot_gpu_emit_packets(
            h, hp, H, sp, len(rows), aptrs[k % reps], optr, lptr, n, dptrs[k % len(sps)],
            doptr, sps[k % len(sps)])

    def run(self, steps, gate=None):
        return _timed(self.torch, self.streams, self.launch, steps, gate=gate)


class ReadRunner:
    """parse_read over chunk lists: arena k % R with the shared segment tables
    (dense: one (offset << 16) | length entry per chunk,
    ingot_gpu_parse_read_dense)."""

    def __init__(self, torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg, outs,
                 streams, dense=False, first=False):
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
        if first:  # chunk 0 per packet (ingot_gpu_parse_read_first)
            import ingot_amd

            self.first = ingot_amd.first_chunks(seg_off, seg_len, pkt_seg)
            fp = self.first.data_ptr()
            self.launch = lambda k: lib.ingot_gpu_parse_read_first(
                h, aptrs[k % reps], so, sl, ps, fp, n, c, outptrs[k % reps], None, sps[k % ns])
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
                 reduce_fn, flows_only=False, open_before_collective=False):
        """flows_only: launch the parse + hash kernel alone (no histogram, no
        reduce) — the dominant kernel, timed for `roofline`.
        open_before_collective: gate_policy "until_collective" (RCCL at
        N > 1): ring the region's doorbell before the first all-reduce is
        enqueued.  Otherwise ("hold") the gate opens after Gate.HOLD launches
        as in every other config (_timed)."""
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
                # never enqueue a collective behind an unrung doorbell
                # (gate_policy "until_collective"): ring it first
                if self._gate is not None and open_before_collective:
                    self._gate.open()
                w = reduce_fn(hist)
            if w is not None:
                works[k] = w
            return rc

        def finish():
            with torch.cuda.stream(self.streams[0]):
                for k in sorted(works):
                    works.pop(k).wait()

        self.launch, self.finish = launch, finish
        self._gate = None

    def run(self, steps, gate=None):
        self._gate = gate
        try:
            return _timed(self.torch, self.streams, self.launch, steps, self.finish, gate=gate)
        finally:
            self._gate = None


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

    # the region's timing events: HipEvent (no system fence) unless
    # FENCED_EVENTS (bench.py --fenced-events: torch's default events)
    FENCED_EVENTS = False

    def event(self):
        if self.FENCED_EVENTS:
            import torch

            return torch.cuda.Event(enable_timing=True)
        return HipEvent()


class HipEvent:
    """A timing-only HIP event created with hipEventDisableSystemFence
    (hip_runtime_api.h: for events "only being used to measure timing"; on
    AMD GPUs it avoids the cache writeback + invalidation a default event's
    record performs, and that work's delay of the launch that follows it).
    Recorded on a torch stream; read after a device synchronize.  The work
    between two such events is unchanged — only the measurement's own fence
    at the region's edges goes."""

    FLAGS = 0x20000000  # hipEventDisableSystemFence
    _lib = None

    @classmethod
    def lib(cls):
        if cls._lib is None:
            import ctypes

            # the HIP runtime torch already loaded (its streams are the ones
            # recorded on), never a second copy from another path
            path = "libamdhip64.so"
            with open("/proc/self/maps") as f:
                for line in f:
                    if "libamdhip64.so" in line and "/" in line:
                        path = line[line.index("/"):].strip()
                        break
            cls._lib = ctypes.CDLL(path)
        return cls._lib

    def __init__(self):
        import ctypes

        self._c = ctypes
        self.h = ctypes.c_void_p()
        rc = self.lib().hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(self.FLAGS))
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: {rc}")

    def record(self, stream):
        rc = self.lib().hipEventRecord(self.h, self._c.c_void_p(stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: {rc}")

    def elapsed_time(self, other):
        ms = self._c.c_float()
        rc = self.lib().hipEventElapsedTime(self._c.byref(ms), self.h, other.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime: {rc}")
        return ms.value

    def __del__(self):
        try:
            self.lib().hipEventDestroy(self.h)
        except Exception:
            pass


def _timed(torch, streams, launch, steps, finish=None, gate=None, group=1):
    """Run `steps` steps; returns (ms, wall s).  Every stream stamps a
    start event before its first launch and an end event after its last one;
    the region is the earliest start to the latest end (all on the device
    clock).  Ungated, the other streams fork from streams[0]'s start event;
    gated, every stream waits on the doorbell instead.  No stream joins
    another at the end: a cross-stream event wait costs ~7 us of device time
    that would land inside the region (tools/region_probe.py).  group > 1:
    launch(k, m) runs steps k .. k+m-1 (the ring consumer)."""
    s0 = streams[0]
    w0 = time.perf_counter()
    # gated regions: the gate's timing events (Gate.event: timing-only HIP
    # events); ungated: torch's (the other streams wait on the start event)
    mk_event = getattr(gate, "event", None) or (lambda: torch.cuda.Event(enable_timing=True))
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
                e = mk_event()
                e.record(s)
                starts.append(e)
        held = 0
        for k in range(0, steps, group):
            rc = launch(k) if group == 1 else launch(k, min(group, steps - k))
            if rc:
                raise RuntimeError(f"launch failed: {rc}")
            held += 1
            if gate is not None and held == Gate.HOLD:
                gate.open()
        if finish is not None:
            finish()
        for s in streams:
            e = mk_event()
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
    on these exact sources (tools/pmc_traffic.py records the same digest).
    Comments and whitespace are left out, so a documentation edit does not
    detach the profiles; any code change does."""
    import hashlib
    import re

    h = hashlib.sha256()
    files = sorted((ROOT / "ingot_amd" / "csrc").glob("*")) + sorted((ROOT / "include").glob("*.h"))
    for f in files:
        # comm.cpp (the RCCL reduce behind the C ABI) launches no kernel of ours
        if f.suffix in (".hip", ".h", ".cpp") and f.name != "comm.cpp":
            code = re.sub(r"/\*.*?\*/|//[^\n]*", "", f.read_text(), flags=re.S)
            h.update(f.name.encode())
            h.update(re.sub(r"\s+", " ", code).strip().encode())
    return h.hexdigest()[:16]


KERNEL_FILE = {"k_parse_read": "read.hip", "k_flows_bits": "tuple.hip",
               "k_parse_pipe": "ring.hip", "k_modify_pipe": "ring.hip",
               "k_parse_ring": "ring.hip", "k_emit": "emit.hip"}


def kernel_family(mode: str, ring: bool) -> str:
    """The dominant kernel this config launches (parse.hip's dispatch)."""
    if mode == "read":
        return "k_parse_read"
    if mode == "flows":  # offset-addressed frames, 16-bit table (tuple.hip)
        return "k_flows_bits"
    if mode == "emit":
        return "k_emit"
    if mode == "modify":
        return "k_modify_pipe" if ring else "k_parse"
    return "k_parse_pipe" if ring else "k_parse"


def pmc_for(config: str, family: str, sha: str, n: int):
    """The newest profiles/*_pmc_<config>.json taken on these kernel sources,
    over launches of n frames, whose profiled kernel is `family`; None
    otherwise."""
    files = list(ROOT.glob(f"profiles/*_pmc_{config}.json")) + \
        list(ROOT.glob(f"profiles/*_pmc_{config}_ring.json"))
    for f in sorted(files, key=lambda f: f.name, reverse=True):
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


# seconds each teardown step of an N > 1 run may take (bench.teardown)
TEARDOWN_BUDGET_S = 100.0

# --rehearse-one-gpu: RCCL over loopback sockets between ranks sharing a GPU
REHEARSAL_ENV = {"NCCL_P2P_DISABLE": "1", "NCCL_SHM_DISABLE": "1", "NCCL_IB_DISABLE": "1",
                 "NCCL_SOCKET_IFNAME": "lo"}


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


def read_chunks_np(off, stride, lens, recs_np, kind):
    """read_chunks on the host (numpy), for the CPU baseline's sample: the
    same chunk tables (seg_off u64, seg_len u16, pkt_seg u32)."""
    n = len(recs_np)
    L = (lens.astype(np.int64) if lens is not None else np.full(n, stride, np.int64))
    keys = ("payload_off",) if kind == "split2" else ("l3_off", "l4_off", "payload_off")
    cuts = np.stack([recs_np[k].astype(np.int64) for k in keys], 1)
    prev = np.zeros(n, np.int64)
    keep = np.zeros(cuts.shape, bool)
    for k in range(cuts.shape[1]):
        c = cuts[:, k]
        keep[:, k] = (c > prev) & (c < L)
        prev = np.where(keep[:, k], c, prev)
    bounds = np.concatenate([np.zeros((n, 1), np.int64), cuts, L[:, None]], 1)
    valid = np.concatenate([np.ones((n, 1), bool), keep], 1)
    nxt = np.empty_like(bounds[:, :-1])
    run = L.copy()
    for k in range(valid.shape[1] - 1, -1, -1):
        nxt[:, k] = run
        run = np.where(valid[:, k], bounds[:, k], run)
    starts, ends = bounds[:, :-1][valid], nxt[valid]
    nchunks = valid.sum(1)
    base = off.astype(np.int64) if off is not None else np.arange(n, dtype=np.int64) * stride
    seg_off = (np.repeat(base, nchunks) + starts).astype(np.uint64)
    seg_len = (ends - starts).astype(np.uint16)
    pkt_seg = np.zeros(n + 1, np.uint32)
    pkt_seg[1:] = np.cumsum(nchunks)
    return seg_off, seg_len, pkt_seg


def cpu_baseline_first(name: str, budget_s: float):
    """The CPU baseline of config `name`, measured before this process
    touches the GPU (no HIP runtime or torch threads yet): the first
    min(n, 1 M) frames of the batch, generated on the host by the same
    generator (ingot_amd.hostgen — the bytes the device generator writes),
    parsed by the oracle's C port on the host cores (cpu_baseline)."""
    import oracle
    from ingot_amd import Chain, GenProfile
    from ingot_amd.hostgen import gen_frames_host

    prof_name, n, stride, chain_name, _ = CONFIGS[name]
    mode = MODES.get(name, "parse")
    m = min(n, 1 << 20)
    arena, off, lens = gen_frames_host(GenProfile[prof_name], m, stride=stride)
    chain = Chain[chain_name]
    segs = None
    if mode == "read":
        recs = oracle.parse_batch(arena, off, lens, chain, stride=stride or 0, n=m, nthreads=8)
        segs = read_chunks_np(off, stride, lens, recs, READ_CHUNKS[name])
    cpu = cpu_baseline(arena, off, lens, stride or 0, m, chain, budget_s,
                       mode="parse" if mode in ("flows", "packed") else mode, segs=segs)
    cpu["measured"] = "before the process touched the GPU (host-generated sample)"
    return cpu


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


def gate_policy(flows: bool, world: int, backend: str, no_gate: bool) -> str:
    """How the timed region starts.
      "off"   — from host submission: --no-gate, or the gloo rehearsal of
                config 5 at N > 1, whose histogram reduce copies through the
                host (a held stream would block it);
      "until_collective" — config 5 over RCCL (the library's one-rank
                communicator at N = 1, the ranks' at N > 1): launches are held
                behind the doorbell only up to the first collective of the
                region; the runner rings it before issuing any all-reduce, so
                no collective is ever enqueued while a stream of this process
                waits on an unrung doorbell (a held stream would hold RCCL's
                hardware queue too, include/ingot_gpu.h);
      "hold"  — everything else: the first Gate.HOLD launches are held."""
    if no_gate:
        return "off"
    if flows:
        return "off" if backend == "gloo" and world > 1 else "until_collective"
    return "hold"


def jsonable(x, path="line"):
    """The line with numpy scalars / arrays made plain Python (an array is
    named on stderr: it should have been reduced to a number)."""
    if isinstance(x, dict):
        return {k: jsonable(v, f"{path}.{k}") for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [jsonable(v, f"{path}[{i}]") for i, v in enumerate(x)]
    if isinstance(x, np.ndarray):
        log(f"[bench] {path} is an array {x.shape}")
        return x.tolist() if x.size <= 64 else f"<array {x.shape} at {path}>"
    if isinstance(x, np.generic):
        return x.item()
    return x


T_START = time.perf_counter()


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
    ap.add_argument("--timing", default="launches", choices=("ring", "launches"),
                    help="launches (default): one launch per batch over the config's streams "
                         "(c2: 2 streams, the second started 6 us late); ring: the persistent "
                         "ring consumer (ingot_gpu_parse_ring), one launch per group of up to 64 "
                         "batches — measured slower on C2 (DESIGN.md §5: one long-lived launch "
                         "sustains ~5.5 TB/s, two overlapped per-batch launches ~7 TB/s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the live host-inclusive (PCIe) measurement")
    ap.add_argument("--no-sublines", action="store_true",
                    help="c2: skip the sub-lines (--sublines)")
    ap.add_argument("--sublines", default="c3,c4,c5",
                    help="c2: the configs carried as sub-lines of the default line")
    ap.add_argument("--no-gate", action="store_true",
                    help="time from host submission (no doorbell-held first launches)")
    ap.add_argument("--stagger-us", type=float, default=None,
                    help="gated, >= 2 streams: stream i starts i * this many us behind "
                         "stream 0 (default: the config's STAGGER_US, else 0)")
    ap.add_argument("--plan", action="store_true",
                    help="print the ranks' shares and exit without touching a GPU")
    ap.add_argument("--fenced-events", action="store_true",
                    help="time gated regions with torch's default (system-fenced) events "
                         "instead of timing-only HIP events")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="INGOT_TUNE_* knob for this run, e.g. window_indexed=1056 (A/B and "
                         "profiling of variants; results never depend on it)")
    ap.add_argument("--cpu-budget", type=float, default=1.5)
    ap.add_argument("--cpu-workers", type=int, default=0,
                    help="workers of the all-core CPU baseline (0: one short of the CPU quota)")
    ap.add_argument("--rotate-mib", type=int, default=512,
                    help="minimum bytes of distinct arenas rotated across steps")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (default); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--group-backend", default="gloo", choices=("gloo", "nccl"),
                    help="backend of the torch.distributed group at N > 1, which carries only "
                         "control (the communicator id, barriers, max over ranks, checks); "
                         "config 5's reduce is the library's own RCCL communicator either way. "
                         "gloo (default): one RCCL communicator per process; nccl: torch's "
                         "group is a second one (DESIGN.md §6)")
    ap.add_argument("--subline-budget-s", type=float, default=SUBLINE_BUDGET_S,
                    help="N > 1: seconds the sub-lines may take before the line is printed "
                         "without the unfinished ones (SublineGuard)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 ranks on ONE GPU with RCCL: each rank gets its own "
                         "NCCL_HOSTID and the ranks talk over loopback sockets (P2P, SHM, "
                         "InfiniBand off), so RCCL accepts them on one device; the N > 1 path "
                         "runs with real RCCL kernels, the rates mean nothing")
    args = ap.parse_args()
    if args.streams <= 0:
        args.streams = STREAMS.get(args.config, 2)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    subline_names(args)  # a bad --sublines fails before any GPU work
    global CPU_WORKERS
    CPU_WORKERS = args.cpu_workers

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
    if world > 1:
        # a rank that stops making progress shows where, on stderr, every
        # 150 s (a run at N > 1 takes about a minute)
        import faulthandler

        faulthandler.dump_traceback_later(150, repeat=True)
    if args.rehearse_one_gpu and world > 1:
        # before anything initialises RCCL (tests/test_comm_world2.py: the same
        # settings for the product reduce alone)
        os.environ.update(REHEARSAL_ENV)
        os.environ["NCCL_HOSTID"] = f"ingot-rehearsal-rank{rank}"
    # The CPU baselines first, while no GPU runtime or torch thread shares
    # this process's CPU quota: N=1, rank 0.
    args.cpu_pre = {}
    if world == 1 and not args.no_cpu_baseline:
        for name in [args.config] + subline_names(args):
            try:
                args.cpu_pre[name] = cpu_baseline_first(name, args.cpu_budget)
            except Exception as e:  # noqa: BLE001 — fall back to the post-GPU sample
                log(f"[bench] host-generated CPU baseline for {name} failed ({e})")

    import torch
    import torch.distributed as dist

    import ingot_amd

    # one GPU per rank; a --dist-backend gloo rehearsal may fold ranks onto
    # fewer GPUs (e.g. the 1-GPU test box)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        from ingot_amd.dist import _stdout_to_stderr

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL prints a version banner on stdout when a communicator comes up:
        # keep it off the one-line stdout (eager init with device_id, then a
        # barrier, inside the redirect)
        # The group carries control only; config 5's device reduce is the
        # library's communicator.  Over gloo (the default) each process holds
        # one RCCL communicator, not two (the world-2 rehearsal
        # stalled with torch's group on RCCL as well).
        with _stdout_to_stderr():
            if args.dist_backend == "nccl" and args.group_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group("gloo")
            dist.barrier()
    ctx = ingot_amd.Context(local)
    from ingot_amd import abi

    for kv in args.tune:
        k, v = kv.split("=")
        ctx.set_tuning(getattr(abi, f"TUNE_{k.upper()}"), int(v))
    env = (torch, dist, ingot_amd, ingot_amd.load_library(), ctx, world, rank, local, dev)
    result = run_config(args, args.config, env)
    # The metric names 64-1500 B frames, and BASELINE.json names four configs
    # past C2: the default (c2) line carries C3 (configs[2], mixed frames),
    # C4 (configs[3], VLAN/QinQ + IPv6 EHs) and C5 (configs[4], flows +
    # histogram + the RCCL all-reduce at N > 1) as sub-lines, each timed by
    # the same rules with its own roofline and CPU baseline.  C4 and C5 are
    # weak-scaled at 8,388,608 frames per GPU: at N = 8 exactly the 64 M-frame
    # jobs BASELINE.json names.
    done = {}
    guard = None
    if world > 1 and subline_names(args):
        names = subline_names(args)

        def emit_partial():
            log(f"[bench] sub-lines not finished after {args.subline_budget_s:g} s at N = {world}: "
                "printing the line without them")
            if rank == 0 and result is not None:
                result["sublines"] = {k: v for k, v in done.items() if v is not None}
                result["sublines_unfinished"] = {
                    k: f"not finished within {args.subline_budget_s:g} s at N = {world}"
                    for k in names if k not in done}
                result["wall_s_command"] = round(time.perf_counter() - T_START, 2)
                print(json.dumps(jsonable(compact_line(result, args.config))), flush=True)

        # rank 0 (the printer) first: the other ranks outlast it by 5 s, and
        # a collective that fails when rank 0 leaves only waits for their guard
        guard = SublineGuard(args.subline_budget_s + (5.0 if rank else 0.0),
                             emit_partial).start()
    try:
        subs = run_sublines(args, env, run_config, torch.cuda.empty_cache, out=done)
    except Exception as e:  # noqa: BLE001 — only ranks > 0 with a guard, below
        if guard is None or rank == 0:
            raise
        log(f"[bench] rank {rank}: a sub-line failed ({e!r}); the sub-line guard ends the run")
        time.sleep(3600)
    if guard is not None and not guard.finish():
        time.sleep(3600)  # the guard is printing the line and ending the process
    if result is not None and subs is not None:
        result["sublines"] = subs
        result["wall_s_command"] = round(time.perf_counter() - T_START, 2)
    if rank == 0:
        print(json.dumps(jsonable(compact_line(result, args.config))), flush=True)
    teardown(dist, world, getattr(ctx, "_flow_comm", None))


def teardown(dist, world, comm, budget_s=None):
    """End of the run, every step logged on stderr: config 5's communicator,
    then the process group.  At N > 1 each step gets a time budget: the line
    is printed and every rank has passed the final barrier, so a library
    teardown that does not return (seen once in the one-GPU RCCL rehearsal:
    ncclCommDestroy on both ranks) must not turn a finished run into a hung
    one — the process then exits 0 without waiting for it."""
    import threading

    budget = budget_s if budget_s is not None else TEARDOWN_BUDGET_S

    def guarded(what, fn):
        def run():
            try:
                fn()
            except Exception as e:  # noqa: BLE001 — the run is finished; say so and go on
                log(f"[bench] teardown: {what} failed: {e}")
        return run

    def bounded(what, fn):
        t0 = time.perf_counter()
        log(f"[bench] teardown: {what}")
        fn = guarded(what, fn)
        if world <= 1:
            fn()
            return True
        th = threading.Thread(target=fn, daemon=True)
        th.start()
        th.join(budget)
        dt = time.perf_counter() - t0
        if th.is_alive():
            log(f"[bench] teardown: {what} did not return in {dt:.0f} s; exiting without it")
            return False
        log(f"[bench] teardown: {what} took {dt:.2f} s")
        return True

    ok = True
    if world > 1:
        log("[bench] teardown: barrier")
        dist.barrier()
    if comm is not None:
        # every rank's streams have drained: at N > 1 the communicator is
        # released locally (ingot_gpu_comm_abort — the graceful destroy did
        # not return in the one-GPU RCCL rehearsal); at N = 1 gracefully
        if world > 1:
            ok = bounded("ingot_gpu_comm_abort", comm.abort)
        else:
            ok = bounded("ingot_gpu_comm_destroy", comm.close)
    if ok and world > 1:
        ok = bounded("destroy_process_group", dist.destroy_process_group)
    if not ok:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    log("[bench] teardown: done")
    if world > 1:
        import faulthandler

        faulthandler.cancel_dump_traceback_later()


def _summary_entry(line):
    r = line["roofline"]
    c = line.get("cpu_baseline") or {}
    td = r.get("traffic_detail") or {}
    cpu = None
    if c:
        cpu = (f"{c['value']} Mpkt/s, {c['cores']} workers, "
               f"{'clean' if c.get('sample', '').startswith('clean') else 'contended'}")
    return {"Mpkt_s": line["value"], "us_step": round(line["ms_per_step"] * 1e3, 3),
            "kernel_frac": r["frac"], "step_read_frac": r.get("pipelined_read_frac"),
            "traffic_ratio": td.get("ratio_to_algorithmic"), "cpu": cpu}


def _short_cpu(c):
    if not c:
        return None
    out = {k: c.get(k) for k in ("value", "unit", "cores", "kind", "single_core_value")}
    out["sample"] = (c.get("sample") or "")[:110]
    return out


def _short_roofline(r):
    td = r.get("traffic_detail") or {}
    out = {k: r.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")}
    out["traffic_ratio"] = td.get("ratio_to_algorithmic")
    k = r.get("kernel") or ""
    k = k.replace("void ingot_gpu::(anonymous namespace)::", "")
    out["kernel"] = (k.rsplit("(ingot_gpu::", 1)[0] if "(ingot_gpu::" in k else k)[:70]
    for key in ("launch_mean_us", "algorithmic_bytes_per_launch", "read_frac",
                "pipelined_read_frac", "read_frac_records_dram"):
        if r.get(key) is not None:
            out[key] = r[key]
    return out


def _short_line(line, top):
    """One config's line cut to what the record must show; everything is in
    gpurun_out/bench_full.json."""
    keep = (("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
             "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if top else
            ("value", "ms_per_step"))
    out = {k: line.get(k) for k in keep}
    cfg = line.get("config") or {}
    out["config"] = {k: cfg.get(k) for k in (
        ("workload", "frames_per_gpu", "frames_total", "chain", "layout", "record_bytes",
         "streams", "parallelism") if top else ("workload", "frames_per_gpu", "streams"))}
    out["roofline"] = _short_roofline(line["roofline"])
    out["cpu_baseline"] = _short_cpu(line.get("cpu_baseline"))
    d = line.get("distributed") or {}
    chk = d.get("flow_hist_check")
    out["distributed"] = {"world_size": d.get("world_size"), "backend": d.get("backend")}
    if d.get("group"):
        out["distributed"]["group"] = "control only"
    if d.get("rehearsal"):
        out["distributed"]["rehearsal"] = d["rehearsal"]
    if d.get("collective"):
        out["distributed"]["collective"] = d["collective"][:90]
    if chk:
        out["distributed"]["flow_hist_check_ok"] = chk.get("ok")
    if line.get("host_inclusive"):
        h = line["host_inclusive"]
        out["host_inclusive"] = {k: h.get(k) for k in ("frames_per_batch", "memcpy_Mpkt_s",
                                                       "zero_copy_Mpkt_s")}
    return out


def compact_line(result, name):
    """The printed line: every config's numbers cut to the fields the record
    needs (value, ms/step, roofline, CPU baseline, host-inclusive rate,
    collective check), short enough that the driver's stdout tail keeps all
    of it (~8,000 characters); the full result goes to
    gpurun_out/bench_full.json."""
    if result is None:
        return None
    try:
        out_dir = ROOT / "gpurun_out"
        out_dir.mkdir(exist_ok=True)
        (out_dir / "bench_full.json").write_text(json.dumps(jsonable(result), indent=1))
    except OSError:
        pass
    out = _short_line(result, top=True)
    subs = result.get("sublines") or {}
    if subs:
        out["sublines"] = {k: _short_line(v, top=False) for k, v in subs.items() if v is not None}
    summary = {name: _summary_entry(result)}
    v64 = (result.get("variants") or {}).get("streams2_rec16_records64")
    if v64:
        summary["c2_records_1GiB_ring"] = {"us_step": v64["us_per_step"],
                                           "step_read_frac": v64["read_frac"]}
    for k, v in subs.items():
        if v is None:
            continue
        summary[k] = _summary_entry(v)
        pp = (v.get("variants") or {}).get("plain_parse_streams1_rec16")
        if pp:
            summary[k]["over_plain_parse"] = pp["flows_over_plain"]
    if result.get("wall_s_command") is not None:
        out["wall_s_command"] = result["wall_s_command"]
    if result.get("sublines_unfinished"):
        out["sublines_unfinished"] = result["sublines_unfinished"]
    out["summary"] = summary
    out["full"] = "gpurun_out/bench_full.json"
    return out


def subline_names(args) -> list:
    """The configs the default line carries as sub-lines (none for other
    configs, --no-sublines or a --tune run)."""
    if args.config != "c2" or args.no_sublines or args.tune:
        return []
    names = [c for c in args.sublines.split(",") if c]
    bad = [c for c in names if c not in CONFIGS or c == "c2"]
    if bad:
        raise SystemExit(f"--sublines: unknown config(s) {bad}")
    return names


# Sub-line warm-up floor (launches).  The gather-bound configs read 4 arena
# copies of 6.5-13 GB; their first few dozen launches after the allocation
# run 6-8% slower than the steady state (C5 at 20 steps: warm-up 5 -> 333 /
# 331 us per flows launch, frac 0.445 / 0.449; warm-up 50 -> 309 us, 0.480;
# 100 steps after warm-up 5 -> 313 us; tools/sessions/r04_c5_edge.sh,
# profiles/r04_subline_warmup.json).  The main line keeps the driver's W.
SUBLINE_WARMUP = 50


# N > 1: seconds the sub-lines may take, all together, before the line is
# printed without those not finished (SublineGuard)
SUBLINE_BUDGET_S = 150.0


class SublineGuard:
    """At N > 1 the default line's main config (C2, no collective) is
    measured before its sub-lines, and C5's sub-line issues an RCCL
    all-reduce every step.  Should a collective never complete (DESIGN.md
    §6: seen only with two ranks sharing one GPU), the measured line must
    still be printed: after `budget_s` this guard calls `emit` (rank 0 prints
    the line with the sub-lines finished so far) and ends the process with
    status 0.  finish() claims the line for the main thread; False means the
    guard has already fired and is ending the process."""

    def __init__(self, budget_s, emit):
        import threading

        self._lock = threading.Lock()
        self._done = False
        self._emit = emit
        self._timer = threading.Timer(budget_s, self._fire)
        self._timer.daemon = True

    def start(self):
        self._timer.start()
        return self

    def finish(self) -> bool:
        with self._lock:
            if self._done:
                return False
            self._done = True
        self._timer.cancel()
        return True

    def _fire(self):
        with self._lock:
            if self._done:
                return
            self._done = True
        try:
            self._emit()
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)


def run_sublines(args, env, run, release=lambda: None, out=None):
    """Each sub-line is `run(sub_args, name, env)` with the main line's steps,
    a warm-up of max(W, SUBLINE_WARMUP) launches, the config's own stream
    count, 16-B records and no variants or host path; every rank runs them in
    the same order (their barriers and collectives pair up).  Returns
    {name: line} on rank 0, None elsewhere or when there are none; `out`
    (optional) receives each finished line as it completes."""
    names = subline_names(args)
    if not names:
        return None
    out = {} if out is None else out
    for name in names:
        sub = argparse.Namespace(**vars(args))
        sub.config, sub.streams, sub.record, sub.timing = name, STREAMS[name], 16, "launches"
        sub.no_variants, sub.no_host_path = True, True
        sub.stagger_us = None
        sub.warmup = max(args.warmup, SUBLINE_WARMUP)
        t0 = time.perf_counter()
        line = run(sub, name, env)
        if line is not None:
            line["wall_s_subline"] = round(time.perf_counter() - t0, 2)
        out[name] = line
        release()
    return out if env[6] == 0 else None


def run_config(args, config, env):
    Gate.FENCED_EVENTS = bool(getattr(args, "fenced_events", False))
    """One config's bench line (rank 0 returns the dict, other ranks None)."""
    torch, dist, ingot_amd, lib, ctx, world, rank, local, dev = env
    from ingot_amd import Chain, GenProfile
    from ingot_amd import dist as idist

    prof_name, _, stride, chain_name, desc = CONFIGS[config]
    profile, chain = GenProfile[prof_name], Chain[chain_name]
    mode = MODES.get(config, "parse")
    flows = mode == "flows"
    emit = mode == "emit"
    no_variants = args.no_variants or flows or emit
    # the persistent ring consumer serves fixed slots without a length array
    # (the ring kernel's layout), 16- or 8-B records, not the tunnel chain
    ring_ok = (mode == "parse" and stride is not None and stride >= 64 and prof_name == "V4UDP64"
               and chain != Chain.GeneveOverV6Tunnel)
    use_ring = args.timing == "ring"
    if use_ring and not ring_ok:
        raise SystemExit(f"--timing ring: {config} is not a slot ring without lengths")
    streams_n = 1 if use_ring else args.streams

    # --- data: this rank's share (pure in (seed, index)) + R copies ---
    first, n, n_total = frames_for_rank(config, args.scaling, rank, world)
    arena, off, lens = ingot_amd.gen_frames(profile, n, first=first, stride=stride,
                                            device=local)
    # >= 512 MiB of distinct arenas (the 256 MiB MALL cannot serve a step from
    # the previous one), and a copy per stream in flight (launches running
    # together never read the same bytes) — up to ROTATE_CAP_BYTES; above it
    # (a 50 GB strong-scaling arena is far past every cache) one copy, and
    # only single-stream variants
    need = max(1, -(-(args.rotate_mib << 20) // arena.numel()))
    # (config 5's runner rotates its histograms with the arenas: >= 4)
    reps = max(need, streams_n, 4 if flows or not no_variants else 1)
    multi_stream_variants = True
    if arena.numel() * reps > ROTATE_CAP_BYTES:
        reps = max(need, streams_n)
        multi_stream_variants = False
    arenas = [arena] + [arena.clone() for _ in range(reps - 1)]
    outs = [torch.empty((n, 16), dtype=torch.uint8, device=dev) for _ in range(reps)]
    G = ring_group(args.steps)
    ring_outs = None
    if use_ring:  # every batch of a ring launch writes its own record buffer
        ring_outs = outs + [torch.empty((n, 16), dtype=torch.uint8, device=dev)
                            for _ in range(max(0, G - reps))]
    torch.cuda.synchronize(dev)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev)
                                                  for _ in range(max(3, args.streams - 1))]

    if flows:
        hists = [torch.zeros(FLOW_BINS, dtype=torch.int32, device=dev) for _ in range(reps)]
        flow_ids = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(reps)]
        # config 5's reduce is the product's (ingot_gpu_flow_hist_allreduce over
        # the library's RCCL communicator, a one-rank one at N = 1); the gloo
        # rehearsal of N > 1 reduces through torch.distributed instead.
        # Communicators up before any gated region (eager, ungated).
        comm = None
        if args.dist_backend == "gloo" and world > 1:
            reduce_fn = idist.reduce_histogram_async
            idist.reduce_histogram(hists[0])
        else:
            comm = getattr(ctx, "_flow_comm", None)
            if comm is None:
                comm = ctx._flow_comm = idist.product_comm(ctx)
            reduce_fn = idist.product_reduce(comm)
            comm.allreduce_hist(hists[0])
        hists[0].zero_()
        torch.cuda.synchronize(dev)
    recs0 = None
    if mode == "read":
        # mblk-style packets over the same frames (chunks inside each frame)
        recs0 = ingot_amd.records_to_numpy(
            ctx.parse_strided(arena, stride, n, chain) if stride is not None else
            ctx.parse(arena, off, lens, chain))
        rlens = lens if lens is not None else torch.full((n,), stride, dtype=torch.int32,
                                                         device=dev).to(torch.uint16)
        seg_off, seg_len, pkt_seg, head_chunks = read_chunks(
            torch, off, stride, rlens.to(torch.int32), recs0, READ_CHUNKS[config], dev)

    read_first = config in READ_FIRST
    read_lazy = read_first and config in READ_LAZY and not args.tune
    if read_lazy:
        from ingot_amd import abi as _abi

        ctx.set_tuning(_abi.TUNE_READ_PLAN, 17)

    def runner(nstreams, record, flows_only=False, dense=False, ring=False, group=G,
               first=read_first):
        if ring:
            return RingRunner(torch, lib, ctx, chain, n, stride, arenas,
                              ring_outs if record == 16 else outs8, streams[0], record, group)
        if flows:
            return FlowRunner(torch, lib, ctx, chain, n, arenas, off, lens, hists, flow_ids,
                              streams[:nstreams], reduce_fn, flows_only,
                              open_before_collective=policy == "until_collective")
        if mode == "modify":
            return ModifyRunner(torch, lib, ctx, chain, n, stride, arenas, off, lens,
                                streams[:nstreams])
        if emit:
            return EmitRunner(torch, lib, ctx, n, arenas, off, lens, first, streams[:nstreams])
        if mode == "packed":
            return PackedRunner(torch, lib, ctx, chain, n, arenas, lens, outs,
                                streams[:nstreams])
        if mode == "read":
            return ReadRunner(torch, lib, ctx, chain, n, arenas, seg_off, seg_len, pkt_seg,
                              outs, streams[:nstreams], dense, first and not dense)
        return Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs,
                      streams[:nstreams], record)

    if mode in ("modify", "read", "packed", "emit") and args.record == 8:
        raise SystemExit("8-B records are not offered for this config")
    if chain == Chain.GeneveOverV6Tunnel and args.record == 8:
        raise SystemExit("8-B records are not offered for the tunnel chain (include/ingot_gpu.h)")
    outs8 = None
    if use_ring and args.record == 8:
        outs8 = [torch.empty((n, 8), dtype=torch.uint8, device=dev) for _ in range(max(G, reps))]
    policy = gate_policy(flows, world, args.dist_backend, args.no_gate)
    gate = None
    gate_note = {"off": "off (--no-gate)" if args.no_gate else
                 "off (gloo rehearsal: the histogram reduce copies through the host)"}.get(policy)
    if policy != "off":
        try:
            stagger = (args.stagger_us if args.stagger_us is not None
                       else STAGGER_US.get(config, 0.0))
            gate = Gate(ingot_amd, ctx, stagger)
            gate_note = (f"first {Gate.HOLD} launches held behind a doorbell "
                         "(ingot_gpu_doorbell_wait); region from the first step's start" +
                         ("" if Gate.FENCED_EVENTS else
                          "; timing-only HIP events (hipEventDisableSystemFence)"))
            if policy == "until_collective":
                gate_note = ("launches held behind a doorbell until the first RCCL collective "
                             "of the region, which is issued only after the ring")
            if stagger and streams_n > 1:
                gate_note += (f"; stream i starts i x {stagger:g} us behind stream 0 "
                              "(ingot_gpu_stream_delay), inside the region")
        except RuntimeError as e:
            gate_note = f"unavailable ({e}); region from host submission"
    if use_ring:
        gate_note = (f"persistent ring consumer: ingot_gpu_parse_ring, {args.steps // G} "
                     f"launch(es) of {G} batches on one stream (k_parse_ring; every batch reads "
                     f"its own 1 M-frame arena copy and writes its own 1 M records inside the "
                     f"region); " + (gate_note or ""))
    main_run = runner(streams_n, args.record, ring=use_ring)
    if use_ring:
        main_run.warm(args.warmup, gate)
    else:
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
    region_ms_per_rank = idist.gather_over_ranks(ms_region, device=dev)
    if flows:  # the last timed step's reduced histogram and this rank's flow ids
        last = (args.steps - 1) % reps
        hist_last, fid_last = hists[last].clone(), flow_ids[last].clone()
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
        # (read_first: chunk 0's 8-B (offset << 16) | length per packet
        # instead of its table entry, later header chunks from the table)
        # (read_lazy: pkt_seg only for the packets whose walk needed the
        # bounds: more than one header chunk, or a parse error)
        hc = head_chunks.cpu().numpy().astype(np.int64)
        dbytes = 4 + 8 + 10 * np.maximum(hc - 1, 0) if read_first else 4 + 10 * hc
        if read_lazy:
            dbytes = dbytes - 4 * ((hc <= 1) & (recs_np["status"] == 0))
        rd, wr = algorithmic_bytes(recs_np, recs_np["payload_off"], 0, dbytes, 16)
    elif mode == "packed":
        # descriptors: the u16 length, read by the parse and once more by the
        # tile-sum pass; tile sums and bases: 12 B per 64 packets
        rd, wr = algorithmic_bytes(recs_np, lens_np, 0, 2, args.record)
        rd += 2 * n + 12 * ((n + 63) // 64)
    elif emit:
        # the payload bytes copied + descriptors and setter values read; the
        # outer stack + payload written per packet
        H = len(emit_stack()[0])
        rd = int(lens_np.astype(np.int64).sum()) + EMIT_DESC_BYTES * n
        wr = int(lens_np.astype(np.int64).sum()) + H * n
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
    pipelined_gbs = (step_rd + step_wr) / (ms_step / 1e3) / 1e9
    # Roofline of the dominant kernel: launches back to back on one stream,
    # region / launches = one launch's duration, what rocprofv3's
    # per-dispatch mean of that kernel measures.  Per-batch launches: a
    # single-stream pass (in the pipelined schedule two launches overlap, so
    # per-dispatch durations are not per-step).  The ring: launches of the
    # same G batches as the timed region's.  Its own floor of warm-up and
    # launches, so that a short run (--steps 1 --warmup 0) does not report a
    # cold single launch as the kernel's rate.
    if use_ring:
        iso = main_run
        iso_launches = max(4, min(50, 1000 // G))
        iso.warm(G)
        ms_iso, _ = iso.run(iso_launches * G, gate)
        launch_ms = ms_iso / iso_launches
        per_launch = G
    else:
        # (C6e: its single-stream runner is the main one; a second would
        # hold another destination arena)
        iso = main_run if emit else runner(1, args.record, flows_only=True)
        iso.run(max(10, min(args.warmup, 50)))
        iso_steps = max(20, min(args.steps, 1000))
        ms_iso, _ = iso.run(iso_steps, gate)
        launch_ms = ms_iso / iso_steps
        per_launch = 1
    bytes_launch = (rd + wr) * per_launch
    achieved = bytes_launch / (launch_ms / 1e3) / 1e9
    ok_frac = float((recs_np["status"] == 0).mean())
    hist_check = None
    if flows:
        ok_l3 = int(((recs_np["status"] == 0) & (recs_np["l3_kind"] != 0)).sum())
        hist_check = idist.flow_hist_check(hist_last, fid_last, ok_l3, FLOW_BINS)
        hist_check["step"] = args.steps - 1
        del hist_last, fid_last
    # the multi-tile ring kernels serve slot rings without a length array
    # (launch_parse / launch_modify in parse.hip); everything else is k_parse
    ring_k = (mode in ("parse", "modify") and stride is not None and stride >= 64
              and lens is None and chain != Chain.GeneveOverV6Tunnel)
    family = "k_parse_ring" if use_ring else kernel_family(mode, ring_k)
    sha = kernel_sources_sha()
    traffic = None
    t, pf = (pmc_for(config, family, sha, n * per_launch) if args.record == 16 and not args.tune
             else (None, None))
    if t is not None:
        traffic = {"bytes_per_launch": t["traffic_bytes_per_launch"],
                   "ratio_to_algorithmic": round(t["traffic_bytes_per_launch"] / bytes_launch, 4),
                   "source": f"{pf.relative_to(ROOT)} (rocprofv3 --pmc FETCH_SIZE x2 + "
                             "WRITE_SIZE, separate passes, same kernel sources)",
                   "kernel": t.get("kernel")}
        if t.get("fetch_bytes_sized"):
            # the x2 correction cross-checked by the L2 -> memory read
            # requests counted by size (32/64/128 B) in a pass of their own
            traffic["fetch_bytes_sized"] = t["fetch_bytes_sized"]
            traffic["sized_vs_corrected"] = t.get("sized_vs_corrected")

    # --- variants (outside the timed region; same data) ---
    variants = {}
    if not no_variants:
        vsteps = min(args.steps, 1000)
        combos = [(1, 16), (2, 8), (1, 8), (4, 16)]
        if ring_ok and not use_ring:  # the persistent ring consumer over the same batches
            combos += [("ring", 16)]
        if use_ring:  # the per-batch launches the ring replaces, and 8-B ring records
            combos = [(2, 16), (1, 16), (2, 8), ("ring", 8)]
        for ns, rb in combos:
            if not use_ring and (ns, rb) == (args.streams, args.record):
                continue
            if ns != "ring" and ns > 1 and not multi_stream_variants:
                continue
            if rb == 8 and (chain == Chain.GeneveOverV6Tunnel or mode != "parse"):
                continue
            if ns == "ring":
                if rb == 8 and outs8 is None:
                    outs8 = [torch.empty((n, 8), dtype=torch.uint8, device=dev)
                             for _ in range(max(G, reps))]
                if rb == 16 and ring_outs is None:
                    ring_outs = outs + [torch.empty((n, 16), dtype=torch.uint8, device=dev)
                                        for _ in range(max(0, G - reps))]
                r = runner(1, rb, ring=True)
                r.warm(min(args.warmup, 50), gate)
                name = f"ring_rec{rb}"
            else:
                r = runner(ns, rb)
                r.run(min(args.warmup, 50), gate if ns > 1 else None)
                name = f"{'launches_' if use_ring else ''}streams{ns}_rec{rb}"
            ms, _ = r.run(vsteps, gate)
            bpl = rd + (rb * n if mode != "modify" else wr)
            variants[name] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3),
                "hbm_GBps": round(bpl / (ms / vsteps / 1e3) / 1e9, 1),
                "read_frac": round(rd / (ms / vsteps / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            }
        if stride == 64 and mode == "parse" and not use_ring and args.record == 16:
            # the headline schedule with 64 record buffers rotated (1 GiB):
            # the default's R buffers (R x 16 MiB) fit the 256 MiB Infinity
            # Cache, so their stores need not reach HBM inside the region;
            # 1 GiB of them cannot stay there (tools/record_footprint.py)
            outs64 = outs + [torch.empty((n, 16), dtype=torch.uint8, device=dev)
                             for _ in range(max(0, 64 - len(outs)))]
            r = Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs64,
                       streams[:args.streams], 16)
            r.run(min(args.warmup, 50), gate)
            ms, _ = r.run(vsteps, gate)
            variants[f"streams{args.streams}_rec16_records64"] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3),
                "read_frac": round(rd / (ms / vsteps / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "record_buffers_rotated": len(outs64)}
            del outs64, r
        if mode == "read":  # the same chunks as one dense 8-B entry each
            r = runner(args.streams, 16, dense=True)
            r.run(min(args.warmup, 50))
            ms, _ = r.run(vsteps, gate)
            variants[f"streams{args.streams}_dense_table"] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3)}
            # the other descriptor form: chunk 0 from the table
            # (ingot_gpu_parse_read) / per packet (ingot_gpu_parse_read_first)
            r = runner(args.streams, 16, first=not read_first)
            r.run(min(args.warmup, 50))
            ms, _ = r.run(vsteps, gate)
            variants[f"streams{args.streams}_" +
                     ("chunk_table" if read_first else "first_chunk_inline")] = {
                "value": round(n * vsteps / (ms / 1e3) / 1e6, 2),
                "us_per_step": round(ms * 1e3 / vsteps, 3)}
            del r

    if flows and not args.tune:
        # the plain parse (16-B records) of the same frames, one stream, as
        # the flows kernel's roofline pass: the cost of the hash and the flow
        # window, from one run (k_parse beside k_parse<..., OUT_FLOWS16> in a
        # rocprofv3 trace of this command)
        r = Runner(torch, lib, ctx, chain, n, stride, arenas, off, lens, outs, streams[:1], 16)
        r.run(max(10, min(args.warmup, 50)))
        vsteps = max(20, min(args.steps, 1000))
        ms, _ = r.run(vsteps, gate if policy == "hold" else None)
        us = ms * 1e3 / vsteps
        variants["plain_parse_streams1_rec16"] = {
            "us_per_launch": round(us, 3),
            "flows_kernel_us_per_launch": round(launch_ms * 1e3, 3),
            "flows_over_plain": round(launch_ms * 1e3 / us, 4),
            "frac": round((rd + 16 * n) / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
        }

    host_path = None
    if (world == 1 and mode == "parse" and args.record == 16 and not args.no_host_path
            and not args.tune):
        host_path = host_inclusive_live(torch, ingot_amd, ctx, arenas[0], off, lens, stride,
                                        chain, n)

    if read_lazy:
        ctx.set_tuning(_abi.TUNE_READ_PLAN, 0)
    if rank != 0:
        return None
    cpu = (getattr(args, "cpu_pre", None) or {}).get(config)
    if cpu is None and world == 1 and not args.no_cpu_baseline:
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
        cpu["measured"] = "after the GPU run (device-generated sample copied back)"
    kname = {"modify": ", parse + setters",
             "emit": " (ingot_gpu_emit_packets: a group of 256 packets as one flat run of 16-B "
                     "destination chunks taken in turns by the workgroup's sixteen waves, header "
                     "blocks patched once per packet in LDS)",
             "read": ", LAYOUT_SEGMENTED (parse_read" +
                     (", chunk 0 per packet: ingot_gpu_parse_read_first" if read_first else "") +
                     (", chunk bounds on demand: INGOT_TUNE_READ_PLAN 17)" if read_lazy else ")"),
             "packed": ", LAYOUT_PACKED + k_tile_sums/k_group_scan",
             "flows": " (tuple.hip: the plain parse's 4-5 chunk window and walk, then the "
                      "table-free Toeplitz hash, bit by bit from the key windows FlowArgs::w in "
                      "SGPRs; the step adds k_flow_count16 / k_flow_reduce16)"}.get(mode, "")
    read_frac_step = step_rd / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS
    return {
        "metric": EMIT_METRIC if emit else METRIC,
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
            "layout": (("chunk lists: u32 pkt_seg bounds, u64 seg_off + u16 seg_len per chunk" +
                        ("; chunk 0 as one u64 (offset << 16) | length per packet"
                         if read_first else "") +
                        ("; bounds loaded only by walks that leave chunk 0 or fail "
                         "(INGOT_TUNE_READ_PLAN 17)" if read_lazy else "") +
                        f" ({READ_CHUNKS[config]})")
                       if mode == "read" else
                       f"strided {stride} B" if stride else "packed, u64 offsets + u16 lengths"),
            "record_bytes": args.record,
            "streams": streams_n,
            "arena_copies_rotated": reps,
            "record_buffers_rotated": (G if use_ring else reps),
            "parallelism": (f"{args.scaling} scaling, contiguous share per GPU x{world}" +
                            (f"; {'gloo' if args.dist_backend == 'gloo' and world > 1 else 'RCCL'}"
                             f" all-reduce (sum) of the {FLOW_BINS} x u32 flow "
                             "histogram every step" if flows else
                             " (no data-path collective)")),
            "ok_fraction": round(ok_frac, 6),
            "timing": gate_note,
            "timing_mode": "ring" if use_ring else "launches",
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
                      f"{family} (ingot_amd/csrc/{KERNEL_FILE.get(family, 'parse.hip')}){kname}",
            "kernel_sources_sha": sha,
            "batches_per_launch": per_launch,
            "launch_mean_us": round(launch_ms * 1e3, 3),
            "launch_timing": ("ring launches of the region's batch count back to back, one "
                              "stream, HIP events, region / launches" if use_ring else
                              "single-stream pass, HIP events, region/K"),
            "pipelined_GBps": round(pipelined_gbs, 1),
            "pipelined_frac": round(pipelined_gbs / HBM_PEAK_GBS, 4),
            "pipelined_read_frac": round(read_frac_step, 4),
            "north_star_read_frac": round(read_frac_step, 4),
            "north_star_read_frac_def": ("HBM-read roofline fraction of the timed region: "
                                         "algorithmic read bytes per step / ms_per_step / 8 TB/s"),
            "algorithmic_bytes_per_launch": bytes_launch,
            "read_bytes_per_batch": rd,
            "write_bytes_per_batch": wr,
            "read_frac": round(rd * per_launch / (launch_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_of_measured_copy_ceiling": round(achieved / HBM_MEASURED_GBS, 4),
            # the headline schedule with 1 GiB of record buffers rotated: the
            # records cannot stay in the 256 MiB Infinity Cache and reach HBM
            # inside the region (the default's few buffers stay cached)
            "read_frac_records_dram": (variants.get(f"streams{args.streams}_rec16_records64")
                                       or {}).get("read_frac"),
        },
        "distributed": {
            **idist.world_info(),
            **({"group": ("torch.distributed group: control only (communicator id, barriers, "
                          "max over ranks, checks); the data-path reduce is "
                          + ("RCCL" if args.dist_backend == "nccl" else "gloo"))}
               if world > 1 else {}),
            **({"rehearsal": f"{world} ranks on one GPU, RCCL over loopback sockets "
                             "(--rehearse-one-gpu): the path runs, the rates mean nothing"}
               if getattr(args, "rehearse_one_gpu", False) and world > 1 else {}),
            "region_ms_per_rank": [round(x, 5) for x in region_ms_per_rank],
            "collective": ((f"ingot_gpu_flow_hist_allreduce every step: RCCL all-reduce SUM "
                            f"(ncclUint32) of the {FLOW_BINS} x u32 flow histogram over the "
                            f"library's {world}-rank communicator, on the step's stream"
                            if args.dist_backend == "nccl" or world == 1 else
                            f"gloo rehearsal: torch all_reduce SUM of the {FLOW_BINS} x u32 "
                            "histogram through host memory")
                           if flows else None),
            "flow_hist_check": hist_check,
        },
        "ms_per_step_ungated": ungated,
        "variants": variants,
        "cpu_baseline": cpu,
        "wall_s_timed_region": round(wall, 4),
        "host_inclusive": host_path,
    }


if __name__ == "__main__":
    main()
