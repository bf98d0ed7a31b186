"""bench.py's accounting, on CPU: the SURVEY §8d algorithmic bytes behind
`roofline.achieved`, the config table, and the C5 runner's overlap of the
per-step histogram all-reduce (every reduce waited before the timed region
ends; a buffer reused only after its reduce) over several streams."""
import time

import numpy as np
import pytest

import bench
import oracle
from ingot_amd import REC_DTYPE, Chain
from tests.frames import build_frames, pack


def test_algorithmic_bytes_c2_shape():
    """C2: 64-B slots, 42-B header span -> R = 64, W = 16: 80 B per packet."""
    n = 1000
    recs = np.zeros(n, dtype=REC_DTYPE)
    recs["payload_off"] = 42
    rd, wr = bench.algorithmic_bytes(recs, None, 64, 0, 16)
    assert (rd, wr) == (64 * n, 16 * n)
    assert bench.algorithmic_bytes(recs, None, 64, 0, 8) == (64 * n, 8 * n)


def test_algorithmic_bytes_rule():
    """R_i = min(len_i, 128) + max(0, H_i - 128) + D, per packet."""
    recs = np.zeros(4, dtype=REC_DTYPE)
    recs["payload_off"] = [42, 128, 200, 90]
    lens = np.array([60, 1500, 1500, 100], dtype=np.uint16)
    rd, wr = bench.algorithmic_bytes(recs, lens, 0, 10, 16)
    assert rd == (60 + 10) + (128 + 10) + (128 + 72 + 10) + (100 + 10)
    assert wr == 64


def test_algorithmic_bytes_of_oracle_records():
    """On real records: the header span never exceeds the frame, so
    R_i <= len_i + D, and R_i >= min(len_i, 128)."""
    frames = build_frames(500, seed=3)
    arena, off, lens = pack(frames)
    recs = oracle.parse_batch(arena, off, lens, Chain.GenericUlp).view(REC_DTYPE)
    rd, _ = bench.algorithmic_bytes(recs, lens, 0, 10, 16)
    L = lens.astype(np.int64)
    assert np.minimum(L, 128).sum() + 10 * len(L) <= rd <= L.sum() + 10 * len(L)


def test_config_table():
    for name, (prof, n, stride, chain, desc) in bench.CONFIGS.items():
        assert n > 0 and desc
        assert stride is None or (stride % 16 == 0 and stride >= 64)
        Chain[chain]
    # the metric's configuration (BASELINE.json configs[1]) is the default
    assert bench.CONFIGS["c2"][:4] == ("V4UDP64", 1 << 20, 64, "UdpParser")
    assert set(bench.MODES.values()) <= {"flows", "modify", "read", "packed", "emit"}
    assert set(bench.STREAMS) == set(bench.CONFIGS)
    assert all(1 <= v <= 4 for v in bench.STREAMS.values())


class _Work:
    def __init__(self, log, k):
        self.log, self.k = log, k

    def wait(self):
        self.log.append(("wait", self.k))


class _Stream:
    cuda_stream = 0

    def wait_event(self, ev):
        pass


class _FakeTorch:
    """Just enough of torch for FlowRunner/_timed without a GPU."""

    class cuda:  # noqa: N801
        class Event:
            def __init__(self, enable_timing=False):
                pass

            def record(self, s=None):
                pass

            def elapsed_time(self, other):
                return 1.0

        @staticmethod
        def synchronize():
            pass

        class stream:  # noqa: N801
            def __init__(self, s):
                pass

            def __enter__(self):
                return self

            def __exit__(self, *a):
                return False

    uint8 = "u8"

    @staticmethod
    def empty(n, dtype=None, device=None):
        class _T:
            def data_ptr(self):
                return 0
        return _T()


class _Hist:
    def __init__(self, log, i):
        self.log, self.i = log, i

    def zero_(self):
        self.log.append(("zero", self.i))

    def numel(self):
        return 16

    def data_ptr(self):
        return 0

    device = "cpu"


class _Lib:
    def __init__(self, log):
        self.log = log

    def ingot_gpu_flow_hist_workspace_size(self, n, bins):
        return 0

    def ingot_gpu_flow_hist_ws(self, h, arena, *a):
        self.log.append(("kernel", arena))
        return 0


class _Ctx:
    _h = None


def test_flow_runner_overlaps_reduce_and_waits_before_reuse():
    log = []
    reps = 4

    class _Buf:
        def __init__(self, i):
            self.i = i

        def data_ptr(self):
            return self.i

    arenas = [_Buf(i) for i in range(reps)]
    hists = [_Hist(log, i) for i in range(reps)]
    issued = []

    def reduce_fn(h):
        k = len(issued)
        issued.append(h.i)
        log.append(("reduce", k))
        return _Work(log, k)

    r = bench.FlowRunner(_FakeTorch, _Lib(log), _Ctx(), Chain.VlanUlp, 8, arenas, _Buf(0),
                         _Buf(0), hists, [_Buf(0)] * reps, [_Stream(), _Stream()], reduce_fn)
    r.run(7)
    waits = [k for op, k in log if op == "wait"]
    assert sorted(waits) == list(range(7))  # every reduce waited inside run()
    # step k's buffer is zeroed again at step k + reps: only after reduce k
    # has been waited for
    for k in range(7):
        zeros = [i for i, e in enumerate(log) if e == ("zero", k % reps)]
        after = [i for i in zeros if i > log.index(("reduce", k))]
        if after:
            assert log.index(("wait", k)) < after[0]
    # reduces overlap later steps: reduce k is still in flight at step k + 1
    assert log.index(("reduce", 1)) < log.index(("wait", 0))


class _ClockStream:
    """A stream with its own device clock; launches advance it."""

    def __init__(self, t0=0.0):
        self.t = t0
        self.cuda_stream = 0

    def wait_event(self, ev):
        self.t = max(self.t, ev.t)


class _ClockTorch:
    class cuda:  # noqa: N801
        class Event:
            def __init__(self, enable_timing=False):
                self.t = None

            def record(self, s):
                self.t = s.t

            def elapsed_time(self, other):
                return other.t - self.t

        @staticmethod
        def synchronize():
            pass


class _Gate:
    def __init__(self, log):
        self.log = log

    def arm(self, streams):
        self.log.append("arm")

    def open(self):
        self.log.append("open")

    def event(self):  # the gated region's timing events (bench.HipEvent on a GPU)
        return _ClockTorch.cuda.Event()


def test_timed_region_spans_earliest_start_to_latest_end(monkeypatch):
    """_timed: every stream stamps its own start and end; the region is the
    earliest start to the latest end (no join of one stream into another),
    and the doorbell gate opens after the held launches and again at the end
    (idempotent), also when a launch fails."""
    s0, s1 = _ClockStream(10.0), _ClockStream(10.5)
    durations = {0: 3.0, 1: 2.0}
    log = []

    def launch(k):
        s = (s0, s1)[k % 2]
        s.t += durations[k % 2]
        log.append(k)
        return 0

    monkeypatch.setattr(bench.Gate, "HOLD", 2)
    ms, _ = bench._timed(_ClockTorch, [s0, s1], launch, 4, gate=_Gate(log))
    # s0: 10 -> 16, s1: 10.5 -> 14.5; region = 16 - 10
    assert ms == pytest.approx(6.0)
    assert log[0] == "arm" and log[1:3] == [0, 1] and log[3] == "open" and log[-1] == "open"
    # ungated: the other streams fork from streams[0]'s start event
    a, b = _ClockStream(0.0), _ClockStream(5.0)
    ms, _ = bench._timed(_ClockTorch, [a, b], lambda k: ([a, b][k % 2].__setattr__(
        "t", [a, b][k % 2].t + 1.0), 0)[1], 2)
    assert ms == pytest.approx(6.0)  # b starts at 5 (its own clock), ends at 6
    # a failing launch still opens the gate before raising
    log2 = []
    with pytest.raises(RuntimeError):
        bench._timed(_ClockTorch, [_ClockStream()], lambda k: -1, 3, gate=_Gate(log2))
    assert log2 == ["arm", "open"]


def test_gate_policy():
    """No collective behind an unrung doorbell: config 5 reduces through the
    library's RCCL communicator at every N (one rank at N = 1) and holds
    launches only until its first collective; the gloo rehearsal (host-side
    reduce) is not gated; everything else holds Gate.HOLD."""
    assert bench.gate_policy(False, 1, "nccl", False) == "hold"
    assert bench.gate_policy(True, 1, "nccl", False) == "until_collective"
    assert bench.gate_policy(True, 1, "gloo", False) == "until_collective"
    assert bench.gate_policy(False, 8, "nccl", False) == "hold"
    assert bench.gate_policy(True, 8, "nccl", False) == "until_collective"
    assert bench.gate_policy(True, 2, "gloo", False) == "off"
    assert bench.gate_policy(True, 8, "nccl", True) == "off"


def test_flow_runner_rings_the_doorbell_before_every_collective():
    """Under a gate, FlowRunner opens it before issuing the first all-reduce
    of the region: every reduce in the log comes after an "open"."""
    log = []
    reps = 4

    class _Buf:
        def __init__(self, i):
            self.i = i

        def data_ptr(self):
            return self.i

    class _LogGate:
        def arm(self, streams):
            log.append(("arm",))

        def open(self):
            log.append(("open",))

    def reduce_fn(h):
        log.append(("reduce", h.i))
        return _Work(log, h.i)

    hists = [_Hist(log, i) for i in range(reps)]
    r = bench.FlowRunner(_FakeTorch, _Lib(log), _Ctx(), Chain.VlanUlp, 8,
                         [_Buf(i) for i in range(reps)], _Buf(0), _Buf(0), hists,
                         [_Buf(0)] * reps, [_Stream(), _Stream()], reduce_fn,
                         open_before_collective=True)
    r.run(6, gate=_LogGate())
    ops = [e[0] for e in log]
    assert ops[0] == "arm"
    first_reduce = ops.index("reduce")
    assert "open" in ops[:first_reduce]
    assert ops.count("reduce") == 6
    # and without a gate nothing is opened
    log.clear()
    r.run(2)
    assert "open" not in [e[0] for e in log]


def test_ring_group_divides_the_steps():
    assert bench.ring_group(20) == 20
    assert bench.ring_group(2000) == 50
    assert bench.ring_group(64) == 64
    assert bench.ring_group(67) == 1  # prime above the cap
    assert bench.ring_group(200) == 50
    assert bench.ring_group(1) == 1


class _Buf:
    def __init__(self, p):
        self.p = p

    def data_ptr(self):
        return self.p


class _S:
    def __init__(self, i):
        self.cuda_stream = i


def test_runner_rotates_arenas_and_records_independently():
    """bench.Runner: step k reads arena k % len(arenas) and writes record
    buffer k % len(outs) on stream k % len(streams) — so the 64-record-buffer
    variant of the C2 line keeps the default's 8-arena rotation
    (config.record_buffers_rotated)."""
    calls = []

    class Lib:
        def ingot_gpu_parse_strided(self, h, arena, stride, lens, n, chain, out, stream):
            calls.append((arena, out, stream))
            return 0

    class Ctx:
        _h = 0

    arenas = [_Buf(1000 + i) for i in range(8)]
    outs = [_Buf(5000 + i) for i in range(64)]
    r = bench.Runner(None, Lib(), Ctx(), Chain.UdpParser, 16, 64, arenas, None, None, outs,
                     [_S(0), _S(1)], 16)
    for k in range(70):
        assert r.launch(k) == 0
    assert [a for a, _, _ in calls] == [1000 + k % 8 for k in range(70)]
    assert [o for _, o, _ in calls] == [5000 + k % 64 for k in range(70)]
    assert [s for _, _, s in calls] == [k % 2 for k in range(70)]


def test_flow_runner_hold_policy_opens_only_at_hold(monkeypatch):
    """gate_policy "hold" (one GPU: no collective in the region): the doorbell
    is rung after Gate.HOLD launches or in _timed's finally, never by the
    runner after the first step — the region holds HOLD launches, as
    config.timing says."""
    monkeypatch.setattr(bench.Gate, "HOLD", 5)
    log = []
    reps = 4

    class _LogGate:
        def arm(self, streams):
            log.append(("arm",))

        def open(self):
            log.append(("open",))

    hists = [_Hist(log, i) for i in range(reps)]
    bufs = [_Buf(i) for i in range(reps)]
    r = bench.FlowRunner(_FakeTorch, _Lib(log), _Ctx(), Chain.VlanUlp, 8, bufs, _Buf(0),
                         _Buf(0), hists, [_Buf(0)] * reps, [_Stream(), _Stream()],
                         lambda h: None)
    r.run(8, gate=_LogGate())
    ops = [e[0] for e in log]
    kernels_before_open = ops[:ops.index("open")].count("kernel")
    assert kernels_before_open == 5  # exactly Gate.HOLD launches held
    # a run shorter than HOLD: the only open is the finally
    log.clear()
    r.run(3, gate=_LogGate())
    ops = [e[0] for e in log]
    assert ops.count("open") == 1 and ops[-1] == "open" and ops.count("kernel") == 3


def test_sublines_carry_c3_c4_c5_in_order():
    """The default line's sub-lines: C3, C4, C5 (BASELINE configs[2..4]),
    each with the main line's steps, a warm-up of at least SUBLINE_WARMUP
    launches and its own stream count, no
    variants; rank 0 returns them, other ranks None; other configs, --tune
    and --no-sublines carry none; unknown names fail early."""
    import argparse

    args = argparse.Namespace(config="c2", no_sublines=False, tune=[], sublines="c3,c4,c5",
                              steps=20, warmup=5, streams=2, record=16, timing="launches",
                              no_variants=False, no_host_path=False, stagger_us=None)
    seen, released = [], []

    def run(sub, name, env):
        seen.append((name, sub.config, sub.steps, sub.warmup, sub.streams, sub.no_variants,
                     sub.no_host_path, sub.record))
        return None if env[6] else {"config": name}

    env0 = (None,) * 6 + (0,)
    out = bench.run_sublines(args, env0, run, lambda: released.append(1))
    assert list(out) == ["c3", "c4", "c5"]
    assert [s[0] for s in seen] == ["c3", "c4", "c5"]
    assert all(s[1] == s[0] and s[2:4] == (20, bench.SUBLINE_WARMUP) and s[5] and s[6]
               and s[7] == 16 for s in seen)
    assert [s[4] for s in seen] == [bench.STREAMS[c] for c in ("c3", "c4", "c5")]
    assert all("wall_s_subline" in v for v in out.values()) and len(released) == 3
    seen.clear()
    assert bench.run_sublines(args, (None,) * 6 + (1,), run) is None
    assert len(seen) == 3  # every rank runs them (their collectives pair up)
    for kw in ({"config": "c3"}, {"no_sublines": True}, {"tune": ["x=1"]}):
        a = argparse.Namespace(**{**vars(args), **kw})
        assert bench.subline_names(a) == []
    with pytest.raises(SystemExit):
        bench.subline_names(argparse.Namespace(**{**vars(args), "sublines": "c3,c9"}))


def test_physical_core_pick_skips_smt_and_spreads_over_l3(monkeypatch):
    """cpu_baseline's pinning: one CPU per physical core (SMT sibling
    dropped), round-robin over L3 domains (CCDs), capped at `want`."""
    # 2 CCDs x 4 cores x 2 threads: cpu c and c + 8 are siblings; CCD = core // 4
    def fake(path):
        parts = str(path).split("/")
        c = int(parts[5][3:])
        core = c % 8
        rel = "/".join(parts[6:])
        return {"topology/physical_package_id": "0", "topology/die_id": "0",
                "topology/core_id": str(core), "cache/index3/id": str(core // 4)}.get(rel)

    monkeypatch.setattr(bench, "_read", fake)
    picked, info = bench.physical_core_pick(list(range(16)), 6)
    assert len(picked) == 6 and len({c % 8 for c in picked}) == 6  # distinct cores
    assert all(c < 8 for c in picked)  # first thread of each core
    assert {c // 4 for c in picked[:2]} == {0, 1}  # alternate CCDs
    assert info["physical_cores_available"] == 8 and info["smt_siblings_skipped"] == 8
    assert info["l3_domains_used"] == 2
    monkeypatch.setattr(bench, "_read", lambda p: None)
    assert bench.physical_core_pick([3, 1, 2], 2)[0] == [3, 1]


def test_physical_core_pick_stays_in_one_socket(monkeypatch):
    """Two sockets x 2 CCDs x 4 cores (cpu c: socket c // 8, CCD c // 4):
    the workers stay in the first allowed CPU's socket (NUMA-local sample)
    unless it has too few cores."""
    def fake(path):
        parts = str(path).split("/")
        c = int(parts[5][3:])
        rel = "/".join(parts[6:])
        return {"topology/physical_package_id": str(c // 8), "topology/die_id": "0",
                "topology/core_id": str(c % 8), "cache/index3/id": str(c // 4)}.get(rel)

    monkeypatch.setattr(bench, "_read", fake)
    picked, info = bench.physical_core_pick(list(range(16)), 6)
    assert all(c < 8 for c in picked) and info["socket"] == "0"
    assert info["sockets_available"] == 2 and info["l3_domains_used"] == 2
    picked, info = bench.physical_core_pick(list(range(6, 16)), 6)  # socket 0 has 2 cores here
    assert all(c >= 8 for c in picked) and info["socket"] == "1"


def _fake_line(value, cpu_label="clean", variants=None, ratio=1.3):
    return {"metric": bench.METRIC, "value": value, "ms_per_step": 0.0118,
            "config": {"workload": "x"},
            "roofline": {"frac": 0.72, "pipelined_read_frac": 0.71,
                         "traffic_detail": {"ratio_to_algorithmic": ratio, "pad": "p" * 900}},
            "variants": variants or {},
            "cpu_baseline": {"value": 800.0, "cores": 15, "kind": "port",
                             "sample": f"{cpu_label}: median of ...", "detail": {"runs": [1] * 500}},
            "pad": "q" * 3000}


def test_compact_line_ends_in_a_summary_of_every_config(tmp_path, monkeypatch):
    """The driver keeps the last ~8,000 characters of stdout:
    the whole line fits in 7,000, every config keeps its value, step time,
    roofline fraction and CPU baseline, C2 its host-inclusive rate and
    1 GiB record-ring read share, and the line ends in a summary that names
    C2, C3, C4 and C5 (traffic ratio, CPU baseline clean / contended)."""
    import json

    monkeypatch.setattr(bench, "ROOT", tmp_path)
    main = _fake_line(88_000, variants={"streams2_rec16_records64": {
        "us_per_step": 12.5, "read_frac": 0.667}})
    main["roofline"]["read_frac_records_dram"] = 0.667
    main["host_inclusive"] = {"frames_per_batch": 1 << 20, "memcpy_Mpkt_s": 700.7,
                              "zero_copy_Mpkt_s": 827.6, "source": "x" * 400}
    subs = {"c3": _fake_line(29_000, "contended"), "c4": _fake_line(29_100),
            "c5": _fake_line(26_000, variants={"plain_parse_streams1_rec16": {
                "flows_over_plain": 1.07}})}
    out = bench.compact_line({**main, "sublines": subs, "wall_s_command": 20.0}, "c2")
    text = json.dumps(out)
    tail = text[-1800:]
    for key in ('"c2"', '"c2_records_1GiB_ring"', '"c3"', '"c4"', '"c5"', '"over_plain_parse"',
                '"traffic_ratio"', '"kernel_frac"', 'contended"'):
        assert key in tail, key
    assert "\"detail\"" not in text
    assert json.loads((tmp_path / "gpurun_out" / "bench_full.json").read_text())[
        "cpu_baseline"]["detail"]
    s = out["summary"]
    assert s["c3"]["cpu"].endswith("contended") and s["c4"]["cpu"].endswith("clean")
    assert s["c2_records_1GiB_ring"]["step_read_frac"] == 0.667
    assert len(text) < 7000, len(text)
    c3 = out["sublines"]["c3"]
    assert c3["value"] == 29_000 and c3["ms_per_step"] and c3["roofline"]["frac"] == 0.72
    assert c3["cpu_baseline"]["value"] == 800.0
    assert out["host_inclusive"]["zero_copy_Mpkt_s"] == 827.6
    assert out["roofline"]["read_frac_records_dram"] == 0.667


def test_compact_line_with_unfinished_sublines(tmp_path, monkeypatch):
    """The line SublineGuard prints: the sub-lines that finished, the others
    named under sublines_unfinished, the summary of what was measured."""
    import json

    monkeypatch.setattr(bench, "ROOT", tmp_path)
    main = _fake_line(88_000)
    result = {**main, "sublines": {"c3": _fake_line(29_000)},
              "sublines_unfinished": {"c4": "not finished within 150 s at N = 8",
                                      "c5": "not finished within 150 s at N = 8"}}
    out = bench.compact_line(result, "c2")
    assert set(out["sublines"]) == {"c3"} and set(out["summary"]) == {"c2", "c3"}
    assert set(out["sublines_unfinished"]) == {"c4", "c5"}
    assert out["value"] == 88_000 and len(json.dumps(out)) < 7000


def test_read_chunks_np_equals_read_chunks():
    """The host chunk tables of the CPU baseline's sample equal the device
    path's (read_chunks, run here on CPU tensors)."""
    import torch

    frames = build_frames(3000, seed=5, broken=0.2)
    arena, off, lens = pack(frames)
    recs = oracle.parse_batch(arena, off, lens, Chain.GenericUlp)
    for kind in ("split2", "per_header"):
        a = bench.read_chunks_np(off, None, lens, recs, kind)
        b = bench.read_chunks(torch, torch.from_numpy(off.astype(np.int64)), None,
                              torch.from_numpy(lens.astype(np.int32)), recs, kind, "cpu")
        assert (a[0] == b[0].numpy().astype(np.uint64)).all()
        assert (a[1] == b[1].numpy().view(np.uint16)).all() if b[1].dtype != torch.int32 else True
        assert (a[2] == b[2].numpy().astype(np.uint32)).all()


def test_cpu_baseline_labels_what_it_measured():
    """cpu_baseline names its placements, says clean or contended in the
    first words of `sample`, and names the measured cause of a low share."""
    from ingot_amd.hostgen import gen_frames_host
    from ingot_amd import GenProfile

    arena, off, lens = gen_frames_host(GenProfile.MIXED, 20_000)
    c = bench.cpu_baseline(arena, off, lens, 0, 20_000, Chain.GenericUlp, budget_s=0.06,
                           workers=2)
    assert c["sample"].split(":")[0] in ("clean", "contended")
    assert c["value"] > 0 and c["cores"] in (1, 2) and c["kind"] == "port"
    assert {p["placement"].split()[1] for p in c["placements"]} >= {"pinned", "free"}
    assert isinstance(c["contention"], str) and c["contention"]
    assert len(c["sample"]) < 200


def test_emit_config_stack_and_values():
    """C6e's owned stack is OPTE's outer Eth / IPv6 / UDP / Geneve + 1 option
    (74 B) and its per-packet setter values are pure in the packet index."""
    hdr, sets = bench.emit_stack()
    assert len(hdr) == 74 and hdr[12:14] == b"\x86\xdd" and hdr[56:58] == (6081).to_bytes(2, "big")
    assert [s[0] for s in sets] == [14, 54, 54, 62]
    p0, v0 = bench.emit_values(1000, first=0)
    p1, v1 = bench.emit_values(500, first=500)
    assert (p0[500:] == p1).all() and (v0[500:] == v1).all()
    assert (p0 >= 0xC000).all() and (v0 < (1 << 24)).all()


def test_teardown_is_bounded_at_n_above_one():
    """bench.teardown at N > 1: a communicator destroy that never returns
    (seen once in the one-GPU RCCL rehearsal) ends the process with exit
    status 0 after its budget, the line having been printed; one that
    returns lets the process group go down normally."""
    import subprocess
    import sys

    code = r"""
import sys, threading, time
sys.path.insert(0, {root!r})
import bench

class Dist:
    def barrier(self): print("barrier", flush=True)
    def destroy_process_group(self): print("pg destroyed", flush=True)

class Comm:
    def __init__(self, hang): self.hang = hang
    def abort(self):
        if self.hang:
            threading.Event().wait()
        print("comm aborted", flush=True)

print("line", flush=True)
bench.teardown(Dist(), 2, Comm({hang}), budget_s=0.5)
print("after teardown", flush=True)
"""
    from pathlib import Path

    root = str(Path(bench.__file__).resolve().parent)
    for hang in (False, True):
        r = subprocess.run([sys.executable, "-c", code.format(root=root, hang=hang)],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        out = r.stdout.split()
        if hang:
            assert out == ["line", "barrier"] and "did not return" in r.stderr
        else:
            assert "pg" in out and "after" in out and "aborted" in out


def test_subline_guard_prints_and_ends_a_stalled_run():
    """bench.SublineGuard at N > 1: sub-lines that never finish (a collective
    that never completes) leave the process after the budget with status 0,
    the partial line printed by `emit`; a run that finishes in time claims
    the line and the guard never fires."""
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(bench.__file__).resolve().parent)
    code = r"""
import sys, threading, time
sys.path.insert(0, {root!r})
import bench

g = bench.SublineGuard({budget}, lambda: print("partial line", flush=True)).start()
if {stall}:
    threading.Event().wait()  # a sub-line stuck in a collective
time.sleep(0.05)
print("claimed" if g.finish() else "lost", flush=True)
time.sleep(0.6)
print("full line", flush=True)
"""
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code.format(root=root, budget=0.3, stall=True)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.split() == ["partial", "line"], r
    assert time.perf_counter() - t0 < 30
    r = subprocess.run([sys.executable, "-c", code.format(root=root, budget=0.3, stall=False)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.splitlines() == ["claimed", "full line"], r
