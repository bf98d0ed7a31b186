"""bench.py's process model, on CPU (gloo): `--gpus N` without a launcher
starts N ranks itself (one process per GPU, before any GPU call) and the
line reports n_gpus == N; under a launcher, WORLD_SIZE must equal --gpus;
weak shards are disjoint full batches and strong shares (dist.split) cover
the job's frames exactly once.  `--plan` runs the whole distributed
plumbing (rendezvous, shares, gather on rank 0, one JSON line) without a GPU."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

import bench
from ingot_amd import dist as idist

ROOT = Path(__file__).resolve().parent.parent


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r


def _line(r):
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout  # rank 0 only
    return json.loads(lines[0])


def _covers_once(shards, total):
    shards = sorted(shards)
    pos = 0
    for first, n in shards:
        assert first == pos, shards
        assert n > 0
        pos += n
    assert pos == total, (pos, total)


def test_gpus2_spawns_two_ranks_weak():
    d = _line(_run(["--gpus", "2", "--dist-backend", "gloo", "--config", "c2", "--plan"]))
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    n = bench.CONFIGS["c2"][1]
    assert d["shards"] == [[0, n], [n, n]]
    assert d["total_frames"] == 2 * n


@pytest.mark.parametrize("world", [2, 3])
def test_strong_shares_cover_the_job_once(world):
    d = _line(_run(["--gpus", str(world), "--dist-backend", "gloo", "--config", "c4",
                    "--scaling", "strong", "--plan"]))
    assert d["n_gpus"] == world and d["scaling"] == "strong"
    assert d["total_frames"] == bench.STRONG_TOTAL["c4"] == 64 << 20
    _covers_once(d["shards"], d["total_frames"])


def test_split_covers_every_world_size():
    for total in (1, 7, 1 << 20, (64 << 20) + 5):
        for world in (1, 2, 3, 4, 8):
            _covers_once([idist.split(total, r, world) for r in range(world)
                          if idist.split(total, r, world)[1]], total)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "1", "--plan"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "--gpus 1 but WORLD_SIZE=2" in r.stderr


def test_single_process_default_is_one_gpu():
    d = _line(_run(["--plan"]))
    assert d["n_gpus"] == 1 and d["shards"] == [[0, bench.CONFIGS["c2"][1]]]


def test_failing_rank_fails_the_launch():
    """An unknown config fails every rank; the launcher returns non-zero."""
    r = _run(["--gpus", "2", "--config", "nope", "--plan"])
    assert r.returncode != 0
