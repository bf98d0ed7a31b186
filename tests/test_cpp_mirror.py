"""The C++ host mirror (include/ingot_amd.hpp): the reference's chain tests
restated in C++ (tests/cpp/test_reference_kats.cpp), run on the GPU."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def test_cpp_mirror_compiles():
    from ingot_amd.build import build, build_cpp_tests

    build()
    exes = build_cpp_tests()
    assert exes and all(e.exists() for e in exes)


@pytest.mark.gpu
def test_cpp_reference_kats_on_device():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = ROOT / "tests" / "cpp" / "build" / "test_reference_kats"
    if not exe.exists():
        from ingot_amd.build import build_cpp_tests

        build_cpp_tests()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout


@pytest.mark.gpu
def test_cpp_host_ring_example_on_device():
    """tests/cpp/example_host_ring.cpp: a C++ consumer of the ABI parsing
    frames in pageable host memory, zero-copy."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = ROOT / "tests" / "cpp" / "build" / "example_host_ring"
    if not exe.exists():
        from ingot_amd.build import build_cpp_tests

        build_cpp_tests()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout


@pytest.mark.gpu
def test_cpp_doorbell_ring_on_device():
    """tests/cpp/example_doorbell_ring.cpp: a C++ ring consumer enqueues 8
    batches' parses behind doorbells before their frames exist; a producer
    thread copies each slot in and rings; the first parse is held until its
    doorbell and every record is UdpParser's."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = ROOT / "tests" / "cpp" / "build" / "example_doorbell_ring"
    if not exe.exists():
        from ingot_amd.build import build_cpp_tests

        build_cpp_tests()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "first held: ok" in r.stdout


@pytest.mark.gpu
def test_cpp_flow_reduce_example_on_device():
    """tests/cpp/example_flow_reduce.cpp: config 5's step from a host that
    binds only the C ABI — flow hash + histogram, then the RCCL reduce over a
    communicator made from rank 0's id (one rank on this box; RCCL opened by
    the library itself, no PyTorch in the process)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = ROOT / "tests" / "cpp" / "build" / "example_flow_reduce"
    if not exe.exists():
        from ingot_amd.build import build_cpp_tests

        build_cpp_tests()
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout and "rccl reduce over 1 rank(s)" in r.stdout
    assert "lent communicator: reduce ok" in r.stdout


@pytest.mark.gpu
def test_cpp_flow_reduce_world2_on_one_gpu(tmp_path):
    """The same C-ABI-only host at world 2: two processes of
    example_flow_reduce, rank 0's communicator id carried in a file, each rank
    counting its contiguous shard of 262,144 frames.  Both ranks share the
    box's one GPU (bench.REHEARSAL_ENV + a host id per rank, as
    tests/test_comm_world2.py).  Every rank's reduced histogram equals the sum
    of the ranks' own bincounts and the oracle's histogram of both shards."""
    import os

    import numpy as np
    import torch

    import bench
    import oracle
    from ingot_amd import Chain, GenProfile
    from ingot_amd.hostgen import gen_frames_host

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = ROOT / "tests" / "cpp" / "build" / "example_flow_reduce"
    if not exe.exists():
        from ingot_amd.build import build_cpp_tests

        build_cpp_tests()
    world, n, bins = 2, 1 << 18, 1 << 16
    procs = []
    for r in range(world):
        env = dict(os.environ, **bench.REHEARSAL_ENV, NCCL_HOSTID=f"ingot-cpp-rank{r}")
        procs.append(subprocess.Popen([str(exe), str(world), str(r), str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=100)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    print("\n".join(outs))
    assert [p.returncode for p in procs] == [0] * world, outs
    local = sum(np.fromfile(tmp_path / f"local.{r}", dtype=np.uint32).astype(np.int64)
                for r in range(world))
    want = np.zeros(bins, np.uint32)
    for r in range(world):
        a, o, ln = gen_frames_host(GenProfile.FLOWS, n, first=r * n)
        oracle.flow_hist(a, o, ln, Chain.VlanUlp, bins=bins, hist=want)
    assert want.sum() > 0 and (local == want).all()
    for r in range(world):
        got = np.fromfile(tmp_path / f"hist.{r}", dtype=np.uint32)
        assert (got == want).all()
