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
