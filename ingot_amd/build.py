"""Build the native library in-tree: ingot_amd/lib/libingot_gpu.so (gfx950).

    python -m ingot_amd.build [--force]

Each HIP/C++ source is compiled to an object with hipcc (in parallel), then
linked into one shared library.  Objects are rebuilt when a source or any
header under include/ or csrc/ is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
BUILD = PKG / "build"
LIB = PKG / "lib" / "libingot_gpu.so"
SOURCES = ["parse.hip", "read.hip", "ring.hip", "flow.hip", "tuple.hip", "header.hip", "packed.hip",
           "pktgen.hip", "pktgen_host.cpp", "stream.hip", "emit.hip", "api.cpp", "comm.cpp"]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def _headers() -> list[Path]:
    return sorted((ROOT / "include").glob("*.h")) + sorted(CSRC.glob("*.h"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _compile(src: Path, obj: Path) -> None:
    cmd = [
        hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
        "-Wall", "-Wno-unused-function",
        f"-I{ROOT / 'include'}", "-c", str(src), "-o", str(obj),
    ]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-x", "hip"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    LIB.parent.mkdir(exist_ok=True)
    headers = _headers()
    jobs = []
    objs = []
    for name in SOURCES:
        src = CSRC / name
        obj = BUILD / (name + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + headers):
            jobs.append((src, obj))
    if jobs:
        try:
            with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 6)) as ex:
                for f in [ex.submit(_compile, s, o) for s, o in jobs]:
                    f.result()
        except Exception:
            # never leave a stale library behind a failed build
            LIB.unlink(missing_ok=True)
            for _, o in jobs:
                o.unlink(missing_ok=True)
            raise
    if force or jobs or _stale(LIB, objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB)]
        cmd += [str(o) for o in objs] + ["-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


HOST_PKTGEN = PKG / "lib" / "libingot_pktgen_host.so"


def build_host_pktgen(force: bool = False, verbose: bool = False) -> Path:
    """The synthetic traffic generator for the host (csrc/pktgen_host.cpp,
    g++, no HIP): bench.py builds its CPU baseline's sample with it before
    the process touches the GPU."""
    src = CSRC / "pktgen_host.cpp"
    deps = [src, CSRC / "pktgen_core.h", ROOT / "include" / "ingot_pktgen.h",
            ROOT / "include" / "ingot_gpu.h"]
    HOST_PKTGEN.parent.mkdir(exist_ok=True)
    if force or _stale(HOST_PKTGEN, deps):
        cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread",
               "-Wall", f"-I{ROOT / 'include'}", str(src), "-o", str(HOST_PKTGEN)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            HOST_PKTGEN.unlink(missing_ok=True)
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {HOST_PKTGEN}")
    return HOST_PKTGEN


CPP_TESTS = ROOT / "tests" / "cpp"


def build_cpp_tests(verbose: bool = False) -> list[Path]:
    """Compile the C++ mirror tests (tests/cpp/*.cpp) against the library."""
    out_dir = CPP_TESTS / "build"
    out_dir.mkdir(exist_ok=True)
    outs = []
    deps = _headers() + [ROOT / "include" / "ingot_amd.hpp", LIB]
    for src in sorted(CPP_TESTS.glob("*.cpp")):
        exe = out_dir / src.stem
        outs.append(exe)
        if not _stale(exe, [src] + deps):
            continue
        cmd = [hipcc(), "-std=c++17", "-O2", f"-I{ROOT / 'include'}", str(src),
               f"-L{LIB.parent}", "-lingot_gpu", "-Wl,-rpath,$ORIGIN/../../../ingot_amd/lib",
               # example_flow_reduce makes an RCCL communicator of its own
               "-L/opt/rocm/lib", "-Wl,--as-needed", "-lrccl",
               "-o", str(exe)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            exe.unlink(missing_ok=True)
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"built {exe}")
    return outs


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    build_host_pktgen(force="--force" in sys.argv, verbose=True)
    build_cpp_tests(verbose=True)
