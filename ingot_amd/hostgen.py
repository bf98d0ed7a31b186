"""The synthetic traffic generator on the host (lib/libingot_pktgen_host.so,
include/ingot_pktgen.h): the same bytes as `ingot_amd.gen_frames` for the same
arguments, into numpy arrays, without loading the HIP library — bench.py
builds its CPU baseline's sample with it before the process touches the GPU.
Bench infrastructure, not the parse path."""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

import numpy as np

from .abi import GEN_SEED, GenProfile

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libingot_pktgen_host.so"
_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: run python -m ingot_amd.build")
        lib = ctypes.CDLL(str(LIB_PATH))
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        lib.ingot_pktgen_lengths_host.argtypes = [ctypes.c_int, u64, u64, u64, vp, ctypes.c_int]
        lib.ingot_pktgen_lengths_host.restype = ctypes.c_int
        lib.ingot_pktgen_fill_host.argtypes = [ctypes.c_int, u64, u64, u64, vp, ctypes.c_uint32,
                                               vp, vp, u64, ctypes.c_int]
        lib.ingot_pktgen_fill_host.restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _aligned(nbytes: int) -> np.ndarray:
    """A 16-B aligned u8 array of nbytes (the generator's word stores)."""
    raw = np.empty(nbytes + 16, dtype=np.uint8)
    o = (-raw.ctypes.data) % 16
    return raw[o:o + nbytes]


def gen_frames_host(profile: GenProfile, n: int, seed: int = GEN_SEED, first: int = 0,
                    stride: Optional[int] = None, slack: int = 256,
                    threads: Optional[int] = None):
    """-> (arena u8, off u64 or None, lens u16 or None) as numpy arrays, laid
    out exactly as gen_frames lays them out on the device."""
    lib = load()
    threads = threads or min(16, os.cpu_count() or 1)
    lens = None
    if stride is None or profile != GenProfile.V4UDP64:
        lens = np.empty(max(n, 1), dtype=np.uint16)[:n]
        if lib.ingot_pktgen_lengths_host(int(profile), seed, first, n, _p(lens), threads) != 0:
            raise RuntimeError("ingot_pktgen_lengths_host failed")
    if stride is not None:
        if lens is not None:
            lens = np.minimum(lens, stride).astype(np.uint16)
        nbytes = n * stride + slack
        arena = _aligned(nbytes)
        rc = lib.ingot_pktgen_fill_host(int(profile), seed, first, n, None, int(stride), _p(lens),
                                        _p(arena), nbytes, threads)
        if rc != 0:
            raise RuntimeError("ingot_pktgen_fill_host failed")
        return arena, None, lens
    ends = np.cumsum(lens, dtype=np.int64)
    off = (ends - lens).astype(np.uint64)
    nbytes = (int(ends[-1]) if n else 0) + slack
    arena = _aligned(nbytes)
    rc = lib.ingot_pktgen_fill_host(int(profile), seed, first, n, _p(off), 0, _p(lens),
                                    _p(arena), nbytes, threads)
    if rc != 0:
        raise RuntimeError("ingot_pktgen_fill_host failed")
    return arena, off, lens
