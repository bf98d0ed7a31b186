"""Host-side synthetic frames for CPU tests (the device generator is GPU-only).

Frames are built field by field with the standard wire layouts; the oracle
parses them, so nothing here restates parse logic.
"""
from __future__ import annotations

import numpy as np


def _u16(v):
    return bytes([(v >> 8) & 0xFF, v & 0xFF])


def build_frames(n: int, seed: int = 0, vlan: bool = False, broken: float = 0.05):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        eth = rng.integers(0, 256, 12, dtype=np.uint8).tobytes()
        tags = b""
        if vlan and rng.random() < 0.5:
            tags = _u16(0x8100) + _u16(int(rng.integers(0, 65536)))
        v6 = rng.random() < 0.5
        l4 = int(rng.choice([6, 17, 1, 58]))
        if v6:
            l3 = (bytes([0x60, 0, 0, 0]) + _u16(0) + bytes([l4, 64]) +
                  rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
            et = 0x86DD
        else:
            l3 = (bytes([0x45, 0, 0, 0, 0, 0, 0, 0, 64, l4, 0, 0]) +
                  rng.integers(0, 256, 8, dtype=np.uint8).tobytes())
            et = 0x0800
        if l4 == 6:
            l4b = rng.integers(0, 256, 4, dtype=np.uint8).tobytes() + bytes(8) + bytes([0x50, 2]) \
                + bytes(6)
        else:
            l4b = rng.integers(0, 256, 4, dtype=np.uint8).tobytes() + bytes(4)
        if tags:
            frame = eth + tags + _u16(et) + l3 + l4b
        else:
            frame = eth + _u16(et) + l3 + l4b
        frame += bytes(int(rng.integers(0, 24)))
        if rng.random() < broken:
            frame = frame[: int(rng.integers(0, len(frame)))]
        out.append(frame)
    return out


def pack(frames):
    """-> (arena u8, off u64, len u16) numpy arrays, frames back-to-back."""
    off, o = [], 0
    for f in frames:
        off.append(o)
        o += len(f)
    arena = np.frombuffer(b"".join(frames) + bytes(64), dtype=np.uint8).copy()
    return (arena, np.array(off, dtype=np.uint64),
            np.array([len(f) for f in frames], dtype=np.uint16))
