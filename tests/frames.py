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


def geneve_outer(rng, opts=((0x0129, 0, b""),), hbh: bool = False, vni: int | None = None,
                 flags: int = 0) -> bytes:
    """Outer Ethernet / IPv6 (optional 8-B hop-by-hop EH) / UDP 6081 / Geneve
    with `opts` = ((class, type, data), ...) as in RFC 8926 / geneve.rs:16-102."""
    optb = b""
    for cls, ty, data in opts:
        assert len(data) % 4 == 0
        optb += _u16(cls) + bytes([ty, len(data) // 4]) + data
    vni = int(rng.integers(0, 1 << 24)) if vni is None else vni
    gen = bytes([len(optb) // 4, flags]) + _u16(0x6558) + vni.to_bytes(3, "big") + b"\0" + optb
    udp = _u16(int(rng.integers(49152, 65536))) + _u16(6081) + _u16(8 + len(gen)) + _u16(0)
    ehb = bytes([17, 0]) + bytes(6) if hbh else b""
    v6 = (bytes([0x60, 0, 0, 0]) + _u16(len(ehb) + len(udp) + len(gen)) +
          bytes([0 if hbh else 17, 255]) + bytes([0xFD]) +
          rng.integers(0, 256, 15, dtype=np.uint8).tobytes() + bytes([0xFD]) +
          rng.integers(0, 256, 15, dtype=np.uint8).tobytes())
    eth = rng.integers(0, 256, 12, dtype=np.uint8).tobytes() + _u16(0x86DD)
    return eth + v6 + ehb + udp + gen
