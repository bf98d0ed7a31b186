"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU parse oracle.

A scalar C restatement of ingot's parse path (oracle/ingot_oracle.c), pinned
by the reference's own known-answer vectors (tests/golden/).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (ingot_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

from ingot_amd.abi import (FIELDS_DTYPE, GENEVE_FIELDS_DTYPE, REC_DTYPE, Chain,  # ABI layouts only
                           edits_array, emit_sets_array)

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "libingot_oracle.so"

_lib = None


def build(out_dir: str | os.PathLike | None = None, native: bool = False) -> Path:
    """Compile the oracle with make.  `native` adds -march=native (used on the
    GPU box for the CPU baseline); `out_dir` redirects the build."""
    env = dict(os.environ)
    args = ["make", "-s", "-C", str(HERE)]
    target = LIB_PATH
    if out_dir is not None:
        args.append(f"OUT={out_dir}")
        target = Path(out_dir) / "libingot_oracle.so"
    if native:
        args.append("ARCH=-march=native")
    subprocess.run(args, check=True, env=env, capture_output=True)
    return target


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        build()
    lib = ctypes.CDLL(str(p))
    vp = ctypes.c_void_p
    lib.oracle_parse_one.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, vp, vp]
    lib.oracle_parse_one.restype = None
    lib.oracle_parse_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_int, vp, vp, ctypes.c_int]
    lib.oracle_parse_batch.restype = ctypes.c_int
    lib.oracle_be_bits.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32]
    lib.oracle_be_bits.restype = ctypes.c_uint64
    lib.oracle_v6eh_class.argtypes = [ctypes.c_uint8]
    lib.oracle_v6eh_class.restype = ctypes.c_int
    lib.oracle_toeplitz.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint32]
    lib.oracle_toeplitz.restype = ctypes.c_uint32
    lib.oracle_parse_geneve.argtypes = [vp, ctypes.c_uint32, vp]
    lib.oracle_parse_geneve.restype = None
    lib.oracle_geneve_fields_batch.argtypes = [vp, vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp]
    lib.oracle_geneve_fields_batch.restype = ctypes.c_int
    lib.oracle_parse_read_batch.argtypes = [vp, vp, vp, vp, ctypes.c_uint64, ctypes.c_int, vp,
                                            vp, vp, vp, ctypes.c_int]
    lib.oracle_parse_read_batch.restype = ctypes.c_int
    lib.oracle_set_passes.argtypes = [ctypes.c_int]
    lib.oracle_set_passes.restype = None
    lib.oracle_set_affinity.argtypes = [vp, ctypes.c_int]
    lib.oracle_set_affinity.restype = None
    if path is None:
        _lib = lib
    return lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def parse_one(frame: bytes, chain: Chain):
    """-> (ingot_rec, ingot_fields) as numpy structured scalars."""
    lib = load()
    buf = np.frombuffer(bytes(frame) + b"\0" * 8, dtype=np.uint8).copy()
    rec = np.zeros(1, dtype=REC_DTYPE)
    fld = np.zeros(1, dtype=FIELDS_DTYPE)
    lib.oracle_parse_one(_p(buf), len(frame), int(chain), _p(rec), _p(fld))
    return rec[0], fld[0]


def parse_batch(arena: np.ndarray, off: np.ndarray | None, lens: np.ndarray | None,
                chain: Chain, stride: int = 0, n: int | None = None, fields: bool = False,
                nthreads: int = 1, lib: ctypes.CDLL | None = None):
    lib = lib or load()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) if n is None else n
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        raise ValueError("n is required for the strided layout")
    rec = np.zeros(n, dtype=REC_DTYPE)
    fld = np.zeros(n, dtype=FIELDS_DTYPE) if fields else None
    rc = lib.oracle_parse_batch(_p(arena), _p(off), _p(lens), stride, n, int(chain), _p(rec),
                                _p(fld), nthreads)
    if rc != 0:
        raise ValueError("oracle_parse_batch: bad arguments")
    return (rec, fld) if fields else rec


def parse_geneve(frame: bytes):
    """GeneveOverV6Tunnel -> ingot_geneve_fields (numpy structured scalar;
    ["inner"]["rec"] is the record)."""
    lib = load()
    buf = np.frombuffer(bytes(frame) + b"\0" * 8, dtype=np.uint8).copy()
    out = np.zeros(1, dtype=GENEVE_FIELDS_DTYPE)
    lib.oracle_parse_geneve(_p(buf), len(frame), _p(out))
    return out[0]


def geneve_fields_batch(arena: np.ndarray, off: np.ndarray | None, lens: np.ndarray | None,
                        stride: int = 0, n: int | None = None, lib: ctypes.CDLL | None = None):
    lib = lib or load()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) if n is None else n
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    if n is None:
        raise ValueError("n is required for the strided layout")
    out = np.zeros(n, dtype=GENEVE_FIELDS_DTYPE)
    if lib.oracle_geneve_fields_batch(_p(arena), _p(off), _p(lens), stride, n, _p(out)) != 0:
        raise ValueError("oracle_geneve_fields_batch: bad arguments")
    return out


def segments(packets):
    """[[chunk bytes, ...], ...] -> (arena, seg_off u64, seg_len u16, pkt_seg u32):
    every chunk stored separately (16-B aligned, a gap after each)."""
    seg_off, seg_len, pkt_seg, parts, o = [], [], [0], [], 0
    for chunks in packets:
        for c in chunks:
            seg_off.append(o)
            seg_len.append(len(c))
            pad = (len(c) + 15) // 16 * 16 + 16
            parts.append(bytes(c) + b"\xee" * (pad - len(c)))
            o += pad
        pkt_seg.append(len(seg_off))
    # one unreferenced trailing entry keeps the tables non-empty (device
    # pointers must be non-NULL even when no packet has chunks)
    seg_off.append(o)
    seg_len.append(0)
    arena = np.frombuffer(b"".join(parts) + bytes(64), dtype=np.uint8).copy()
    return (arena, np.array(seg_off, dtype=np.uint64), np.array(seg_len, dtype=np.uint16),
            np.array(pkt_seg, dtype=np.uint32))


def parse_read_batch(arena, seg_off, seg_len, pkt_seg, chain: Chain, fields: str | None = None,
                     lib: ctypes.CDLL | None = None, nthreads: int = 1):
    """parse_read over multi-segment packets -> (records, field blocks or None,
    chunk index u16[n]).  fields: None, "fields" (ingot_fields) or "geneve"."""
    lib = lib or load()
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    seg_off = np.ascontiguousarray(seg_off, dtype=np.uint64)
    seg_len = np.ascontiguousarray(seg_len, dtype=np.uint16)
    pkt_seg = np.ascontiguousarray(pkt_seg, dtype=np.uint32)
    n = len(pkt_seg) - 1
    rec = np.zeros(n, dtype=REC_DTYPE)
    chunk = np.zeros(n, dtype=np.uint16)
    fld = gf = None
    if fields == "fields":
        fld = np.zeros(n, dtype=FIELDS_DTYPE)
    elif fields == "geneve":
        gf = np.zeros(n, dtype=GENEVE_FIELDS_DTYPE)
    rc = lib.oracle_parse_read_batch(_p(arena), _p(seg_off), _p(seg_len), _p(pkt_seg), n,
                                     int(chain), _p(rec), _p(fld), _p(gf), _p(chunk), nthreads)
    if rc != 0:
        raise ValueError("oracle_parse_read_batch: bad arguments")
    return rec, (fld if fld is not None else gf), chunk


def parse_read(chunks, chain: Chain, fields: str | None = None):
    """One packet given as a list of chunks -> (record, fields, chunk index)."""
    rec, f, ch = parse_read_batch(*segments([chunks]), chain, fields=fields)
    return rec[0], (None if f is None else f[0]), int(ch[0])


def be_set_bits(hdr: bytes, first_bit: int, n_bits: int, value: int) -> bytes:
    lib = load()
    lib.oracle_be_set_bits.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint64]
    buf = np.frombuffer(bytes(hdr), dtype=np.uint8).copy()
    lib.oracle_be_set_bits(_p(buf), first_bit, n_bits, value)
    return buf.tobytes()


def parse_modify_batch(arena: np.ndarray, off, lens, chain: Chain, edits, stride: int = 0,
                       n: int | None = None, lib: ctypes.CDLL | None = None, nthreads: int = 1):
    """In place on `arena` (numpy u8); returns the parse records."""
    lib = lib or load()
    lib.oracle_parse_modify_batch.argtypes = [ctypes.c_void_p] * 3 + [
        ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
        ctypes.c_void_p, ctypes.c_int]
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) if n is None else n
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    e = edits_array(edits)
    rec = np.zeros(n, dtype=REC_DTYPE)
    if lib.oracle_parse_modify_batch(_p(arena), _p(off), _p(lens), stride, n, int(chain), _p(e),
                                     len(e), _p(rec), nthreads) != 0:
        raise ValueError("oracle_parse_modify_batch: bad arguments")
    return rec


def parse_modify(frame: bytes, chain: Chain, edits):
    """-> (rewritten frame bytes, record)."""
    buf = np.frombuffer(bytes(frame) + bytes(8), dtype=np.uint8).copy()
    rec = parse_modify_batch(buf, np.array([0], dtype=np.uint64),
                             np.array([len(frame)], dtype=np.uint16), chain, edits)
    return buf[:len(frame)].tobytes(), rec[0]


def emit_batch(hdr: bytes, sets, src, off, lens, dst, dst_off=None, stride: int = 0,
               copy: bool = True, nthreads: int = 1, lib: ctypes.CDLL | None = None):
    """ingot_gpu_emit_packets (copy) / ingot_gpu_emit_headers semantics into
    the numpy u8 array `dst`, in place.  sets = [(at, Field, EmitSource, add[,
    per-packet numpy u16/u32 array]), ...]."""
    lib = lib or load()
    vp = ctypes.c_void_p
    lib.oracle_emit_batch.argtypes = [vp, ctypes.c_uint32, vp, ctypes.c_uint32, vp, vp, vp,
                                      ctypes.c_uint64, vp, vp, ctypes.c_uint32, ctypes.c_int,
                                      ctypes.c_int]
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    keep = []
    rows = []
    for e in sets:
        vals = e[4] if len(e) > 4 else None
        if vals is not None:
            vals = np.ascontiguousarray(vals)
            keep.append(vals)
        rows.append((e[0], e[1], e[2], e[3], None if vals is None else vals.ctypes.data))
    a = emit_sets_array(rows)
    hb = np.frombuffer(bytes(hdr) + b"\0", dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
    if dst_off is not None:
        dst_off = np.ascontiguousarray(dst_off, dtype=np.uint64)
    if lib.oracle_emit_batch(_p(hb), len(bytes(hdr)), _p(a), len(a), _p(src), _p(off), _p(lens),
                             len(lens), _p(dst), _p(dst_off), stride, int(copy),
                             nthreads) != 0:
        raise ValueError("oracle_emit_batch: bad arguments")
    return dst


def be_bits(hdr: bytes, first_bit: int, n_bits: int) -> int:
    buf = np.frombuffer(bytes(hdr) + b"\0" * 16, dtype=np.uint8).copy()
    return int(load().oracle_be_bits(_p(buf), first_bit, n_bits))


def v6eh_class(proto: int) -> int:
    return int(load().oracle_v6eh_class(proto))


def toeplitz(key: bytes, data: bytes) -> int:
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    d = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8).copy()
    return int(load().oracle_toeplitz(_p(k), len(key), _p(d), len(data)))


RSS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c"
                        "6a42b73bbeac01fa")


def flow_hist(arena, off, lens, chain: Chain, stride: int = 0, n: int | None = None,
              key: bytes = RSS_KEY, bins: int = 65536, hist: np.ndarray | None = None):
    """-> (hist u32[bins] (accumulated), per-packet hash u32[n]); the per-packet
    flow bins (INGOT_FLOW_NONE when not counted) are in `flow_hist.last_flows`."""
    lib = load()
    lib.oracle_flow_hist.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32, ctypes.c_uint64,
                                                             ctypes.c_int, ctypes.c_void_p,
                                                             ctypes.c_void_p, ctypes.c_uint32,
                                                             ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_flow_hist.restype = ctypes.c_int
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) if n is None else n
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    if hist is None:
        hist = np.zeros(bins, dtype=np.uint32)
    hashes = np.zeros(n, dtype=np.uint32)
    flows = np.zeros(n, dtype=np.uint32)
    k = np.frombuffer(bytes(key), dtype=np.uint8).copy()
    rc = lib.oracle_flow_hist(_p(arena), _p(off), _p(lens), stride, n, int(chain), _p(k),
                              _p(hist), bins, _p(hashes), _p(flows))
    if rc != 0:
        raise ValueError("oracle_flow_hist: bad arguments")
    flow_hist.last_flows = flows
    return hist, hashes


HEADER_KINDS = {"ethernet": 0, "vlan": 1, "ipv4": 2, "ipv6": 3, "tcp": 4, "udp": 5, "icmp": 6,
                "repeated_udp": 7, "geneve": 8}


def parse_header(kind: str, data: bytes):
    """Single-header `ValidX::parse`: -> (status, used, hint or None)."""
    lib = load()
    lib.oracle_parse_header.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint32)]
    lib.oracle_parse_header.restype = ctypes.c_int
    buf = np.frombuffer(bytes(data) + b"\0" * 8, dtype=np.uint8).copy()
    used, hint = ctypes.c_uint32(0), ctypes.c_uint32(0)
    st = lib.oracle_parse_header(HEADER_KINDS[kind], _p(buf), len(data), ctypes.byref(used),
                                 ctypes.byref(hint))
    h = None if hint.value == 0xFFFFFFFF else hint.value
    return st, used.value, h


def parse_header_batch(arena, off, lens, kind: int, hint=None, hints=None, stride: int = 0,
                       n: int | None = None) -> np.ndarray:
    """ingot_gpu_parse_header semantics: one ingot_hdr (8 B, as raw bytes
    per row) per slice."""
    lib = load()
    lib.oracle_parse_header_batch.argtypes = [ctypes.c_void_p] * 3 + [
        ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32,
        ctypes.c_void_p]
    lib.oracle_parse_header_batch.restype = ctypes.c_int
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) if n is None else n
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint16)
    if hints is not None:
        hints = np.ascontiguousarray(hints, dtype=np.uint32)
    out = np.zeros((n, 8), dtype=np.uint8)
    h = 0xFFFFFFFF if hint is None else int(hint)
    rc = lib.oracle_parse_header_batch(_p(arena), _p(off), _p(lens), stride, n, int(kind),
                                       _p(hints), h, _p(out))
    if rc != 0:
        raise ValueError("oracle_parse_header_batch: bad arguments")
    return out
