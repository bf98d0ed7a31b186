"""ingot_amd — MI355X-native batched L2/L3/L4 header extraction with ingot's
parse semantics.

Host-side mirror of the reference's parse interface above the C ABI
(include/ingot_gpu.h).  The batch API (`Context.parse*`) is the hot path; the
per-packet classes `UdpParser`, `GenericUlp`, `VlanUlp`, `GeneveOverV6Tunnel` mirror ingot's
`#[derive(Parse)]` chains (`Chain::parse(bytes) -> (headers, None, remainder)`
raising `PacketParseError{label, inner}`) so tests read like the reference's
own (ingot-examples/src/tests.rs); `GeneveOverV6Tunnel` adds the outer
layers (packets.rs:27-40).  Everything runs through the gfx950
library; nothing here parses bytes on the CPU.

Device memory, streams and torch.distributed come from PyTorch (plumbing).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

from . import _lib
from .abi import (  # noqa: F401  (re-exports)
    ABI_VERSION,
    CHAIN_LABELS,
    FIELDS_BYTES,
    FIELDS_DTYPE,
    GEN_SEED,
    GENEVE_FIELDS_DTYPE,
    MAX_GENEVE_OPT_FIELDS,
    REC_INNER,
    MAX_EH_FIELDS,
    REC_ACCEPTED,
    REC8_BYTES,
    REC8_DTYPE,
    REC_BYTES,
    REC_DTYPE,
    STATUS_OK,
    HDR_DTYPE,
    HINT_NONE,
    Chain,
    GenProfile,
    HeaderKind,
    IngotFields,
    IngotRec,
    IngotRec8,
    L3Kind,
    L4Kind,
    EditOp,
    EmitSource,
    Field,
    ParseError,
    edits_array,
    emit_sets_array,
    rec16_to_rec8,
)

__all__ = [
    "Chain", "Context", "GenProfile", "PacketParseError", "ParseError", "UdpParser",
    "GenericUlp", "VlanUlp", "GeneveOverV6Tunnel", "gen_frames", "gen_lengths", "records_to_numpy",
    "fields_to_numpy", "load_library", "Parsed", "chunk_tables", "HeaderKind", "parse_header",
    "HeaderParseError", "first_chunks",
]


def load_library() -> ctypes.CDLL:
    return _lib.load()


def _torch():
    import torch

    return torch


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(stream, device: Optional[int] = None) -> Optional[int]:
    """hipStream_t of `stream`; None = torch's current stream on `device`."""
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream(device)
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


# dtype names accepted for each C type of the ABI (16- and 32-bit tables may
# arrive as the signed view of the same bits)
_U8 = ("uint8",)
_U64 = ("int64", "uint64")
_U16 = ("uint16", "int16")
_U32 = ("int32", "uint32")


class PacketParseError(Exception):
    """ingot_types::PacketParseError (ingot-types/src/error.rs:119-171):
    the failing layer's label plus the ParseError."""

    def __init__(self, label: str, inner: ParseError):
        super().__init__(f"{label}: {inner.name}")
        self.label = label
        self.inner = inner

    def header(self) -> str:
        return self.label

    def error(self) -> ParseError:
        return self.inner


def _one_hip_runtime() -> None:
    """Refuse to run with two HIP runtimes mapped in this process (the
    library's from /opt/rocm beside PyTorch's own copy; _lib.load)."""
    try:
        with open("/proc/self/maps") as f:
            paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln and "/" in ln}
    except OSError:
        return
    real = {os.path.realpath(p) for p in paths}
    if len(real) > 1:
        raise RuntimeError(f"two HIP runtimes are loaded in this process: {sorted(real)}; "
                           "import torch before loading libingot_gpu.so")


class Context:
    """One device.  Mirrors `ingot_gpu_ctx`; all calls are async on `stream`
    (default: torch's current stream on that device)."""

    def __init__(self, device: int = 0):
        self._lib = _lib.load()
        _one_hip_runtime()
        h = ctypes.c_void_p()
        _lib.check(self._lib.ingot_gpu_ctx_create(int(device), ctypes.byref(h)),
                   "ingot_gpu_ctx_create")
        self._h = h
        self.device = int(device)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.ingot_gpu_ctx_destroy(self._h)
            self._h = None

    __del__ = close

    def set_tuning(self, key: int, value: int) -> None:
        """INGOT_TUNE_* knobs (window sizes, grid cap); never change results."""
        _lib.check(self._lib.ingot_gpu_ctx_set_tuning(self._h, int(key), int(value)),
                   "ingot_gpu_ctx_set_tuning")

    def get_tuning(self, key: int) -> int:
        return int(self._lib.ingot_gpu_ctx_get_tuning(self._h, int(key)))

    def stream_delay(self, ns: int, stream=None) -> None:
        """ingot_gpu_stream_delay: work enqueued on `stream` after this call
        starts `ns` nanoseconds (device wall clock) later — staggers the
        streams of a multi-stream ring consumer."""
        if not 0 <= int(ns) < (1 << 32):
            raise ValueError(f"ns out of range: {ns}")
        _lib.check(self._lib.ingot_gpu_stream_delay(self._h, int(ns),
                                                    _stream(stream, self.device)),
                   "ingot_gpu_stream_delay")

    def parse_packed(self, arena, lens, chain: Chain, out=None, off_out=None, workspace=None,
                     stream=None):
        """ingot_gpu_parse_packed: frames back to back in `arena`, only their
        lengths given (uint16); offsets derived on the device (optionally
        written to `off_out`, int64).  Returns the (n, 16) records."""
        torch = _torch()
        n = lens.numel()
        if out is None:
            out = torch.empty((n, REC_BYTES), dtype=torch.uint8, device=arena.device)
        wb = int(self._lib.ingot_gpu_packed_workspace_size(n))
        if workspace is None:
            workspace = torch.empty(wb, dtype=torch.uint8, device=arena.device)
        self._arg("arena", arena, _U8)
        self._arg("lens", lens, _U16, n)
        self._arg("out", out, _U8, n * REC_BYTES)
        self._arg("off_out", off_out, _U64, n, optional=True)
        self._arg("workspace", workspace, _U8, wb)
        self._on_device(arena=arena, lens=lens, out=out, off_out=off_out, workspace=workspace)
        _lib.check(self._lib.ingot_gpu_parse_packed(
            self._h, _ptr(arena), _ptr(lens), n, int(chain), _ptr(out), _ptr(off_out),
            _ptr(workspace), workspace.numel(), _stream(stream, self.device)),
            "ingot_gpu_parse_packed")
        return out

    def parse_header(self, arena, off, lens, kind, hint=None, hints=None, stride: int = 0,
                     n: Optional[int] = None, out=None, stream=None):
        """ingot_gpu_parse_header: `ValidX::parse(slice)` of header `kind`
        (HeaderKind) at every slice start, or a choice's `parse_choice(slice,
        hint)` (HeaderKind.L3 / L4 / Ulp; `hints` per slice or one `hint`,
        None = no hint).  Returns an (n, 8) uint8 tensor of ingot_hdr."""
        torch = _torch()
        if n is None:
            n = off.numel()
        if out is None:
            out = torch.empty((n, HDR_DTYPE.itemsize), dtype=torch.uint8, device=arena.device)
        self._frames(arena, off, lens, stride, n, align16=False)
        self._arg("hints", hints, _U32, n, optional=True)
        self._arg("out", out, _U8, n * HDR_DTYPE.itemsize)
        h = HINT_NONE if hint is None else int(hint)
        self._on_device(arena=arena, off=off, lens=lens, hints=hints, out=out)
        _lib.check(self._lib.ingot_gpu_parse_header(self._h, _ptr(arena), _ptr(off), _ptr(lens),
                                                    int(stride), n, int(kind), _ptr(hints), h,
                                                    _ptr(out), _stream(stream, self.device)),
                   "ingot_gpu_parse_header")
        return out

    def host_map(self, host) -> int:
        """ingot_gpu_host_map: the device address of host memory (a pinned
        torch tensor, or any C-contiguous numpy array / writable buffer, which
        is then page-locked).  Pass it as a raw pointer to the C ABI: the
        kernels read only the header bytes they touch across PCIe."""
        if hasattr(host, "data_ptr"):
            ptr, nbytes = host.data_ptr(), host.numel() * host.element_size()
        else:
            ptr, nbytes = host.ctypes.data, host.nbytes
        d = ctypes.c_void_p()
        _lib.check(self._lib.ingot_gpu_host_map(self._h, ptr, nbytes, ctypes.byref(d)),
                   "ingot_gpu_host_map")
        return int(d.value)

    def host_unmap(self, host) -> None:
        ptr = host.data_ptr() if hasattr(host, "data_ptr") else host.ctypes.data
        _lib.check(self._lib.ingot_gpu_host_unmap(self._h, ptr), "ingot_gpu_host_unmap")

    def _arg(self, name: str, t, dtypes, numel: Optional[int] = None,
             optional: bool = False) -> None:
        """Validate one buffer before its raw pointer crosses the C ABI:
        dtype (element size), contiguity and element count.  Only the
        buffers' shapes are checked here, not their contents: descriptor
        values (off[i] + lens[i] inside the arena, pkt_seg non-decreasing and
        inside the chunk table) are the caller's contract, as in the C ABI
        (include/ingot_gpu.h), and a bad descriptor is an out-of-bounds
        device read.  check_descriptors() verifies those values on demand."""
        if t is None:
            if optional:
                return
            raise ValueError(f"{name} is required")
        if not hasattr(t, "data_ptr") or not hasattr(t, "dtype"):
            raise TypeError(f"{name} must be a tensor")
        dt = str(t.dtype).replace("torch.", "")
        if dt not in dtypes:
            raise ValueError(f"{name} must be {' or '.join(dtypes)}, not {dt}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if numel is not None and t.numel() < numel:
            raise ValueError(f"{name} holds {t.numel()} elements, needs at least {numel}")

    def _on_device(self, **tensors) -> None:
        """After the shape checks: every buffer lives on the context's device."""
        for name, t in tensors.items():
            if t is not None and (not t.is_cuda or t.device.index != self.device):
                raise ValueError(f"{name} must live on cuda:{self.device}")

    def _frames(self, arena, off, lens, stride: int, n: int, align16: bool = True) -> None:
        """The frame descriptors of an indexed (off/lens) or slot (stride)
        arena: dtypes, counts and, for slots, that n slots fit the arena."""
        self._arg("arena", arena, _U8)
        if off is not None:
            self._arg("off", off, _U64, n)
            self._arg("lens", lens, _U16, n)
        else:
            if stride <= 0 or (align16 and stride % 16):
                raise ValueError("stride must be a positive multiple of 16"
                                 if align16 else "stride must be positive")
            if n * stride > arena.numel():
                raise ValueError(f"{n} slots of {stride} B exceed the {arena.numel()}-B arena")
            self._arg("lens", lens, _U16, n, optional=True)

    def parse(self, arena, off, lens, chain: Chain, out=None, stream=None):
        """Batched `<chain>::parse_slice` over frames (off[i], lens[i]) of arena.

        arena: uint8 cuda tensor; off: int64 (u64 offsets); lens: uint16.
        Returns an (n, 16) uint8 tensor of ingot_rec records.
        """
        torch = _torch()
        n = off.numel()
        if lens.numel() != n:
            raise ValueError("off and lens must have the same length")
        if out is None:
            out = torch.empty((n, REC_BYTES), dtype=torch.uint8, device=arena.device)
        self._frames(arena, off, lens, 0, n)
        self._arg("out", out, _U8, n * REC_BYTES)
        self._on_device(arena=arena, off=off, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_parse(self._h, _ptr(arena), _ptr(off), _ptr(lens), n,
                                             int(chain), _ptr(out), _stream(stream, self.device)),
                   "ingot_gpu_parse")
        return out

    def parse_strided(self, arena, stride: int, n: int, chain: Chain, lens=None, out=None,
                      stream=None):
        torch = _torch()
        if out is None:
            out = torch.empty((n, REC_BYTES), dtype=torch.uint8, device=arena.device)
        self._frames(arena, None, lens, stride, n)
        self._arg("out", out, _U8, n * REC_BYTES)
        self._on_device(arena=arena, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_parse_strided(self._h, _ptr(arena), int(stride),
                                                     _ptr(lens), n, int(chain), _ptr(out),
                                                     _stream(stream, self.device)),
                   "ingot_gpu_parse_strided")
        return out

    def parse_compact(self, arena, off, lens, chain: Chain, out=None, stream=None):
        """As parse(), with 8-byte ingot_rec8 records: (n, 8) uint8 tensor."""
        torch = _torch()
        n = off.numel()
        if out is None:
            out = torch.empty((n, REC8_BYTES), dtype=torch.uint8, device=arena.device)
        self._frames(arena, off, lens, 0, n)
        self._arg("out", out, _U8, n * REC8_BYTES)
        self._on_device(arena=arena, off=off, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_parse_compact(self._h, _ptr(arena), _ptr(off), _ptr(lens),
                                                     n, int(chain), _ptr(out),
                                                     _stream(stream, self.device)),
                   "ingot_gpu_parse_compact")
        return out

    def parse_strided_compact(self, arena, stride: int, n: int, chain: Chain, lens=None,
                              out=None, stream=None):
        torch = _torch()
        if out is None:
            out = torch.empty((n, REC8_BYTES), dtype=torch.uint8, device=arena.device)
        self._frames(arena, None, lens, stride, n)
        self._arg("out", out, _U8, n * REC8_BYTES)
        self._on_device(arena=arena, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_parse_strided_compact(
            self._h, _ptr(arena), int(stride), _ptr(lens), n, int(chain), _ptr(out),
            _stream(stream, self.device)), "ingot_gpu_parse_strided_compact")
        return out

    def parse_ring(self, arenas, stride: int, n: int, chain: Chain, outs, record_bytes: int = 16,
                   doorbell: "Optional[Doorbell]" = None, db_first: int = 0,
                   timeout_ms: int = 10000, status=None, stream=None) -> None:
        """ingot_gpu_parse_ring: one persistent launch parses len(arenas)
        batches of n slots (batch b: arenas[b] -> outs[b], (n, record_bytes)
        uint8).  doorbell=None: every batch is resident; else batch b starts
        once the doorbell reaches db_first + b (a wave gives up after
        timeout_ms and sets bit 0 of `status`, a zeroed int32 cuda tensor)."""
        nb = len(arenas)
        if len(outs) != nb:
            raise ValueError("one record buffer per batch")
        if nb > RING_MAX_BATCHES:
            raise ValueError(f"at most {RING_MAX_BATCHES} batches per launch")
        batches = (RingBatch * max(1, nb))()
        for b, (a, o) in enumerate(zip(arenas, outs)):
            self._frames(a, None, None, stride, n)
            self._arg("out", o, _U8, n * record_bytes)
            self._on_device(arena=a, out=o)
            batches[b].d_arena, batches[b].d_out = _ptr(a), _ptr(o)
        self._arg("status", status, _U32, 1, optional=True)
        self._on_device(status=status)
        _lib.check(self._lib.ingot_gpu_parse_ring(
            self._h, ctypes.cast(batches, ctypes.c_void_p), nb, int(stride), int(n), int(chain),
            int(record_bytes), doorbell._h if doorbell is not None else None, int(db_first),
            int(timeout_ms), _ptr(status), _stream(stream, self.device)), "ingot_gpu_parse_ring")

    def fields(self, arena, off, lens, chain: Chain, stride: int = 0, n: Optional[int] = None,
               out=None, stream=None):
        """Parity mode: (n, 256) uint8 tensor of ingot_fields blocks."""
        torch = _torch()
        if n is None:
            n = off.numel()
        if out is None:
            out = torch.empty((n, FIELDS_BYTES), dtype=torch.uint8, device=arena.device)
        self._frames(arena, off, lens, stride, n)
        self._arg("out", out, _U8, n * FIELDS_BYTES)
        self._on_device(arena=arena, off=off, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_fields(self._h, _ptr(arena), _ptr(off), _ptr(lens),
                                              int(stride), n, int(chain), _ptr(out),
                                              _stream(stream, self.device)),
                   "ingot_gpu_fields")
        return out

    def geneve_fields(self, arena, off, lens, stride: int = 0, n: Optional[int] = None,
                      out=None, stream=None):
        """GeneveOverV6Tunnel parity mode: (n, 384) uint8 tensor of
        ingot_geneve_fields (inner ingot_fields + outer ingot_tunnel_fields)."""
        torch = _torch()
        if n is None:
            n = off.numel()
        if out is None:
            out = torch.empty((n, GENEVE_FIELDS_DTYPE.itemsize), dtype=torch.uint8,
                              device=arena.device)
        self._frames(arena, off, lens, stride, n)
        self._arg("out", out, _U8, n * GENEVE_FIELDS_DTYPE.itemsize)
        self._on_device(arena=arena, off=off, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_geneve_fields(self._h, _ptr(arena), _ptr(off), _ptr(lens),
                                                     int(stride), n, _ptr(out),
                                                     _stream(stream, self.device)),
                   "ingot_gpu_geneve_fields")
        return out

    def parse_read(self, arena, seg_off, seg_len, pkt_seg, chain: Chain, out=None, chunk=None,
                   fields: Optional[str] = None, stream=None, first=None):
        """Batched `<chain>::parse_read` over multi-chunk packets (packet i =
        chunks pkt_seg[i]..pkt_seg[i+1] of (seg_off int64, seg_len uint16);
        pkt_seg int32/uint32 with n+1 entries).  Returns (out, chunk): records
        (fields=None), ingot_fields blocks (fields="fields") or
        ingot_geneve_fields blocks (fields="geneve"), and per packet the index
        of the chunk holding the remainder (uint16 stored in an int16 tensor).
        `first` (records only; int64/uint64, n entries, see first_chunks()):
        chunk 0 of every packet as (offset << 16) | length, which
        ingot_gpu_parse_read_first loads beside the chunk bounds."""
        torch = _torch()
        n = pkt_seg.numel() - 1
        width = {None: REC_BYTES, "fields": FIELDS_BYTES,
                 "geneve": GENEVE_FIELDS_DTYPE.itemsize}[fields]
        if out is None:
            out = torch.empty((n, width), dtype=torch.uint8, device=arena.device)
        if chunk is None:
            chunk = torch.empty(n, dtype=torch.int16, device=arena.device)
        self._arg("arena", arena, _U8)
        self._arg("pkt_seg", pkt_seg, _U32, n + 1)
        self._arg("seg_off", seg_off, _U64)
        self._arg("seg_len", seg_len, _U16, seg_off.numel())
        self._arg("out", out, _U8, n * width)
        self._arg("chunk", chunk, _U16, n)
        self._on_device(arena=arena, seg_off=seg_off, seg_len=seg_len, pkt_seg=pkt_seg, out=out,
                        chunk=chunk)
        st = _stream(stream, self.device)
        args = (self._h, _ptr(arena), _ptr(seg_off), _ptr(seg_len), _ptr(pkt_seg), n)
        if first is not None:
            if fields is not None:
                raise ValueError("first= is for 16-B records (ingot_gpu_parse_read_first)")
            self._arg("first", first, _U64, n)
            self._on_device(first=first)
            rc = self._lib.ingot_gpu_parse_read_first(*args[:5], _ptr(first), n, int(chain),
                                                      _ptr(out), _ptr(chunk), st)
            _lib.check(rc, "ingot_gpu_parse_read_first")
            return out, chunk
        if fields is None:
            rc = self._lib.ingot_gpu_parse_read(*args, int(chain), _ptr(out), _ptr(chunk), st)
        elif fields == "fields":
            rc = self._lib.ingot_gpu_fields_read(*args, int(chain), _ptr(out), _ptr(chunk), st)
        else:
            rc = self._lib.ingot_gpu_geneve_fields_read(*args, _ptr(out), _ptr(chunk), st)
        _lib.check(rc, "ingot_gpu_parse_read")
        return out, chunk

    def parse_read_dense(self, arena, seg, pkt_seg, chain: Chain, out=None, chunk=None,
                         fields: Optional[str] = None, stream=None):
        """parse_read over a dense chunk table (ingot_gpu_parse_read_dense):
        seg[k] = (offset << 16) | length as int64/uint64, one entry per
        chunk; pkt_seg int32/uint32 with n+1 bounds.  Returns (out, chunk)
        as parse_read does."""
        torch = _torch()
        n = pkt_seg.numel() - 1
        width = {None: REC_BYTES, "fields": FIELDS_BYTES,
                 "geneve": GENEVE_FIELDS_DTYPE.itemsize}[fields]
        if out is None:
            out = torch.empty((n, width), dtype=torch.uint8, device=arena.device)
        if chunk is None:
            chunk = torch.empty(n, dtype=torch.int16, device=arena.device)
        self._arg("arena", arena, _U8)
        self._arg("pkt_seg", pkt_seg, _U32, n + 1)
        self._arg("seg", seg, _U64)
        self._arg("out", out, _U8, n * width)
        self._arg("chunk", chunk, _U16, n)
        self._on_device(arena=arena, seg=seg, pkt_seg=pkt_seg, out=out, chunk=chunk)
        mode = {None: 0, "fields": 1, "geneve": 2}[fields]
        _lib.check(self._lib.ingot_gpu_parse_read_dense(
            self._h, _ptr(arena), _ptr(seg), _ptr(pkt_seg), n, int(chain), mode, _ptr(out),
            _ptr(chunk), _stream(stream, self.device)), "ingot_gpu_parse_read_dense")
        return out, chunk

    def parse_modify(self, arena, off, lens, chain: Chain, edits, stride: int = 0,
                     n: Optional[int] = None, out=None, stream=None):
        """Parse, then rewrite header fields in place (ingot's setters):
        edits = [(layer, Field, EditOp, value[, vlan index]), ...] applied in
        order to packets that parse Ok.  Returns the parse records if `out`
        (an (n, 16) uint8 tensor) is given, else None."""
        if n is None:
            n = off.numel()
        self._frames(arena, off, lens, stride, n)
        self._arg("out", out, _U8, n * REC_BYTES, optional=True)
        e = edits_array(edits)
        self._on_device(arena=arena, off=off, lens=lens, out=out)
        _lib.check(self._lib.ingot_gpu_parse_modify(
            self._h, _ptr(arena), _ptr(off), _ptr(lens), int(stride), n, int(chain),
            e.ctypes.data_as(ctypes.c_void_p), len(e), _ptr(out), _stream(stream, self.device)),
            "ingot_gpu_parse_modify")
        return out

    def _emit_sets(self, sets, n: int):
        """[(at, Field, EmitSource, add[, per-packet cuda tensor]), ...] ->
        (ingot_emit_set array, tensors kept alive for the call)."""
        rows, keep = [], []
        for e in sets:
            vals = e[4] if len(e) > 4 else None
            if vals is not None:
                want = _U16 if int(e[2]) == EmitSource.U16 else _U32
                self._arg("set values", vals, want, n)
                self._on_device(values=vals)
                keep.append(vals)
            rows.append((e[0], e[1], e[2], e[3], None if vals is None else vals.data_ptr()))
        return emit_sets_array(rows), keep

    def emit_packets(self, hdr: bytes, sets, src, off, lens, dst, dst_off, stream=None):
        """Batched Emit (ingot_gpu_emit_packets): packet i = the header block
        `hdr` (owned headers serialised once on the host, e.g. by emit_headers
        below) with the per-packet setters `sets` applied, then src[off[i] ..
        + lens[i]), written at dst + dst_off[i].  sets = [(at, Field,
        EmitSource, add[, per-packet u16/u32 cuda tensor]), ...]."""
        n = off.numel()
        hdr = bytes(hdr)
        self._arg("src", src, _U8)
        self._arg("off", off, _U64, n)
        self._arg("lens", lens, _U16, n)
        self._arg("dst", dst, _U8)
        self._arg("dst_off", dst_off, _U64, n)
        self._on_device(src=src, off=off, lens=lens, dst=dst, dst_off=dst_off)
        s, keep = self._emit_sets(sets, n)
        h = (ctypes.c_uint8 * max(len(hdr), 1)).from_buffer_copy(hdr or b"\0")
        _lib.check(self._lib.ingot_gpu_emit_packets(
            self._h, ctypes.addressof(h), len(hdr), s.ctypes.data_as(ctypes.c_void_p), len(s),
            _ptr(src), _ptr(off), _ptr(lens), n, _ptr(dst), _ptr(dst_off),
            _stream(stream, self.device)), "ingot_gpu_emit_packets")
        return dst

    def emit_header_blocks(self, hdr: bytes, sets, lens, out, out_off=None, stride: int = 0,
                           stream=None):
        """ingot_gpu_emit_headers: only the header blocks, packet i's at
        out + (out_off[i] if out_off is given else i * stride); LENGTH sets
        count len(hdr) + lens[i]."""
        n = lens.numel()
        hdr = bytes(hdr)
        self._arg("lens", lens, _U16, n)
        self._arg("out", out, _U8)
        self._arg("out_off", out_off, _U64, n, optional=True)
        self._on_device(lens=lens, out=out, out_off=out_off)
        s, keep = self._emit_sets(sets, n)
        h = (ctypes.c_uint8 * max(len(hdr), 1)).from_buffer_copy(hdr or b"\0")
        _lib.check(self._lib.ingot_gpu_emit_headers(
            self._h, ctypes.addressof(h), len(hdr), s.ctypes.data_as(ctypes.c_void_p), len(s),
            _ptr(lens), n, _ptr(out), _ptr(out_off), int(stride), _stream(stream, self.device)),
            "ingot_gpu_emit_headers")
        return out

    def flow_hist(self, arena, off, lens, chain: Chain, hist=None, bins: Optional[int] = None,
                  stride: int = 0, n: Optional[int] = None, key: Optional[bytes] = None,
                  flow=None, hashes=None, workspace=None, stream=None):
        """Flow classification (ingot_gpu_flow_hist / _ws).  Returns the
        per-packet flow bins (n x int32; INGOT_FLOW_NONE = -1 when not
        counted); `hist` (int32/uint32 cuda tensor of `bins` entries) is
        accumulated into if given; optional full Toeplitz hashes into
        `hashes`.  key=None: the standard RSS key.  `workspace`: a cuda
        tensor of >= flow_hist_workspace_size(n, bins) bytes selects the
        atomics-free histogram pass (flow_hist_workspace() makes one)."""
        torch = _torch()
        if n is None:
            n = off.numel()
        if bins is None:
            bins = hist.numel() if hist is not None else 65536
        if flow is None:
            flow = torch.empty(n, dtype=torch.int32, device=arena.device)
        self._frames(arena, off, lens, stride, n)
        self._arg("flow", flow, _U32, n)
        self._arg("hashes", hashes, _U32, n, optional=True)
        self._arg("hist", hist, _U32, bins, optional=True)
        if key is not None and len(bytes(key)) != 40:
            raise ValueError("key must be 40 bytes (the RSS key length)")
        kbuf = None if key is None else ctypes.create_string_buffer(bytes(key), 40)
        wbytes = 0 if workspace is None else workspace.numel() * workspace.element_size()
        if workspace is not None:
            self._arg("workspace", workspace, _U8)
        self._on_device(arena=arena, off=off, lens=lens, flow=flow, hashes=hashes, hist=hist, workspace=workspace)
        _lib.check(self._lib.ingot_gpu_flow_hist_ws(
            self._h, _ptr(arena), _ptr(off), _ptr(lens), int(stride), n, int(chain),
            ctypes.cast(kbuf, ctypes.c_void_p) if kbuf is not None else None, int(bins),
            _ptr(flow), _ptr(hashes), _ptr(hist), _ptr(workspace), wbytes,
            _stream(stream, self.device)),
            "ingot_gpu_flow_hist_ws")
        return flow

    def flow_hist_workspace_size(self, n: int, bins: int) -> int:
        """Bytes of workspace the atomics-free histogram pass needs (0: none)."""
        return int(self._lib.ingot_gpu_flow_hist_workspace_size(n, bins))

    def flow_hist_workspace(self, n: int, bins: int):
        """A device workspace for flow_hist(n, bins), or None when not used."""
        b = self.flow_hist_workspace_size(n, bins)
        if not b:
            return None
        return _torch().empty(b, dtype=_torch().uint8, device=f"cuda:{self.device}")


def first_chunks(seg_off, seg_len, pkt_seg):
    """ingot_gpu_parse_read_first's per-packet array from a chunk table:
    first[i] = (seg_off[pkt_seg[i]] << 16) | seg_len[pkt_seg[i]], 0 for a
    packet without chunks (int64 tensor on the tables' device)."""
    torch = _torch()
    ps = pkt_seg.to(torch.int64) & 0xFFFFFFFF
    lo, hi = ps[:-1], ps[1:]
    has = hi > lo
    idx = torch.where(has, lo, torch.zeros_like(lo))
    if seg_off.numel() == 0:
        return torch.zeros(lo.numel(), dtype=torch.int64, device=pkt_seg.device)
    o = seg_off.to(torch.int64)[idx]
    ln = seg_len.to(torch.int64)[idx] & 0xFFFF
    return torch.where(has, (o << 16) | ln, torch.zeros_like(o))


def check_descriptors(arena, off=None, lens=None, seg_off=None, seg_len=None, pkt_seg=None,
                      seg=None) -> None:
    """Check descriptor VALUES against the arena before a call (the calls
    check only shapes and dtypes): every frame (off[i], lens[i]) and every
    chunk (seg_off[k], seg_len[k]) — or dense entry seg[k] = offset << 16 |
    length — lies inside the arena, and pkt_seg is non-decreasing from 0 and
    ends inside the chunk table.  Raises ValueError; one reduction per array,
    on the arrays' own device."""
    size = int(arena.numel())

    def inside(o, ln, what):
        if o is None or o.numel() == 0:
            return
        end = o.to(_torch().int64) + ln.to(_torch().int64) if ln is not None else o
        if int(o.min()) < 0 or int(end.max()) > size:
            raise ValueError(f"{what} reach past the {size}-B arena")

    if off is not None:
        inside(off, lens.to(_torch().int32) & 0xFFFF, "frames (off + lens)")
    if seg_off is not None:
        inside(seg_off, seg_len.to(_torch().int32) & 0xFFFF, "chunks (seg_off + seg_len)")
    nseg = seg_off.numel() if seg_off is not None else (seg.numel() if seg is not None else None)
    if seg is not None:
        inside(seg >> 16, seg & 0xFFFF, "dense chunks")
    if pkt_seg is not None:
        ps = pkt_seg.to(_torch().int64) & 0xFFFFFFFF
        if ps.numel() == 0 or int(ps[0]) != 0:
            raise ValueError("pkt_seg must start at 0")
        if ps.numel() > 1 and bool((ps[1:] < ps[:-1]).any()):
            raise ValueError("pkt_seg must be non-decreasing")
        if nseg is not None and int(ps[-1]) > nseg:
            raise ValueError(f"pkt_seg ends at {int(ps[-1])}, past the {nseg}-chunk table")


RING_MAX_BATCHES = 64  # INGOT_RING_MAX_BATCHES


class RingBatch(ctypes.Structure):
    """ingot_ring_batch"""
    _fields_ = [("d_arena", ctypes.c_void_p), ("d_out", ctypes.c_void_p)]


class Doorbell:
    """ingot_gpu_doorbell: launches enqueued after `wait(value, stream)` run
    once the doorbell word reaches `value` (rung from the host by `ring`)."""

    def __init__(self, ctx: Context):
        self._lib = _lib.load()
        h, word = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(self._lib.ingot_gpu_doorbell_create(ctx._h, ctypes.byref(h),
                                                       ctypes.byref(word)),
                   "ingot_gpu_doorbell_create")
        self._h = h
        self.device = ctx.device

    def wait(self, value: int, stream=None) -> None:
        _lib.check(self._lib.ingot_gpu_doorbell_wait(self._h, int(value),
                                                     _stream(stream, self.device)),
                   "ingot_gpu_doorbell_wait")

    def ring(self, value: int) -> None:
        _lib.check(self._lib.ingot_gpu_doorbell_ring(self._h, int(value)),
                   "ingot_gpu_doorbell_ring")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.ingot_gpu_doorbell_destroy(self._h)
            self._h = None


COMM_ID_BYTES = 128  # INGOT_COMM_ID_BYTES


def comm_unique_id() -> bytes:
    """ingot_gpu_comm_unique_id: a new communicator id (rank 0 makes it; the
    host sends the bytes to every rank)."""
    lib = _lib.load()
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    _lib.check(lib.ingot_gpu_comm_unique_id(buf), "ingot_gpu_comm_unique_id")
    return bytes(buf)


class Comm:
    """ingot_gpu_comm: the RCCL communicator of config 5's histogram reduce,
    bound to `ctx`'s device.  Creating it blocks until all `nranks` ranks
    have joined with the same `uid`."""

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"a communicator id is {COMM_ID_BYTES} bytes")
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        _lib.check(self._lib.ingot_gpu_comm_create(ctx._h, int(nranks), int(rank), buf,
                                                   ctypes.byref(h)), "ingot_gpu_comm_create")
        self._bind(h, ctx)

    def _bind(self, h, ctx, owner=None):
        self._h = h
        self._owner = owner  # a borrowed communicator's owner, kept alive
        self.device = ctx.device
        self.size = int(self._lib.ingot_gpu_comm_size(h))
        self.rank = int(self._lib.ingot_gpu_comm_rank(h))

    @classmethod
    def wrap(cls, ctx: Context, nccl_comm: int, owner=None) -> "Comm":
        """ingot_gpu_comm_wrap: borrow an RCCL communicator the process
        already holds (an ncclComm_t address) instead of creating a second
        one; close()/abort() release only the handle.  `owner` is kept alive
        with it."""
        self = cls.__new__(cls)
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.ingot_gpu_comm_wrap(ctx._h, ctypes.c_void_p(int(nccl_comm)),
                                                 ctypes.byref(h)), "ingot_gpu_comm_wrap")
        self._bind(h, ctx, owner)
        return self

    @classmethod
    def from_process_group(cls, ctx: Context, group=None) -> "Comm":
        """The communicator of torch.distributed's RCCL group (the default
        group unless `group`) on ctx's device, borrowed: one RCCL
        communicator per process.  The group must be up on
        that device (init_process_group(..., device_id=...) or a first
        collective) and must outlive the handle."""
        torch = _torch()
        import torch.distributed as dist

        pg = group if group is not None else dist.group.WORLD
        backend = pg._get_backend(torch.device("cuda", ctx.device))
        ptr = backend._comm_ptr()
        if not ptr:
            raise RuntimeError("the process group has no RCCL communicator on "
                               f"cuda:{ctx.device} yet")
        return cls.wrap(ctx, ptr, owner=pg)

    def allreduce_hist(self, hist, stream=None):
        """ingot_gpu_flow_hist_allreduce: in-place sum of a (bins,) u32 / i32
        histogram over the ranks, enqueued on `stream` (default: torch's
        current stream).  Returns `hist`."""
        if hist.element_size() != 4 or not hist.is_contiguous() or not hist.is_cuda:
            raise ValueError("hist must be a contiguous 32-bit device tensor")
        if hist.device.index != self.device:
            raise ValueError(f"hist is on {hist.device}, the communicator on cuda:{self.device}")
        _lib.check(self._lib.ingot_gpu_flow_hist_allreduce(
            self._h, hist.data_ptr(), hist.numel(), _stream(stream, self.device)),
            "ingot_gpu_flow_hist_allreduce")
        return hist

    def close(self) -> None:
        """ingot_gpu_comm_destroy: every rank together, after its reduces."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _lib.check(self._lib.ingot_gpu_comm_destroy(h), "ingot_gpu_comm_destroy")

    def abort(self) -> None:
        """ingot_gpu_comm_abort: local and immediate."""
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _lib.check(self._lib.ingot_gpu_comm_abort(h), "ingot_gpu_comm_abort")


def records_to_numpy(t):
    """(n, 16) uint8 tensor/array -> numpy structured array of ingot_rec."""
    import numpy as np

    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return np.ascontiguousarray(a).view(REC_DTYPE).reshape(-1)


def fields_to_numpy(t):
    import numpy as np

    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return np.ascontiguousarray(a).view(FIELDS_DTYPE).reshape(-1)


def geneve_fields_to_numpy(t):
    import numpy as np

    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return np.ascontiguousarray(a).view(GENEVE_FIELDS_DTYPE).reshape(-1)


# ---------------------------------------------------------------------------
# Synthetic traffic (include/ingot_pktgen.h)
# ---------------------------------------------------------------------------
def gen_lengths(profile: GenProfile, n: int, seed: int = GEN_SEED, first: int = 0,
                device: int = 0, stream=None):
    torch = _torch()
    lens = torch.empty(n, dtype=torch.uint16, device=f"cuda:{device}")
    _lib.check(_lib.load().ingot_pktgen_lengths(int(profile), seed, first, n, _ptr(lens),
                                                _stream(stream, device)), "ingot_pktgen_lengths")
    return lens


def gen_frames(profile: GenProfile, n: int, seed: int = GEN_SEED, first: int = 0,
               stride: Optional[int] = None, device: int = 0, stream=None, slack: int = 256):
    """Generate n frames on `device`.  Returns (arena, off, lens).

    stride=None packs frames back-to-back (u64 offsets); a stride lays them
    out one per slot (off=None).  `slack` extra arena bytes follow the last
    frame.
    """
    torch = _torch()
    dev = f"cuda:{device}"
    lib = _lib.load()
    if stride is not None:
        if profile == GenProfile.V4UDP64:
            lens = None
        else:
            lens = gen_lengths(profile, n, seed, first, device, stream)
            lens = torch.minimum(lens.to(torch.int32), torch.tensor(stride, device=dev)).to(
                torch.uint16)
        nbytes = n * stride + slack
        arena = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        _lib.check(lib.ingot_pktgen_fill(int(profile), seed, first, n, None, int(stride),
                                         _ptr(lens), _ptr(arena), nbytes,
                                         _stream(stream, device)),
                   "ingot_pktgen_fill")
        return arena, None, lens
    lens = gen_lengths(profile, n, seed, first, device, stream)
    ends = lens.to(torch.int64).cumsum(0)
    off = ends - lens.to(torch.int64)
    total = int(ends[-1].item()) if n else 0
    nbytes = total + slack
    arena = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    _lib.check(lib.ingot_pktgen_fill(int(profile), seed, first, n, _ptr(off), 0, _ptr(lens),
                                     _ptr(arena), nbytes, _stream(stream, device)),
               "ingot_pktgen_fill")
    return arena, off, lens


# ---------------------------------------------------------------------------
# Per-packet mirror of ingot's chain API, on the device path.
# ---------------------------------------------------------------------------
@dataclass
class _View:
    """Getter view over one parsed header (values from the ingot_fields block)."""

    frame: bytes
    f: object  # numpy.void of FIELDS_DTYPE
    off: int


class EthernetView(_View):
    def destination(self) -> bytes:
        return bytes(self.f["eth_destination"])

    def source(self) -> bytes:
        return bytes(self.f["eth_source"])

    def ethertype(self) -> int:
        return int(self.f["eth_ethertype"])


class OuterEthernetView(_View):
    def destination(self) -> bytes:
        return bytes(self.f["outer_eth_destination"])

    def source(self) -> bytes:
        return bytes(self.f["outer_eth_source"])

    def ethertype(self) -> int:
        return int(self.f["outer_eth_ethertype"])


class OuterIpv6View(_View):
    def __getattr__(self, name):
        key = "outer_v6_" + name
        if key in GENEVE_FIELDS_DTYPE["outer"].names:
            v = self.f[key]
            return (lambda: bytes(v)) if v.shape else (lambda: int(v))
        raise AttributeError(name)

    def v6ext_bytes(self) -> bytes:
        return self.frame[self.off + 40:self.off + 40 + int(self.f["outer_v6_ext_len"])]

    def next_layer(self) -> int:
        return int(self.f["outer_l4_proto"])


class OuterUdpView(_View):
    def source(self) -> int:
        return int(self.f["outer_udp_source"])

    def destination(self) -> int:
        return int(self.f["outer_udp_destination"])

    def length(self) -> int:
        return int(self.f["outer_udp_length"])

    def checksum(self) -> int:
        return int(self.f["outer_udp_checksum"])


@dataclass
class GeneveOpt:
    """ingot::geneve::GeneveOpt (geneve.rs:80-102) with its data bytes."""

    opt_class: int
    option_type: int
    reserved: int
    length: int
    data: bytes

    def is_critical(self) -> bool:
        return (self.option_type >> 7) == 1


class GeneveView(_View):
    """ingot::geneve::ValidGeneve getters (geneve.rs:16-44)."""

    def version(self) -> int:
        return int(self.f["geneve_version"])

    def opt_len(self) -> int:
        return int(self.f["geneve_opt_len"])

    def flags(self) -> int:
        return int(self.f["geneve_flags"])

    def protocol_type(self) -> int:
        return int(self.f["geneve_protocol_type"])

    def vni(self) -> int:
        return int(self.f["geneve_vni"])

    def reserved(self) -> int:
        return int(self.f["geneve_reserved"])

    def options_ref(self) -> bytes:
        return self.frame[self.off + 8:self.off + 8 + 4 * self.opt_len()]

    def packet_length(self) -> int:
        return 8 + 4 * self.opt_len()

    def options(self) -> list:
        """The first MAX_GENEVE_OPT_FIELDS options (n_options() is exact)."""
        out = []
        for g in self.f["geneve_opt"][:min(self.n_options(), MAX_GENEVE_OPT_FIELDS)]:
            o, ln = int(g["data_off"]), int(g["length"])
            out.append(GeneveOpt(int(g["opt_class"]), int(g["option_type"]), int(g["reserved"]),
                                 ln, self.frame[o:o + 4 * ln]))
        return out

    def n_options(self) -> int:
        return int(self.f["geneve_n_opts"])


class VlanView(_View):
    idx: int = 0

    def priority(self) -> int:
        return int(self.f["vlan_priority"][self.idx])

    def dei(self) -> int:
        return int(self.f["vlan_dei"][self.idx])

    def vid(self) -> int:
        return int(self.f["vlan_vid"][self.idx])

    def ethertype(self) -> int:
        return int(self.f["vlan_ethertype"][self.idx])


class Ipv4View(_View):
    kind = L3Kind.IPV4

    def __getattr__(self, name):
        key = "v4_" + name
        if key in FIELDS_DTYPE.names:
            v = self.f[key]
            return (lambda: bytes(v)) if v.shape else (lambda: int(v))
        raise AttributeError(name)

    def options_ref(self) -> bytes:
        o, n = int(self.f["v4_options_off"]), int(self.f["v4_options_len"])
        return self.frame[o:o + n]

    def next_layer(self) -> int:
        return int(self.f["v4_protocol"])


@dataclass
class V6Eh:
    kind: int
    next_header: int
    ext_len: int
    fragment_offset: int
    res: int
    more_frags: int
    ident: int
    off: int


class Ipv6View(_View):
    kind = L3Kind.IPV6
    hint: int = 0

    def __getattr__(self, name):
        key = "v6_" + name
        if key in FIELDS_DTYPE.names:
            v = self.f[key]
            return (lambda: bytes(v)) if v.shape else (lambda: int(v))
        raise AttributeError(name)

    def extension_headers(self) -> list:
        n = min(int(self.f["rec"]["n_v6ext"]), MAX_EH_FIELDS)
        out = []
        for e in self.f["v6_eh"][:n]:
            frm = int(e["frag_res_more"])
            out.append(V6Eh(int(e["kind"]), int(e["next_header"]), int(e["ext_len"]),
                            int(e["frag_offset"]), frm >> 1, frm & 1, int(e["ident"]),
                            int(e["off"])))
        return out

    def v6ext_bytes(self) -> bytes:
        o, n = int(self.f["v6_ext_off"]), int(self.f["v6_ext_len"])
        return self.frame[o:o + n]

    def next_layer(self) -> int:
        return self.hint


class TcpView(_View):
    kind = L4Kind.TCP

    def source(self) -> int:
        return int(self.f["l4_source"])

    def destination(self) -> int:
        return int(self.f["l4_destination"])

    def __getattr__(self, name):
        key = "tcp_" + name
        if key in FIELDS_DTYPE.names:
            return lambda: int(self.f[key])
        raise AttributeError(name)

    def options_ref(self) -> bytes:
        o, n = int(self.f["tcp_options_off"]), int(self.f["tcp_options_len"])
        return self.frame[o:o + n]


class UdpView(_View):
    kind = L4Kind.UDP

    def source(self) -> int:
        return int(self.f["l4_source"])

    def destination(self) -> int:
        return int(self.f["l4_destination"])

    def length(self) -> int:
        return int(self.f["udp_length"])

    def checksum(self) -> int:
        return int(self.f["udp_checksum"])


class IcmpView(_View):
    def ty(self) -> int:
        return int(self.f["icmp_ty"])

    def code(self) -> int:
        return int(self.f["icmp_code"])

    def checksum(self) -> int:
        return int(self.f["icmp_checksum"])

    def rest_of_hdr(self) -> bytes:
        return bytes(self.f["icmp_rest_of_hdr"])


class IcmpV4View(IcmpView):
    kind = L4Kind.ICMPV4


class IcmpV6View(IcmpView):
    kind = L4Kind.ICMPV6


@dataclass
class Headers:
    """The parsed chain (`ValidUdpParser` etc.): one attribute per layer,
    named as the reference struct's fields; Option<> layers may be None."""

    names: tuple
    layers: dict
    rec: object

    def __getattr__(self, name):
        layers = self.__dict__.get("layers", {})
        if name in layers:
            return layers[name]
        raise AttributeError(name)


_default_ctx: dict = {}


def _ctx_for(device: int) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def parse_frames(frames: list, chain: Chain, device: int = 0):
    """Run the device fields kernel on a list of frames; returns (records
    structured array, fields structured array)."""
    import numpy as np

    torch = _torch()
    ctx = _ctx_for(device)
    dev = f"cuda:{device}"
    lens_l = [len(f) for f in frames]
    offs_l, o = [], 0
    for ln in lens_l:
        offs_l.append(o)
        o += (ln + 15) // 16 * 16 + 16
    buf = np.zeros(max(o, 16) + 64, dtype=np.uint8)
    for f, off in zip(frames, offs_l):
        buf[off:off + len(f)] = np.frombuffer(bytes(f), dtype=np.uint8)
    arena = torch.from_numpy(buf).to(dev)
    off = torch.tensor(offs_l, dtype=torch.int64, device=dev)
    lens = torch.tensor(lens_l, dtype=torch.int32, device=dev).to(torch.uint16)
    recs = ctx.parse(arena, off, lens, chain)
    if chain == Chain.GeneveOverV6Tunnel:
        flds = geneve_fields_to_numpy(ctx.geneve_fields(arena, off, lens))
    else:
        flds = fields_to_numpy(ctx.fields(arena, off, lens, chain))
    torch.cuda.synchronize(device)
    return records_to_numpy(recs), flds


class HeaderParseError(Exception):
    """A single header's ParseError (HeaderParse::parse returns a bare
    ParseError, ingot-types/src/lib.rs:137-147)."""

    def __init__(self, inner: ParseError):
        super().__init__(inner.name)
        self.inner = inner


def parse_header(kind: HeaderKind, data: bytes, hint: Optional[int] = None, device: int = 0):
    """`ValidX::parse(data)` for header `kind`, or a choice's
    `parse_choice(data, hint)` (HeaderKind.L3 / L4 / Ulp), on the device:
    -> (variant HeaderKind, HeaderLen, NextLayer hint or None, remainder
    bytes), or raises HeaderParseError."""
    import numpy as np

    torch = _torch()
    data = bytes(data)
    dev = f"cuda:{device}"
    arena = torch.from_numpy(np.frombuffer(data + bytes(16), np.uint8).copy()).to(dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    lens = torch.tensor([len(data)], dtype=torch.int32).to(torch.uint16).to(dev)
    out = _ctx_for(device).parse_header(arena, off, lens, kind, hint=hint).cpu().numpy()
    status, variant = int(out[0, 0]), int(out[0, 1])
    used = int(out[0, 2]) | int(out[0, 3]) << 8
    h = int(out[0, 4:8].view(np.uint32)[0])
    if status:
        raise HeaderParseError(ParseError(status))
    return HeaderKind(variant), used, (None if h == HINT_NONE else h), data[used:]


def chunk_tables(packets):
    """Host-side chunk tables for Context.parse_read: packets = [[chunk bytes,
    ...], ...] -> (arena u8, seg_off u64, seg_len u16, pkt_seg u32) numpy
    arrays, each chunk stored apart (16-B aligned, a gap after it)."""
    import numpy as np

    seg_off, seg_len, pkt_seg, parts, o = [], [], [0], [], 0
    for chunks in packets:
        for c in chunks:
            pad = (len(c) + 15) // 16 * 16 + 16
            seg_off.append(o)
            seg_len.append(len(c))
            parts.append(bytes(c) + bytes(pad - len(c)))
            o += pad
        pkt_seg.append(len(seg_off))
    seg_off.append(o)  # one unreferenced entry keeps the tables non-empty
    seg_len.append(0)
    arena = np.frombuffer(b"".join(parts) + bytes(64), dtype=np.uint8).copy()
    return (arena, np.array(seg_off, dtype=np.uint64), np.array(seg_len, dtype=np.uint16),
            np.array(pkt_seg, dtype=np.uint32))


@dataclass
class Parsed:
    """ingot_types::Parsed (parse_read's Ok value, ingot-macros/src/parse.rs:
    525-535): the headers, the chunks not yet read, and the rest of the chunk
    holding the remainder (None when that chunk was consumed exactly)."""

    headers: object
    data: list
    last_chunk: Optional[bytes]


class _ChainParser:
    chain: Chain
    names: tuple

    @classmethod
    def parse_read(cls, chunks, device: int = 0) -> Parsed:
        """`<Chain>::parse_read(chunks)` on the device, or raises
        PacketParseError (StraddledHeader when a header crosses a chunk end
        and more chunks follow)."""
        torch = _torch()
        chunks = [bytes(c) for c in chunks]
        arena, so, sl, ps = chunk_tables([chunks])
        dev = f"cuda:{device}"
        d = (torch.from_numpy(arena).to(dev), torch.from_numpy(so.view("int64")).to(dev),
             torch.from_numpy(sl.view("int16")).to(dev), torch.from_numpy(ps.view("int32")).to(dev))
        tun = cls.chain == Chain.GeneveOverV6Tunnel
        out, ch = _ctx_for(device).parse_read(*d, cls.chain, fields="geneve" if tun else "fields")
        torch.cuda.synchronize(device)
        f = (geneve_fields_to_numpy if tun else fields_to_numpy)(out)[0]
        k = int(ch.cpu().numpy().view("uint16")[0])
        frame = b"".join(chunks)
        r = f["inner"]["rec"] if tun else f["rec"]
        hdrs, _, _ = cls._assemble(frame, r, f)
        end = sum(len(c) for c in chunks[:k + 1])
        po = int(r["payload_off"])
        return Parsed(hdrs, chunks[k + 1:], frame[po:end] if end > po else None)

    @classmethod
    def parse(cls, frame: bytes, device: int = 0):
        """`<Chain>::parse(frame)` on the device: (headers, None, remainder),
        or raises PacketParseError(label, ParseError)."""
        recs, flds = parse_frames([bytes(frame)], cls.chain, device)
        return cls._assemble(bytes(frame), recs[0], flds[0])

    parse_slice = parse

    @classmethod
    def _assemble(cls, frame: bytes, r, f):
        status = int(r["status"])
        if status != STATUS_OK:
            raise PacketParseError(CHAIN_LABELS[cls.chain][int(r["err_layer"])],
                                   ParseError(status))
        layers = {}
        eth_name, l3_name, l4_name = cls.names[0], cls.names[-2], cls.names[-1]
        eth_off = 0
        if cls.chain == Chain.GeneveOverV6Tunnel:
            t, f = f["outer"], f["inner"]
            eth_name, eth_off = "inner_eth", int(t["inner_eth_off"])
            layers["outer_eth"] = OuterEthernetView(frame, t, 0)
            layers["outer_v6"] = OuterIpv6View(frame, t, 14)
            layers["outer_udp"] = OuterUdpView(frame, t, int(t["outer_udp_off"]))
            layers["outer_encap"] = GeneveView(frame, t, int(t["geneve_off"]))
        layers[eth_name] = EthernetView(frame, f, eth_off)
        if cls.chain == Chain.VlanUlp:
            tags = []
            for k in range(int(r["n_vlan"])):
                v = VlanView(frame, f, 14 + 4 * k)
                v.idx = k
                tags.append(v)
            layers["vlan"] = tags
        l3 = None
        if int(r["l3_kind"]) == L3Kind.IPV4:
            l3 = Ipv4View(frame, f, int(r["l3_off"]))
        elif int(r["l3_kind"]) == L3Kind.IPV6:
            l3 = Ipv6View(frame, f, int(r["l3_off"]))
            l3.hint = int(r["l4_proto"])
        layers[l3_name] = l3
        l4 = None
        k4 = int(r["l4_kind"])
        cls4 = {L4Kind.TCP: TcpView, L4Kind.UDP: UdpView, L4Kind.ICMPV4: IcmpV4View,
                L4Kind.ICMPV6: IcmpV6View}.get(k4)
        if cls4 is not None:
            l4 = cls4(frame, f, int(r["l4_off"]))
        layers[l4_name] = l4
        hdrs = Headers(cls.names, layers, r)
        return hdrs, None, frame[int(r["payload_off"]):]


class UdpParser(_ChainParser):
    """ingot-examples/src/packets.rs:18-24"""

    chain = Chain.UdpParser
    names = ("eth", "l3", "l4")


class GenericUlp(_ChainParser):
    """ingot-examples/src/packets.rs:54-60"""

    chain = Chain.GenericUlp
    names = ("inner_eth", "inner_l3", "inner_ulp")


class VlanUlp(_ChainParser):
    """Build-defined Ethernet / 0-2 VlanBody / L3 / Ulp chain."""

    chain = Chain.VlanUlp
    names = ("eth", "vlan", "l3", "l4")


class GeneveOverV6Tunnel(_ChainParser):
    """ingot-examples/src/packets.rs:27-40 (OPTE's inbound path)."""

    chain = Chain.GeneveOverV6Tunnel
    names = ("outer_eth", "outer_v6", "outer_udp", "outer_encap", "inner_eth", "inner_l3",
             "inner_ulp")
