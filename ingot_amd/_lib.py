"""ctypes binding of the in-tree native library (ingot_amd/lib/libingot_gpu.so).

The library is the product: there is no Python or CPU fallback for any entry
point.  If it is missing, importing the compute API raises, loudly.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libingot_gpu.so"

c_u8p = ctypes.c_void_p
c_u64 = ctypes.c_uint64

# (name, restype, argtypes) — exactly the declarations of include/ingot_gpu.h
# and include/ingot_pktgen.h.
SIGNATURES = {
    "ingot_gpu_abi_version": (ctypes.c_int, []),
    "ingot_gpu_build_info": (ctypes.c_char_p, []),
    "ingot_gpu_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "ingot_gpu_ctx_destroy": (None, [ctypes.c_void_p]),
    "ingot_gpu_ctx_device": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_packed_workspace_size": (ctypes.c_size_t, [c_u64]),
    "ingot_gpu_parse_packed": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, c_u8p, ctypes.c_void_p,
         ctypes.c_size_t, ctypes.c_void_p],
    ),
    "ingot_gpu_parse_header": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_uint32, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_host_map": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "ingot_gpu_host_unmap": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ingot_gpu_doorbell_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                                 ctypes.POINTER(ctypes.c_void_p)]),
    "ingot_gpu_doorbell_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32,
                                               ctypes.c_void_p]),
    "ingot_gpu_doorbell_ring": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    "ingot_gpu_doorbell_destroy": (None, [ctypes.c_void_p]),
    "ingot_gpu_stream_delay": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]),
    "ingot_gpu_ctx_set_tuning": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "ingot_gpu_ctx_get_tuning": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "ingot_gpu_parse": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_parse_strided": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, ctypes.c_uint32, c_u8p, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_parse_ring": (
        ctypes.c_int,
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, c_u64, ctypes.c_int,
         ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_parse_compact": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_parse_strided_compact": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, ctypes.c_uint32, c_u8p, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_fields": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_geneve_fields": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_parse_read": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_parse_read_first": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_fields_read": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, c_u8p, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_parse_read_dense": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u64, ctypes.c_int, ctypes.c_int, c_u8p, c_u8p,
         ctypes.c_void_p],
    ),
    "ingot_gpu_geneve_fields_read": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, c_u8p, c_u64, c_u8p, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_parse_modify": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_uint32, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_emit_packets": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, ctypes.c_uint32, c_u8p, ctypes.c_uint32, c_u8p, c_u8p, c_u8p,
         c_u64, c_u8p, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_emit_headers": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, ctypes.c_uint32, c_u8p, ctypes.c_uint32, c_u8p, c_u64, c_u8p,
         c_u8p, ctypes.c_uint32, ctypes.c_void_p],
    ),
    "ingot_gpu_flow_hist": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_uint32, c_u8p, c_u8p, c_u8p, ctypes.c_void_p],
    ),
    "ingot_gpu_flow_hist_ws": (
        ctypes.c_int,
        [ctypes.c_void_p, c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u64, ctypes.c_int, c_u8p,
         ctypes.c_uint32, c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_size_t, ctypes.c_void_p],
    ),
    "ingot_gpu_flow_hist_workspace_size": (ctypes.c_size_t, [c_u64, ctypes.c_uint32]),
    "ingot_gpu_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_comm_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "ingot_gpu_comm_wrap": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_void_p)]),
    "ingot_gpu_comm_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_comm_abort": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_comm_size": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_comm_rank": (ctypes.c_int, [ctypes.c_void_p]),
    "ingot_gpu_flow_hist_allreduce": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_uint32,
                                                     ctypes.c_void_p]),
    "ingot_gpu_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "ingot_parse_error_name": (ctypes.c_char_p, [ctypes.c_int]),
    "ingot_chain_layer_label": (ctypes.c_char_p, [ctypes.c_int, ctypes.c_int]),
    "ingot_chain_layer_count": (ctypes.c_int, [ctypes.c_int]),
    "ingot_pktgen_lengths": (
        ctypes.c_int, [ctypes.c_int, c_u64, c_u64, c_u64, c_u8p, ctypes.c_void_p],
    ),
    "ingot_pktgen_fill": (
        ctypes.c_int,
        [ctypes.c_int, c_u64, c_u64, c_u64, c_u8p, ctypes.c_uint32, c_u8p, c_u8p, c_u64,
         ctypes.c_void_p],
    ),
    # the host build of the generator (also in libingot_pktgen_host.so, no HIP)
    "ingot_pktgen_lengths_host": (
        ctypes.c_int, [ctypes.c_int, c_u64, c_u64, c_u64, c_u8p, ctypes.c_int],
    ),
    "ingot_pktgen_fill_host": (
        ctypes.c_int,
        [ctypes.c_int, c_u64, c_u64, c_u64, c_u8p, ctypes.c_uint32, c_u8p, c_u8p, c_u64,
         ctypes.c_int],
    ),
}

_lib: ctypes.CDLL | None = None


class NativeLibraryMissing(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libingot_gpu.so (once) and bind every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryMissing(
            f"{LIB_PATH} is missing: build it with `python -m ingot_amd.build` "
            "(hipcc --offload-arch=gfx950); there is no fallback path"
        )
    # One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64
    # (soname libamdhip64.so.7) and its libraries name it "libamdhip64.so";
    # this library names the soname.  Loaded after torch, the library binds
    # to torch's copy; loaded first, it brings /opt/rocm's in and torch then
    # loads a second runtime beside it (contexts fail: ENODEV).  So torch
    # first, whenever it is installed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(code: int, what: str) -> None:
    if code != 0:
        msg = load().ingot_gpu_strerror(code).decode()
        raise RuntimeError(f"{what} failed: {msg} ({code})")
