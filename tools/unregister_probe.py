#!/usr/bin/env python3
"""Probe (host-side only): what round 5's ingot_gpu_host_unmap did to memory
it had not registered.  It called hipHostUnregister on any pointer; bench's
zero-copy leg (tools/hostpath.py) passed torch-pinned tensors, which torch
allocates with hipHostMalloc.  This asks the HIP runtime, before and after
such a call, whether it still knows the pointer as host memory
(hipPointerGetAttributes).  No kernel or copy touches the buffer after the
call, and the process ends with os._exit so torch never frees it.

    python tools/unregister_probe.py [--inner]
-> one JSON line (also gpurun_out/unregister_probe.json)

--inner: the call on a pointer 4 KiB inside the pinned allocation (a
sub-range mapping of a pinned ring) instead of its start.  Measured on the
box: ROCclr aborts the process (device.cpp:359 "Memobj map does not have
ptr"), exit status 134 — run it last in a command.
"""
import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


class _PtrAttr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int),
                ("devicePointer", ctypes.c_void_p), ("hostPointer", ctypes.c_void_p),
                ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def main():
    import torch

    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded
    hip.hipPointerGetAttributes.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]

    def attr(p):
        a = _PtrAttr()
        rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
        hip.hipGetLastError()
        return {"rc": rc, "type": a.type if rc == 0 else None}

    torch.cuda.init()
    inner = "--inner" in sys.argv
    t = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
    p = t.data_ptr()
    before = attr(p)
    rc = hip.hipHostUnregister(ctypes.c_void_p(p + (4096 if inner else 0)))
    hip.hipGetLastError()
    after = attr(p)
    res = {("hipHostMalloc_inner" if inner else "hipHostMalloc_start"):
           {"before": before, "hipHostUnregister_rc": rc, "after": after},
           "note": "type 1 = hipMemoryTypeHost; rc 0 = hipSuccess"}
    line = json.dumps(res)
    print(line, flush=True)
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "unregister_probe.json").write_text(line)
    os._exit(0)  # torch never frees the two buffers


if __name__ == "__main__":
    main()
