"""The C-ABI boundary, checked without a GPU: the library loads, exports every
symbol include/*.h declares, the Python/ctypes layouts match the C layouts,
and the non-compute entry points behave (no compute calls here)."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

import ingot_amd
from ingot_amd import _lib, abi
from ingot_amd.abi import (CHAIN_LABELS, FIELDS_DTYPE, REC8_DTYPE, REC_DTYPE, Chain, IngotFields,
                           IngotRec, IngotRec8)

ROOT = Path(__file__).resolve().parent.parent


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[a-z_][\w \*]*?\b(ingot_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def lib():
    from ingot_amd.build import build

    build()
    return _lib.load()


def test_every_declared_symbol_is_exported(lib):
    names = declared_functions()
    assert {"ingot_gpu_parse", "ingot_gpu_parse_strided", "ingot_gpu_fields",
            "ingot_pktgen_fill"} <= names
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = names - exported
    assert not missing, missing
    assert set(_lib.SIGNATURES) == names, set(_lib.SIGNATURES) ^ names


def test_layouts_match_c(tmp_path):
    """Compile a probe against include/ingot_gpu.h and compare every offset."""
    structs = {"ingot_rec": IngotRec, "ingot_rec8": IngotRec8, "ingot_v6eh": abi.IngotV6Eh,
               "ingot_fields": IngotFields, "ingot_geneve_opt": abi.IngotGeneveOpt,
               "ingot_tunnel_fields": abi.IngotTunnelFields,
               "ingot_geneve_fields": abi.IngotGeneveFields, "ingot_hdr": abi.IngotHdr}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ingot_gpu.h"',
             "int main(void){"]
    for c, py in structs.items():
        lines.append(f'printf("{c} %zu\\n", sizeof({c}));')
        for f in (f[0] for f in py._fields_):
            lines.append(f'printf("{c}.{f} %zu\\n", offsetof({c}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", str(ROOT / "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True,
                                                       text=True).stdout.splitlines())
    sizes = {"ingot_rec": 16, "ingot_rec8": 8, "ingot_v6eh": 12, "ingot_fields": 256,
             "ingot_geneve_opt": 8, "ingot_tunnel_fields": 128, "ingot_geneve_fields": 384,
             "ingot_hdr": 8}
    for c, py in structs.items():
        assert int(got[c]) == ctypes.sizeof(py) == sizes[c], c
        for f in (f[0] for f in py._fields_):
            assert int(got[f"{c}.{f}"]) == getattr(py, f).offset, (c, f)
    assert REC_DTYPE.itemsize == 16 and FIELDS_DTYPE.itemsize == 256
    assert REC8_DTYPE.itemsize == 8 and abi.GENEVE_FIELDS_DTYPE.itemsize == 384


def test_string_tables(lib):
    assert lib.ingot_gpu_abi_version() == ingot_amd.ABI_VERSION
    assert b"gfx950" in lib.ingot_gpu_build_info()
    # ParseError::as_cstr (ingot-types/src/error.rs:49-60)
    names = [lib.ingot_parse_error_name(i) for i in range(9)]
    assert names == [b"Ok", b"Unwanted", b"NeedsHint", b"TooSmall", b"StraddledHeader",
                     b"NoRemainingChunks", b"CannotAccept", b"Reject", b"IllegalValue"]
    assert lib.ingot_parse_error_name(9) is None
    for chain in Chain:
        n = lib.ingot_chain_layer_count(int(chain))
        labels = tuple(lib.ingot_chain_layer_label(int(chain), i).decode() for i in range(n))
        assert labels == CHAIN_LABELS[chain]
        assert lib.ingot_chain_layer_label(int(chain), n) is None
    assert lib.ingot_chain_layer_count(7) == -1


def test_argument_validation_without_gpu(lib):
    # NULL context / bad chain are rejected before any device work.
    null = ctypes.c_void_p(0)
    assert lib.ingot_gpu_parse(null, None, None, None, 10, 0, None, None) == -1
    assert lib.ingot_gpu_parse_strided(null, None, 64, None, 10, 0, None, None) == -1
    assert lib.ingot_gpu_fields(null, None, None, None, 64, 10, 0, None, None) == -1
    assert lib.ingot_gpu_geneve_fields(null, None, None, None, 64, 10, None, None) == -1
    assert lib.ingot_gpu_parse_compact(null, None, None, None, 10, 0, None, None) == -1
    assert lib.ingot_gpu_parse_strided_compact(null, None, 64, None, 10, 0, None, None) == -1
    assert lib.ingot_pktgen_fill(0, 1, 0, 1, None, 0, None, None, 0, None) == -1
    assert lib.ingot_gpu_parse_header(null, None, None, None, 64, 10, 0, None, 0, None,
                                      None) == -1
    assert lib.ingot_gpu_host_map(null, None, 64, ctypes.byref(ctypes.c_void_p())) == -1
    assert lib.ingot_gpu_strerror(-1) == b"invalid argument"


def test_no_cpu_fallback_when_library_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(_lib.NativeLibraryMissing):
        _lib.load()
