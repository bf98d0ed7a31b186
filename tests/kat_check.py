"""Shared checker: does a (record, fields) pair satisfy a golden KAT's `expect`?

Used for both the CPU oracle (test_oracle_golden.py) and the GPU path
(test_gpu_parity.py), so the two are held to the same reference asserts.
"""
from __future__ import annotations

import re

from ingot_amd.abi import CHAIN_LABELS, REC_ACCEPTED, REC_INNER, Chain, L3Kind, L4Kind, ParseError

L3_NAMES = {"none": L3Kind.NONE, "ipv4": L3Kind.IPV4, "ipv6": L3Kind.IPV6}
L4_NAMES = {"none": L4Kind.NONE, "tcp": L4Kind.TCP, "udp": L4Kind.UDP,
            "icmpv4": L4Kind.ICMPV4, "icmpv6": L4Kind.ICMPV6}
EH_KINDS = {"fragment": 1, "rfc6564": 2}


def _field(f, name):
    if name == "v4_options":
        o, n = int(f["v4_options_off"]), int(f["v4_options_len"])
        return ("slice", o, n)
    v = f[name]
    return bytes(v).hex() if getattr(v, "shape", ()) else int(v)


def _outer_field(t, name):
    m = re.fullmatch(r"(\w+)\[(\d+)\]\.(\w+)", name)
    v = t[m.group(1)][int(m.group(2))][m.group(3)] if m else t[name]
    return bytes(v).hex() if getattr(v, "shape", ()) else int(v)


def kat_frame(kat: dict) -> bytes:
    """The frame bytes (parse_read vectors: the chunks concatenated)."""
    if "chunks" in kat:
        return b"".join(bytes.fromhex(c) for c in kat["chunks"])
    return bytes.fromhex(kat["frame"])


def check(kat: dict, rec, fld, chunk: int | None = None) -> list[str]:
    """Return a list of mismatches (empty = pass).  For the tunnel chain `fld`
    may be an ingot_geneve_fields (inner + outer blocks); for parse_read
    vectors `chunk` is the index of the chunk holding the remainder."""
    frame = kat_frame(kat)
    outer = None
    if fld is not None and fld.dtype.names and "outer" in fld.dtype.names:
        outer, fld = fld["outer"], fld["inner"]
    chain = Chain[kat["chain"]]
    e = kat["expect"]
    bad = []
    status = int(rec["status"])
    if e["ok"]:
        if status != 0:
            lbl = CHAIN_LABELS[chain][int(rec["err_layer"])]
            bad.append(f"expected Ok, got {ParseError(status).name} at {lbl}")
            return bad
        if "remainder" in e and len(frame) - int(rec["payload_off"]) != e["remainder"]:
            bad.append(f"remainder {len(frame) - int(rec['payload_off'])} != {e['remainder']}")
        if "remainder_hex" in e and frame[int(rec["payload_off"]):].hex() != e["remainder_hex"]:
            bad.append("remainder bytes differ")
        if e.get("accepted") and not int(rec["flags"]) & REC_ACCEPTED:
            bad.append("expected the control to accept")
    else:
        if status == 0:
            bad.append(f"expected {e['error']} at {e['label']}, got Ok")
            return bad
        got = (ParseError(status).name, CHAIN_LABELS[chain][int(rec["err_layer"])])
        if got != (e["error"], e["label"]):
            bad.append(f"expected {e['error']} at {e['label']}, got {got}")
    if "chunk" in e:
        lens = [len(bytes.fromhex(c)) for c in kat["chunks"]]
        if chunk != e["chunk"]:
            bad.append(f"chunk {chunk} != {e['chunk']}")
        else:
            last = sum(lens[:chunk + 1]) - int(rec["payload_off"])
            if "last_chunk_len" in e and last != e["last_chunk_len"]:
                bad.append(f"last_chunk_len {last} != {e['last_chunk_len']}")
            if "data_left" in e and len(lens) - chunk - 1 != e["data_left"]:
                bad.append(f"data_left {len(lens) - chunk - 1} != {e['data_left']}")
    if "inner" in e and bool(int(rec["flags"]) & REC_INNER) != e["inner"]:
        bad.append(f"inner flag {int(rec['flags'])} != {e['inner']}")
    if outer is not None:
        for name, want in e.get("outer_fields", {}).items():
            got = _outer_field(outer, name)
            if got != want:
                bad.append(f"outer {name}: {got} != {want}")
    elif e.get("outer_fields") and fld is not None:
        bad.append("outer fields expected but not provided")
    if "l3" in e and int(rec["l3_kind"]) != L3_NAMES[e["l3"]]:
        bad.append(f"l3_kind {int(rec['l3_kind'])} != {e['l3']}")
    if "l4" in e and int(rec["l4_kind"]) != L4_NAMES[e["l4"]]:
        bad.append(f"l4_kind {int(rec['l4_kind'])} != {e['l4']}")
    for k in ("l4_proto", "n_v6ext"):
        if k in e and int(rec[k]) != e[k]:
            bad.append(f"{k} {int(rec[k])} != {e[k]}")
    if fld is not None:
        if "v6_ext_len" in e and int(fld["v6_ext_len"]) != e["v6_ext_len"]:
            bad.append(f"v6_ext_len {int(fld['v6_ext_len'])} != {e['v6_ext_len']}")
        for i, eh in enumerate(e.get("ehs", [])):
            g = fld["v6_eh"][i]
            if int(g["kind"]) != EH_KINDS[eh["kind"]]:
                bad.append(f"eh[{i}].kind {int(g['kind'])} != {eh['kind']}")
            for k in ("next_header", "ext_len"):
                if k in eh and int(g[k]) != eh[k]:
                    bad.append(f"eh[{i}].{k} {int(g[k])} != {eh[k]}")
        for name, want in e.get("fields", {}).items():
            if name == "note":
                continue
            got = _field(fld, name)
            if isinstance(got, tuple):
                got = frame[got[1]:got[1] + got[2]].hex()
            if got != want:
                bad.append(f"{name}: {got} != {want}")
    return bad
