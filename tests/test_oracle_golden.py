"""Pin the CPU oracle to the reference's own known-answer vectors.

The reference (Rust) cannot be compiled or run in this image, so the parity
oracle is a C restatement; these tests check it against every golden vector
transcribed from ingot's tests and benches (tests/golden/kats.json).
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
from ingot_amd.abi import Chain, ParseError
from tests.kat_check import check


def test_golden_file_has_vectors(kats):
    assert len(kats["chain_kats"]) >= 15
    assert len(kats["header_kats"]) >= 8
    assert kats["bitfield_kats"]


_N_CHAIN_KATS = len(json.loads(
    (Path(__file__).resolve().parent / "golden" / "kats.json").read_text())["chain_kats"])


@pytest.mark.parametrize("idx", range(_N_CHAIN_KATS))
def test_chain_kat(kats, idx):
    kat = kats["chain_kats"][idx]
    if Chain[kat["chain"]] == Chain.GeneveOverV6Tunnel:
        fld = oracle.parse_geneve(bytes.fromhex(kat["frame"]))
        rec = fld["inner"]["rec"]
    else:
        rec, fld = oracle.parse_one(bytes.fromhex(kat["frame"]), Chain[kat["chain"]])
    bad = check(kat, rec, fld)
    assert not bad, f"{kat['name']} ({kat['source']}): {bad}"


def test_read_kats(kats):
    """parse_read (multi-chunk) vectors: StraddledHeader, chunk stepping."""
    assert len(kats["read_kats"]) >= 6
    for kat in kats["read_kats"]:
        chunks = [bytes.fromhex(c) for c in kat["chunks"]]
        chain = Chain[kat["chain"]]
        kind = "geneve" if chain == Chain.GeneveOverV6Tunnel else "fields"
        rec, fld, ch = oracle.parse_read(chunks, chain, fields=kind)
        bad = check(kat, rec, fld, chunk=ch)
        assert not bad, f"{kat['name']} ({kat['source']}): {bad}"


def test_read_single_chunk_equals_parse_slice():
    """One chunk holding the whole frame: parse_read == parse_slice, except
    that a layer ending exactly at the frame end before the last layer now
    pulls a (missing) next chunk (parse.rs:205-218)."""
    from tests.frames import build_frames

    for chain in Chain:
        for f in build_frames(1500, seed=int(chain) + 3, vlan=True, broken=0.3):
            r1, _ = oracle.parse_one(f, chain)
            r2, _, ch = oracle.parse_read([f], chain)
            assert ch == 0
            if r1.tobytes() != r2.tobytes():
                # only when a non-final layer ended the only chunk: the slice
                # step then fails with TooSmall at that layer
                assert int(r1["payload_off"]) == len(f) >= 14, (chain, f.hex())
                assert ParseError(int(r2["status"])) == ParseError.TooSmall, f.hex()
                assert int(r2["err_layer"]) < ingot_amd_layers(chain) - 1


def ingot_amd_layers(chain):
    from ingot_amd.abi import CHAIN_LABELS

    return len(CHAIN_LABELS[chain])


def test_header_kats(kats):
    for kat in kats["header_kats"]:
        st, used, hint = oracle.parse_header(kat["header"], bytes.fromhex(kat["bytes"]))
        e = kat["expect"]
        if e["ok"]:
            assert st == 0, kat["name"]
            assert used == e["used"], kat["name"]
            if "hint" in e:
                assert hint == e["hint"], kat["name"]
        else:
            assert ParseError(st).name == e["error"], kat["name"]


def test_setter_kats(kats):
    """BE setters leave neighbouring bits alone (ingot/src/tests.rs:118-164)."""
    for kat in kats["setter_kats"]:
        orig = bytes.fromhex(kat["bytes"])
        b = orig
        for st in kat["sets"]:
            b = oracle.be_set_bits(b, st["bit"], st["bits"], st["value"])
        for st in kat["sets"]:
            assert oracle.be_bits(b, st["bit"], st["bits"]) == st["value"], st["name"]
        for lo, hi in kat["untouched_bytes"]:
            assert b[lo:hi] == orig[lo:hi], (lo, hi)


def test_modify_kats(kats):
    from ingot_amd.abi import EditOp, Field

    assert len(kats["modify_kats"]) >= 6
    for kat in kats["modify_kats"]:
        edits = [(e[0], Field[e[1]], EditOp[e[2]], e[3], *e[4:]) for e in kat["edits"]]
        out, rec = oracle.parse_modify(bytes.fromhex(kat["frame"]), Chain[kat["chain"]], edits)
        assert out.hex() == kat["after"], kat["name"]


def test_bitfield_kats(kats):
    for kat in kats["bitfield_kats"]:
        data = bytes.fromhex(kat["bytes"])
        for f in kat["fields"]:
            assert oracle.be_bits(data, f["bit"], f["bits"]) == f["value"], f["name"]


def test_v6eh_class_matches_ip_rs():
    # IpProtocol::class, ingot/src/ip.rs:40-54
    frag = {44}
    r6564 = {0, 43, 60, 135, 139, 140, 253, 254}
    for p in range(256):
        want = 1 if p in frag else 2 if p in r6564 else 0
        assert oracle.v6eh_class(p) == want, p
    # ESP/AH/NoNext/ICMPv6/TCP/UDP end the chain (ip.rs:31 "Not considered")
    for p in (50, 51, 59, 58, 6, 17):
        assert oracle.v6eh_class(p) == 0


def test_ecn_quirk():
    # Ecn::from_network maps 3 -> Capable0 (ingot/src/ip.rs:111-119)
    v6 = bytes([0x60, 0x30, 0, 0, 0, 8, 17, 64]) + bytes(32) + bytes(8)
    frame = bytes(12) + b"\x86\xdd" + v6
    rec, fld = oracle.parse_one(frame, Chain.UdpParser)
    assert rec["status"] == 0
    assert fld["v6_ecn_raw"] == 3 and fld["v6_ecn"] == 1


def test_truncation_sweep_every_byte():
    """Every prefix of a valid frame fails at the right layer with TooSmall
    (Accessor::read_from_prefix, ingot-types/src/accessor.rs:30-67)."""
    # eth(14) + v4 ihl 6 (24) + tcp doff 6 (24)
    v4 = bytes([0x46, 0, 0, 0, 0, 0, 0, 0, 64, 6, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 1, 1, 1, 1])
    tcp = bytes([0, 1, 0, 2] + [0] * 8 + [0x60, 0x18] + [0] * 6 + [1, 1, 1, 1])
    frame = bytes(12) + b"\x08\x00" + v4 + tcp
    for cut in range(len(frame) + 1):
        rec, _ = oracle.parse_one(frame[:cut], Chain.GenericUlp)
        if cut < 14:
            assert (rec["status"], rec["err_layer"]) == (ParseError.TooSmall, 0), cut
        elif cut < 14 + 24:
            assert (rec["status"], rec["err_layer"]) == (ParseError.TooSmall, 1), cut
        elif cut < len(frame):
            assert (rec["status"], rec["err_layer"]) == (ParseError.TooSmall, 2), cut
        else:
            assert rec["status"] == 0 and rec["payload_off"] == len(frame)


def test_udp_parser_rejects_tcp_after_parsing_it():
    """`from = "L4<Q>"` converts after the TCP parse (parse.rs:196-200):
    a complete TCP header is Unwanted at l4; a truncated one is TooSmall."""
    v4 = bytes([0x45, 0, 0, 0, 0, 0, 0, 0, 64, 6, 0, 0]) + bytes(8)
    tcp = bytes([0, 1, 0, 2] + [0] * 8 + [0x50, 0x18] + [0] * 6)
    frame = bytes(12) + b"\x08\x00" + v4 + tcp
    rec, _ = oracle.parse_one(frame, Chain.UdpParser)
    assert (rec["status"], rec["err_layer"]) == (ParseError.Unwanted, 2)
    assert rec["l4_kind"] == 1 and rec["payload_off"] == len(frame)
    rec, _ = oracle.parse_one(frame[:-1], Chain.UdpParser)
    assert (rec["status"], rec["err_layer"]) == (ParseError.TooSmall, 2)


def test_vlan_chain():
    inner = bytes([0x45, 0, 0, 0, 0, 0, 0, 0, 64, 17, 0, 0]) + bytes(8) + bytes(8)
    tag = lambda tci, et: bytes([tci >> 8, tci & 0xFF, et >> 8, et & 0xFF])  # noqa: E731
    frame = bytes(12) + b"\x91\x00" + tag(0xA123, 0x8100) + tag(0x0FFF, 0x0800) + inner
    rec, fld = oracle.parse_one(frame, Chain.VlanUlp)
    assert rec["status"] == 0 and rec["n_vlan"] == 2 and rec["l3_off"] == 22
    assert fld["vlan_priority"][0] == 5 and fld["vlan_dei"][0] == 0 and fld["vlan_vid"][0] == 0x123
    assert fld["vlan_vid"][1] == 0xFFF and fld["vlan_ethertype"][1] == 0x0800
    # reference chains do not know VLAN: Unwanted at l3
    rec, _ = oracle.parse_one(frame, Chain.UdpParser)
    assert (rec["status"], rec["err_layer"]) == (ParseError.Unwanted, 1)
    # third tag: Unwanted at l3 of the VLAN chain; truncated tag: TooSmall at vlan
    frame3 = bytes(12) + b"\x81\x00" + tag(1, 0x8100) + tag(2, 0x8100) + inner
    rec, _ = oracle.parse_one(frame3, Chain.VlanUlp)
    assert (rec["status"], rec["err_layer"]) == (ParseError.Unwanted, 2)
    rec, _ = oracle.parse_one(frame[:16], Chain.VlanUlp)
    assert (rec["status"], rec["err_layer"]) == (ParseError.TooSmall, 1)


def test_batch_matches_single_and_threads():
    rng = np.random.default_rng(7)
    frames = [rng.integers(0, 256, size=int(rng.integers(0, 90)), dtype=np.uint8).tobytes()
              for _ in range(300)]
    # make some look like real chains
    for i in range(0, 300, 3):
        f = bytearray(frames[i].ljust(60, b"\0"))
        f[12:14] = b"\x08\x00"
        f[14] = 0x45
        f[23] = 17
        frames[i] = bytes(f)
    offs, o = [], 0
    for f in frames:
        offs.append(o)
        o += len(f)
    arena = np.frombuffer(b"".join(frames) + bytes(16), dtype=np.uint8)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    off = np.array(offs, dtype=np.uint64)
    for chain in Chain:
        r1, f1 = oracle.parse_batch(arena, off, lens, chain, fields=True, nthreads=1)
        r4 = oracle.parse_batch(arena, off, lens, chain, nthreads=4)
        assert r1.tobytes() == r4.tobytes()
        for i, fr in enumerate(frames):
            rr, ff = oracle.parse_one(fr, chain)
            assert rr.tobytes() == r1[i].tobytes()
            assert ff.tobytes() == f1[i].tobytes()


CHOICE_KINDS = {"L3": 16, "L4": 17, "Ulp": 18}
VARIANTS = {"ethernet": 0, "vlan": 1, "ipv4": 2, "ipv6": 3, "tcp": 4, "udp": 5, "icmp": 6}


def test_choice_kats(kats):
    """parse_choice of the L3 / L4 / Ulp choices (ingot-examples/benches/
    choice.rs and the choice semantics), through the batched header oracle."""
    assert len(kats["choice_kats"]) >= 6
    for kat in kats["choice_kats"]:
        data = np.frombuffer(bytes.fromhex(kat["bytes"]) + bytes(8), np.uint8)
        n = len(bytes.fromhex(kat["bytes"]))
        out = oracle.parse_header_batch(data, np.array([0]), np.array([n]),
                                        CHOICE_KINDS[kat["choice"]], hint=kat["hint"])
        st, kind = int(out[0, 0]), int(out[0, 1])
        used = int(out[0, 2]) | int(out[0, 3]) << 8
        hint = int(out[0, 4:8].view(np.uint32)[0])
        e = kat["expect"]
        if e["ok"]:
            assert st == 0, kat["name"]
            assert kind == VARIANTS[e["variant"]], kat["name"]
            assert used == e["used"], kat["name"]
            assert hint == e.get("hint", 0xFFFFFFFF), kat["name"]
        else:
            assert ParseError(st).name == e["error"], kat["name"]
            assert used == 0 and hint == 0xFFFFFFFF, kat["name"]


def test_header_batch_agrees_with_header_kats(kats):
    """The batched header oracle (ingot_gpu_parse_header's checker) returns
    what the per-header oracle pinned by the reference's vectors returns."""
    for kat in kats["header_kats"]:
        b = bytes.fromhex(kat["bytes"])
        out = oracle.parse_header_batch(np.frombuffer(b + bytes(8), np.uint8), np.array([0]),
                                        np.array([len(b)]), oracle.HEADER_KINDS[kat["header"]])
        st, used, hint = oracle.parse_header(kat["header"], b)
        assert int(out[0, 0]) == st, kat["name"]
        if st == 0:
            assert int(out[0, 2]) | int(out[0, 3]) << 8 == used
            assert int(out[0, 4:8].view(np.uint32)[0]) == (0xFFFFFFFF if hint is None else hint)
