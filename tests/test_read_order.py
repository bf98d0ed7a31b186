"""parse_read layer order audit (VERDICT r04 "next" item 1).

Every golden frame (tests/golden/kats.json, transcribed from the reference's
tests and benches) is cut at each of its layer boundaries into [head],
[head | tail] and [head | empty | tail], and at every byte into two chunks.
The oracle's parse_read must give what tests/read_model.py derives from the
generated driver (ingot-macros/src/parse.rs:357-416, 511-537): status,
failing layer, accepted flag, the remainder's chunk index and offset.
"""
import numpy as np
import pytest

import oracle
from ingot_amd.abi import REC_ACCEPTED, Chain, ParseError
from tests import read_model
from tests.kat_check import kat_frame

TUN = Chain.GeneveOverV6Tunnel


def golden_frames(kats):
    frames = {c: [] for c in Chain}
    for kat in kats["chain_kats"] + kats["read_kats"]:
        f = kat_frame(kat)
        for c in Chain:  # every frame through every chain: more orders exercised
            frames[c].append(f)
    return frames


def audit_cases(kats, every_byte=True):
    cases = []
    for chain, frames in golden_frames(kats).items():
        for f in frames:
            for chunks in read_model.cuts_at_boundaries(f, chain):
                cases.append((chain, chunks))
            if every_byte:
                for b in range(len(f) + 1):
                    cases.append((chain, [f[:b], f[b:]]))
    return cases


def expected(cases):
    return [read_model.parse_read(chunks, chain) for chain, chunks in cases]


def compare(cases, want, rec, chunk):
    bad = []
    for i, ((chain, chunks), w) in enumerate(zip(cases, want)):
        r = rec[i]
        got = (int(r["status"]), int(r["err_layer"]) if int(r["status"]) else 0xFF,
               int(chunk[i]), bool(int(r["flags"]) & REC_ACCEPTED))
        exp = (int(w.status), w.err_layer if w.status else 0xFF, w.chunk, w.accepted)
        if got != exp or (w.status == 0 and int(r["payload_off"]) != w.payload_off):
            bad.append((chain.name, [len(c) for c in chunks], got, exp))
    return bad


def run_oracle(cases):
    out = {}
    for chain in Chain:
        idx = [i for i, (c, _) in enumerate(cases) if c == chain]
        segs = oracle.segments([cases[i][1] for i in idx])
        rec, _, chunk = oracle.parse_read_batch(*segs, chain)
        for j, i in enumerate(idx):
            out[i] = (rec[j], chunk[j])
    rec = np.array([out[i][0] for i in range(len(cases))])
    chunk = np.array([out[i][1] for i in range(len(cases))])
    return rec, chunk


def test_model_reproduces_read_kats(kats):
    """The driver model itself against the reference's parse_read vectors."""
    for kat in kats["read_kats"]:
        chunks = [bytes.fromhex(c) for c in kat["chunks"]]
        w = read_model.parse_read(chunks, Chain[kat["chain"]])
        e = kat["expect"]
        if e["ok"]:
            assert w.status == 0, kat["name"]
            if "chunk" in e:
                assert w.chunk == e["chunk"], kat["name"]
        else:
            from ingot_amd.abi import CHAIN_LABELS

            got = (ParseError(w.status).name, CHAIN_LABELS[Chain[kat["chain"]]][w.err_layer])
            assert got == (e["error"], e["label"]), kat["name"]


def test_oracle_layer_order_at_every_boundary(kats):
    cases = audit_cases(kats)
    want = expected(cases)
    rec, chunk = run_oracle(cases)
    bad = compare(cases, want, rec, chunk)
    assert not bad, (len(bad), bad[:8])
    # the audit reaches the cases it is for
    st = {(c, w.status, w.err_layer) for (c, _), w in zip(cases, want)}
    assert (TUN, ParseError.TooSmall, 1) in st and (TUN, ParseError.Unwanted, 1) in st
    assert (TUN, ParseError.TooSmall, 2) in st and (TUN, ParseError.Unwanted, 2) in st
    assert any(w.status == ParseError.StraddledHeader for w in want)
    assert any(w.accepted and w.status == 0 for w in want)


@pytest.mark.parametrize("chain", list(Chain))
def test_oracle_layer_order_random_chunking(chain):
    """Synthetic frames (every chain, broken ones too) cut into 1-5 chunks at
    random, empty chunks included: oracle == model."""
    from tests.frames import build_frames

    rng = np.random.default_rng(int(chain) + 40)
    frames = build_frames(400, seed=int(chain) + 17, vlan=True, broken=0.2)
    cases = []
    for f in frames:
        for _ in range(3):
            cuts = sorted(int(x) for x in rng.integers(0, len(f) + 1, int(rng.integers(0, 5))))
            b = [0] + cuts + [len(f)]
            cases.append((chain, [f[x:y] for x, y in zip(b, b[1:])]))
    want = expected(cases)
    rec, chunk = run_oracle(cases)
    bad = compare(cases, want, rec, chunk)
    assert not bad, (len(bad), bad[:8])
