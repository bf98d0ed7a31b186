"""TEST INFRASTRUCTURE — a second, table-driven restatement of the chain
driver that ingot-macros generates for `parse_read`, used to audit the
oracle's (and through it the kernel's) per-layer order on chunked packets.

The oracle (oracle/ingot_oracle.c) hand-writes each chain as straight-line
C.  This module instead states each chain as the field list its
`#[derive(Parse)]` declares (ingot-examples/src/packets.rs:18-60) and runs
the fragments exactly as ingot-macros/src/parse.rs emits them:

  * reader start: `data.next_chunk()`, failing at the first label
    (parse.rs:515-516);
  * `can_accept = true` once the trailing `Option<>` sled is reached
    (parse.rs:144-156, 221-227);
  * per layer (parse.rs:357-416): parse (layer 0) / parse_choice (later
    layers) -> control fn (parse.rs:229-254) -> slice step for every
    non-final layer (parse.rs:208-219) -> `from=` conversion
    (parse.rs:196-206);
  * a parse error goes through `convert_read_parse` (error.rs:65-72):
    TooSmall becomes StraddledHeader iff the reader holds another chunk;
  * an accepted `Option<>` layer is None and hands its slice on unchanged
    (parse.rs:296-333).

Header bodies come from the oracle's header-level entry
(`oracle.parse_header`), which the reference's header KATs pin separately
(tests/test_oracle_golden.py::test_header_kats); choices dispatch on the
hint as ingot-examples/src/choices.rs:17-38 declares (choice.rs:231-246).
"""
from __future__ import annotations

from dataclasses import dataclass

import oracle
from ingot_amd.abi import Chain, ParseError

ET_IPV4, ET_ARP, ET_IPV6, ET_VLAN, ET_QINQ = 0x0800, 0x0806, 0x86DD, 0x8100, 0x9100

# choices.rs:17-38: hint -> header variant
CHOICES = {
    "L3": {ET_IPV4: "ipv4", ET_IPV6: "ipv6"},
    "L4": {6: "tcp", 17: "udp"},
    "Ulp": {6: "tcp", 17: "udp", 1: "icmp", 58: "icmp"},
}


@dataclass(frozen=True)
class Layer:
    label: str
    header: str | None = None   # plain header (ValidX::parse / parse_choice ignoring the hint)
    choice: str | None = None   # #[choice] enum
    conv: str | None = None     # #[ingot(from = ...)]: the one variant TryFrom keeps
    control: bool = False       # #[ingot(control = exit_on_arp)] (packets.rs:45-51)
    optional: bool = False      # Option<...>
    repeat_vlan: bool = False   # build-defined VLAN layer (no reference chain): 0-2 tags


CHAINS = {
    # packets.rs:18-24
    Chain.UdpParser: [Layer("eth", header="ethernet"), Layer("l3", choice="L3"),
                      Layer("l4", choice="L4", conv="udp")],
    # packets.rs:54-60
    Chain.GenericUlp: [Layer("inner_eth", header="ethernet", control=True),
                       Layer("inner_l3", choice="L3", optional=True),
                       Layer("inner_ulp", choice="Ulp", optional=True)],
    # build-defined (SURVEY §7 hard part 5): eth, up to two VlanBody tags, L3, Ulp
    Chain.VlanUlp: [Layer("eth", header="ethernet"), Layer("vlan", header="vlan", repeat_vlan=True),
                    Layer("l3", choice="L3"), Layer("l4", choice="Ulp")],
    # packets.rs:27-40
    Chain.GeneveOverV6Tunnel: [
        Layer("outer_eth", header="ethernet"), Layer("outer_v6", choice="L3", conv="ipv6"),
        Layer("outer_udp", choice="L4", conv="udp"), Layer("outer_encap", header="geneve"),
        Layer("inner_eth", header="ethernet", control=True),
        Layer("inner_l3", choice="L3", optional=True),
        Layer("inner_ulp", choice="Ulp", optional=True)],
}


@dataclass
class Result:
    status: int          # 0 Ok, else ParseError
    err_layer: int       # 0xff on Ok
    chunk: int           # index of the chunk the walk ended in
    payload_off: int     # Ok: remainder start in the chunks' concatenation
    accepted: bool = False
    ends: tuple = ()     # Ok or not: concatenation offset where each parsed layer ended


def _parse(layer: Layer, data: bytes, hint):
    """-> (status, used, hint_out, variant)."""
    if layer.choice is not None:
        if hint is None:
            return ParseError.NeedsHint, 0, None, None
        variant = CHOICES[layer.choice].get(hint)
        if variant is None:
            return ParseError.Unwanted, 0, None, None
    else:
        variant = layer.header
    st, used, h = oracle.parse_header(variant, data)
    return st, used, h, variant


def parse_read(chunks: list[bytes], chain: Chain) -> Result:
    layers = CHAINS[chain]
    n = len(chunks)
    starts = [sum(len(c) for c in chunks[:k]) for k in range(n)]
    any_opt = any(x.optional for x in layers)
    any_ctl = any(x.control for x in layers)
    accept_from = len(layers)
    for i in range(len(layers) - 1, -1, -1):  # parse.rs:145-153
        if layers[i].optional:
            accept_from = i - 1
        else:
            break
    if n == 0:  # parse.rs:515-516
        return Result(ParseError.TooSmall, 0, 0, 0)
    k, slice_ = 0, chunks[0]
    can_accept = accepted = False
    hint = None
    ends: list[int] = []

    def here(rem):  # concatenation offset of `rem`, a suffix of chunk k
        return starts[k] + len(chunks[k]) - len(rem)

    def err(code, i):
        return Result(int(code), i, k, 0, accepted, tuple(ends))

    last = len(layers) - 1
    for i, layer in enumerate(layers):
        if any_opt and any_ctl and i == accept_from:
            can_accept = True
        reps = 1
        if layer.repeat_vlan:
            reps = 0
            while reps < 2 and hint in (ET_VLAN, ET_QINQ):
                st, used, h, _ = _parse(layer, slice_, hint)
                if st != 0:
                    return err(ParseError.StraddledHeader if st == ParseError.TooSmall
                               and k + 1 < n else st, i)
                slice_, hint = slice_[used:], h
                ends.append(here(slice_))
                reps += 1
                if len(slice_) == 0:  # slice step after each tag
                    if k + 1 >= n:
                        return err(ParseError.TooSmall, i)
                    k += 1
                    slice_ = chunks[k]
            continue
        if layer.optional and accepted:
            variant, remainder = None, slice_
            hint = None
        else:
            st, used, h, variant = _parse(layer, slice_, hint)
            if st != 0:
                if st == ParseError.TooSmall and k + 1 < n:  # error.rs:65-72
                    st = ParseError.StraddledHeader
                return err(st, i)
            remainder, hint = slice_[used:], h
            ends.append(here(remainder))
        if layer.control and variant is not None and hint == ET_ARP:  # exit_on_arp
            if not can_accept:
                return err(ParseError.CannotAccept, i)
            accepted = True
        if i != last:  # slice step (parse.rs:208-219)
            if len(remainder) == 0:
                if k + 1 >= n:
                    return err(ParseError.TooSmall, i)
                k += 1
                slice_ = chunks[k]
            else:
                slice_ = remainder
        else:
            slice_ = remainder
        if layer.conv is not None and variant is not None and variant != layer.conv:
            return err(ParseError.Unwanted, i)  # TryFrom, choice.rs:153-187
    return Result(0, 0xFF, k, here(slice_), accepted, tuple(ends))


def layer_ends(frame: bytes, chain: Chain) -> list[int]:
    """Offsets where each layer the single-chunk walk parsed ends (the
    layer boundaries of `frame`), 0 and len(frame) excluded."""
    r = parse_read([frame], chain)
    return sorted({e for e in r.ends if 0 < e < len(frame)})


def cuts_at_boundaries(frame: bytes, chain: Chain) -> list[list[bytes]]:
    """[frame], and for every layer boundary b: [head], [head | tail] and
    [head | empty | tail] (the audit of VERDICT r04 "next" item 1)."""
    out = [[frame]]
    for b in layer_ends(frame, chain):
        head, tail = frame[:b], frame[b:]
        out += [[head], [head, tail], [head, b"", tail]]
    return out
