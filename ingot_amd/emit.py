"""Owned headers -> wire bytes on the host: ingot's `Emit::emit_raw` for owned
`Repr` structs (the generated owned emit blocks, ingot-macros/src/packet/
mod.rs:2097-2255: zero the bitfields, then every field through its setter,
big-endian, declaration order), one function per header of the parse path.

This is the per-flow half of a batched emit: a caller serialises its header
stack once here (or with ingot's own `emit_vec()` on the Rust side) and hands
the bytes to `Context.emit_packets` / `Context.emit_header_blocks`, which put
them in front of every packet on the device with the per-packet setters
applied.  Field values are what the owned structs hold, after
`NetworkRepr::to_network` (Ecn: NotCapable 0, Capable0 1, Capable1 2,
CongestionExperienced 3, ip.rs:95-110; flags: their bits).  Nothing is
derived: like ingot's emit, lengths and `opt_len` are written as given.

Layouts: ethernet.rs:46-65, ip.rs:63-93 / 159-211, tcp.rs:9-30,
udp.rs:8-15, icmp.rs:42-50, geneve.rs:16-104.
"""
from __future__ import annotations

from typing import Iterable


def _bits(n_bytes: int, fields: Iterable[tuple[int, int, int]]) -> bytearray:
    """A zeroed header with (first bit MSB-first, width, value) fields set."""
    b = bytearray(n_bytes)
    for bit, width, value in fields:
        value &= (1 << width) - 1
        for k in range(width):
            if (value >> (width - 1 - k)) & 1:
                pos = bit + k
                b[pos // 8] |= 0x80 >> (pos % 8)
    return b


def _addr(a, n: int, what: str) -> bytes:
    a = bytes(a)
    if len(a) != n:
        raise ValueError(f"{what} must be {n} bytes")
    return a


def ethernet(destination, source, ethertype: int) -> bytes:
    """Ethernet (ethernet.rs:46-55): 14 B."""
    return (_addr(destination, 6, "destination") + _addr(source, 6, "source")
            + bytes(_bits(2, [(0, 16, ethertype)])))


def vlan(vid: int, ethertype: int, priority: int = 0, dei: int = 0) -> bytes:
    """VlanBody (ethernet.rs:57-65): priority u3, dei u1, vid u12be, ethertype."""
    return bytes(_bits(4, [(0, 3, priority), (3, 1, dei), (4, 12, vid), (16, 16, ethertype)]))


def ipv4(source, destination, protocol: int, *, total_len: int = 0, hop_limit: int = 64,
         version: int = 4, ihl: int | None = None, dscp: int = 0, ecn: int = 0,
         identification: int = 0, flags: int = 0, fragment_offset: int = 0, checksum: int = 0,
         options: bytes = b"") -> bytes:
    """Ipv4 (ip.rs:63-93): 20 B + options; ihl defaults to 5 + options/4."""
    if len(options) % 4:
        raise ValueError("IPv4 options are whole 32-bit words")
    ihl = 5 + len(options) // 4 if ihl is None else ihl
    h = _bits(20, [(0, 4, version), (4, 4, ihl), (8, 6, dscp), (14, 2, ecn),
                   (16, 16, total_len), (32, 16, identification), (48, 3, flags),
                   (51, 13, fragment_offset), (64, 8, hop_limit), (72, 8, protocol),
                   (80, 16, checksum)])
    h[12:16] = _addr(source, 4, "source")
    h[16:20] = _addr(destination, 4, "destination")
    return bytes(h) + bytes(options)


def ipv6(source, destination, next_header: int, *, payload_len: int = 0, hop_limit: int = 64,
         version: int = 6, dscp: int = 0, ecn: int = 0, flow_label: int = 0,
         v6ext: bytes = b"") -> bytes:
    """Ipv6 (ip.rs:159-182): 40 B + the extension-header chain's bytes."""
    h = _bits(40, [(0, 4, version), (4, 6, dscp), (10, 2, ecn), (12, 20, flow_label),
                   (32, 16, payload_len), (48, 8, next_header), (56, 8, hop_limit)])
    h[8:24] = _addr(source, 16, "source")
    h[24:40] = _addr(destination, 16, "destination")
    return bytes(h) + bytes(v6ext)


def ipv6_ext_6564(next_header: int, data: bytes, ext_len: int | None = None) -> bytes:
    """IpV6Ext6564 (ip.rs:202-211): next_header, ext_len, 6 + 8 * ext_len data bytes."""
    ext_len = (len(data) - 6) // 8 if ext_len is None else ext_len
    if len(data) != 6 + 8 * ext_len:
        raise ValueError("data must be 6 + 8 * ext_len bytes")
    return bytes([next_header & 0xFF, ext_len & 0xFF]) + bytes(data)


def ipv6_ext_fragment(next_header: int, ident: int, fragment_offset: int = 0,
                      more_frags: int = 0, reserved: int = 0, res: int = 0) -> bytes:
    """IpV6ExtFragment (ip.rs:190-200): 8 B."""
    return bytes(_bits(8, [(0, 8, next_header), (8, 8, reserved), (16, 13, fragment_offset),
                           (29, 2, res), (31, 1, more_frags), (32, 32, ident)]))


def udp(source: int, destination: int, length: int = 0, checksum: int = 0) -> bytes:
    """Udp (udp.rs:8-15): 8 B."""
    return bytes(_bits(8, [(0, 16, source), (16, 16, destination), (32, 16, length),
                           (48, 16, checksum)]))


def tcp(source: int, destination: int, *, sequence: int = 0, acknowledgement: int = 0,
        data_offset: int | None = None, reserved: int = 0, flags: int = 0,
        window_size: int = 0, checksum: int = 0, urgent_ptr: int = 0,
        options: bytes = b"") -> bytes:
    """Tcp (tcp.rs:9-30): 20 B + options; data_offset defaults to 5 + options/4."""
    if len(options) % 4:
        raise ValueError("TCP options are whole 32-bit words")
    data_offset = 5 + len(options) // 4 if data_offset is None else data_offset
    return bytes(_bits(20, [(0, 16, source), (16, 16, destination), (32, 32, sequence),
                            (64, 32, acknowledgement), (96, 4, data_offset), (100, 4, reserved),
                            (104, 8, flags), (112, 16, window_size), (128, 16, checksum),
                            (144, 16, urgent_ptr)])) + bytes(options)


def icmp(ty: int, code: int, checksum: int = 0, rest_of_hdr: bytes = bytes(4)) -> bytes:
    """IcmpV4 / IcmpV6 (icmp.rs:42-50): 8 B."""
    return bytes([ty & 0xFF, code & 0xFF]) + bytes(_bits(2, [(0, 16, checksum)])) + \
        _addr(rest_of_hdr, 4, "rest_of_hdr")


def geneve_opt(opt_class: int, option_type: int, data: bytes = b"", reserved: int = 0,
               length: int | None = None) -> bytes:
    """GeneveOpt (geneve.rs:80-102): class u16be, option_type, reserved u3,
    length u5 (4-byte words), data."""
    if len(data) % 4:
        raise ValueError("Geneve option data is whole 32-bit words")
    length = len(data) // 4 if length is None else length
    return bytes(_bits(4, [(0, 16, opt_class), (16, 8, option_type), (24, 3, reserved),
                           (27, 5, length)])) + bytes(data)


def geneve(vni: int, *, protocol_type: int = 0x6558, flags: int = 0, version: int = 0,
           reserved: int = 0, options: bytes = b"", opt_len: int | None = None) -> bytes:
    """Geneve (geneve.rs:16-44): version u2, opt_len u6, flags, protocol_type,
    vni [u8; 3], reserved, options (opt_len defaults to len(options) / 4)."""
    if len(options) % 4:
        raise ValueError("Geneve options are whole 32-bit words")
    opt_len = len(options) // 4 if opt_len is None else opt_len
    return bytes(_bits(8, [(0, 2, version), (2, 6, opt_len), (8, 8, flags),
                           (16, 16, protocol_type), (32, 24, vni), (56, 8, reserved)])) + \
        bytes(options)
