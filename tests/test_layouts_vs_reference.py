"""The kernel-side field metadata (ingot_amd/csrc/layouts.h) derived
mechanically from the reference's own `#[derive(Ingot)]` declarations.

ingot's macro lays out a header's fields in declaration order, big-endian,
each field `width` bits wide: `uN`/`uNbe` (N bits), `[u8; N]` (8N), `is = "T"`
overrides the declared type, zerocopy types have their wire size (IpProtocol
and the ICMP/Geneve type bytes 8, Ipv4Addr 32, Ipv6Addr 128, MacAddr6 48); the
fixed part ends at the first variable field (`Vec<u8>` / `var_len`,
`Repeated`/`subparse`) (ingot-macros/src/packet/mod.rs:547-821,
bitfield.rs:25-38).  This test reads the struct declarations from the
reference checkout when it is present (CPU only; skipped elsewhere), computes
every field's (first bit, width) and the fixed length, and compares them with
layouts.h — so the restated metadata is pinned to the macro input itself, not
only to the golden vectors."""
import re
from pathlib import Path

import pytest

REF = Path("/root/reference/ingot/src")
LAYOUTS = Path(__file__).resolve().parent.parent / "ingot_amd" / "csrc" / "layouts.h"

ZEROCOPY_BITS = {"IpProtocol": 8, "Ipv4Addr": 32, "Ipv6Addr": 128, "IcmpV4Type": 8,
                 "IcmpV6Type": 8, "GeneveOptionType": 8, "MacAddr6": 48}

# (reference file, struct) -> (layouts.h namespace, field renames)
HEADERS = {
    ("ethernet.rs", "Ethernet"): ("eth", {}),
    ("ethernet.rs", "VlanBody"): ("vlan", {}),
    ("ip.rs", "Ipv4"): ("ipv4", {}),
    ("ip.rs", "Ipv6"): ("ipv6", {}),
    ("ip.rs", "IpV6ExtFragment"): ("v6frag", {}),
    ("ip.rs", "IpV6Ext6564"): ("v6ext6564", {}),
    ("tcp.rs", "Tcp"): ("tcp", {}),
    ("udp.rs", "Udp"): ("udp", {}),
    ("icmp.rs", "IcmpV4"): ("icmp", {}),
    ("icmp.rs", "IcmpV6"): ("icmp", {}),
    ("geneve.rs", "Geneve"): ("geneve", {}),
    ("geneve.rs", "GeneveOpt"): ("geneve_opt", {"class": "opt_class"}),
}


def _type_bits(t: str):
    t = t.strip()
    m = re.fullmatch(r"u(\d+)(be|le|he)?", t)
    if m:
        return int(m.group(1))
    m = re.fullmatch(r"\[u8;\s*(\d+)\]", t)
    if m:
        return 8 * int(m.group(1))
    return ZEROCOPY_BITS.get(t)


def reference_layout(path: Path, struct: str):
    """-> ({field: (bit, width)}, fixed_bits) from the struct declaration."""
    src = path.read_text()
    m = re.search(r"pub struct " + struct + r"\s*\{(.*?)\n\}", src, re.S)
    assert m, struct
    body = re.sub(r"//[^\n]*", "", m.group(1))  # comments (incl. doc comments)
    fields, bit = {}, 0
    attrs = []
    for line in body.splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith("#["):
            attrs.append(line)
            continue
        fm = re.match(r"pub (\w+):\s*(.+?),?$", line)
        if not fm:
            continue
        name, ty = fm.group(1), fm.group(2).rstrip(",")
        a = " ".join(attrs)
        attrs = []
        if "var_len" in a or "subparse" in a or ty.startswith(("Vec<", "Repeated<")):
            break  # the fixed part ends at the first variable field
        im = re.search(r'is\s*=\s*"([^"]+)"', a)
        w = _type_bits(im.group(1) if im else ty)
        assert w is not None, (struct, name, ty)
        fields[name] = (bit, w)
        bit += w
    return fields, bit


def kernel_layouts():
    """-> {namespace: ({field: (bit, width)}, LEN or FIXED bytes)} from layouts.h."""
    src = LAYOUTS.read_text()
    out = {}
    for m in re.finditer(r"namespace (?!ingot_gpu|layout\b)(\w+) \{(.*?)\}  // namespace \1",
                         src, re.S):
        ns, body = m.group(1), m.group(2)
        ln = re.search(r"constexpr uint32_t (?:LEN|FIXED) = (\d+);", body)
        fields = {f: (int(b), int(w)) for f, b, w in re.findall(r"(\w+)\{(\d+), (\d+)\}", body)}
        out[ns] = (fields, int(ln.group(1)) if ln else None)
    return out


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present")
@pytest.mark.parametrize("key", list(HEADERS), ids=lambda k: k[1])
def test_layout_matches_reference_declaration(key):
    fname, struct = key
    ns, renames = HEADERS[key]
    ref_fields, fixed_bits = reference_layout(REF / fname, struct)
    k_fields, k_len = kernel_layouts()[ns]
    assert fixed_bits % 8 == 0
    assert k_len == fixed_bits // 8, (struct, k_len, fixed_bits // 8)
    for name, (bit, width) in ref_fields.items():
        kname = renames.get(name, name)
        if kname in k_fields:
            assert k_fields[kname] == (bit, width), (struct, name, k_fields[kname], (bit, width))
    # every kernel field is a reference field (none invented)
    names = {renames.get(n, n) for n in ref_fields}
    assert set(k_fields) <= names, set(k_fields) - names


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present")
def test_ipv6_address_offsets_match():
    f, _ = reference_layout(REF / "ip.rs", "Ipv6")
    src = LAYOUTS.read_text()
    assert f"SOURCE_BYTE = {f['source'][0] // 8}" in src
    assert f"DESTINATION_BYTE = {f['destination'][0] // 8}" in src


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present")
def test_setter_geometry_matches_reference_declaration():
    """api.cpp's kFieldGeo (the setters' BE geometry, one row per enum
    ingot_field) against the same reference declarations."""
    root = LAYOUTS.parent.parent.parent
    header = (root / "include" / "ingot_gpu.h").read_text()
    enum = re.search(r"enum ingot_field \{(.*?)\};", header, re.S).group(1)
    names = [n for n in re.findall(r"INGOT_F_(\w+)", enum) if n != "COUNT"]
    api = (root / "ingot_amd" / "csrc" / "api.cpp").read_text()
    table = re.search(r"kFieldGeo\[INGOT_F_COUNT\] = \{(.*?)\n\};", api, re.S).group(1)
    rows = re.findall(r"\{ingot_gpu::HK_(\w+), (\d+), (\d+)\}", table)
    assert len(rows) == len(names)
    structs = {"ETH": ("ethernet.rs", "Ethernet"), "VLAN": ("ethernet.rs", "VlanBody"),
               "V4": ("ip.rs", "Ipv4"), "V6": ("ip.rs", "Ipv6"), "TCP": ("tcp.rs", "Tcp"),
               "UDP": ("udp.rs", "Udp"), "ICMP": ("icmp.rs", "IcmpV4"),
               "GENEVE": ("geneve.rs", "Geneve")}
    kinds = {"ETH": "ETH", "VLAN": "VLAN", "V4": "V4", "V6": "V6", "TCP": "TCP", "UDP": "UDP",
             "ICMP": "ICMP", "GENEVE": "GENEVE"}
    for name, (kind, bit, width) in zip(names, rows):
        hdr, field = name.split("_", 1)
        assert kinds[hdr] == kind, name
        ref, _ = reference_layout(REF / structs[hdr][0], structs[hdr][1])
        assert ref[field.lower()] == (int(bit), int(width)), (name, ref[field.lower()], bit, width)


def _consts(src: str, ty: str):
    block = re.search(r"impl " + ty + r" \{(.*?)\n\}", src, re.S).group(1)
    return {k: int(v, 0) for k, v in re.findall(r"pub const (\w+): Self = Self\((\w+)\);", block)}


@pytest.mark.skipif(not REF.exists(), reason="reference checkout not present")
def test_protocol_constants_and_eh_classes_match_reference():
    """Ethertype / IpProtocol constants (ethernet.rs:12-20, ip.rs:20-38) and
    IpProtocol::class (ip.rs:40-54) against layouts.h, the kernel's eh_class
    and the oracle's."""
    import oracle

    et = _consts((REF / "ethernet.rs").read_text(), "Ethertype")
    ip = (REF / "ip.rs").read_text()
    pp = _consts(ip, "IpProtocol")
    lay = LAYOUTS.read_text()
    for ours, theirs in (("ET_IPV4", "IPV4"), ("ET_ARP", "ARP"), ("ET_VLAN", "VLAN"),
                         ("ET_IPV6", "IPV6"), ("ET_QINQ", "QINQ")):
        assert re.search(rf"{ours} = 0x{et[theirs]:04x}\b", lay), ours
    for ours, theirs in (("IPP_ICMP", "ICMP"), ("IPP_TCP", "TCP"), ("IPP_UDP", "UDP"),
                         ("IPP_ICMP_V6", "ICMP_V6")):
        assert re.search(rf"{ours} = {pp[theirs]}\b", lay), ours
    cls = re.search(r"pub fn class\(self\).*?match self \{(.*?)\n\s*_ => None", ip, re.S).group(1)
    frag = {pp[n] for n in re.findall(r"Self::(\w+) => Some\(ExtHdrClass::FragmentHeader\)", cls)}
    r6564_src = cls.split("FragmentHeader),", 1)[1]
    r6564 = {pp[n] for n in re.findall(r"Self::(\w+)", r6564_src)}
    assert frag == {44} and 0 in r6564 and len(r6564) == 8
    # the chain walk (walk.h) and the single-header parsers (header.hip)
    for src in ("walk.h", "header.hip"):
        kernel = (LAYOUTS.parent / src).read_text()
        body = re.search(r"uint32_t eh_class\(uint32_t h\) \{(.*?)\n\}", kernel, re.S).group(1)
        k_frag = {int(x) for x in re.findall(r"h == (\d+)u\) return EH_FRAGMENT", body)}
        k_6564 = {int(x) for x in re.findall(r"h == (\d+)u", body)} - k_frag
        assert k_frag == frag and k_6564 == r6564, src
    for p in range(256):
        want = 1 if p in frag else 2 if p in r6564 else 0
        assert oracle.v6eh_class(p) == want, p


PACKETS = Path("/root/reference/ingot-examples/src/packets.rs")
MACRO = Path("/root/reference/ingot-macros/src/parse.rs")


@pytest.mark.skipif(not PACKETS.exists(), reason="reference checkout not present")
def test_chain_labels_are_the_reference_crstr_labels():
    """ingot_chain_layer_label(chain, i) is the label the generated parser
    attaches to a PacketParseError at layer i: the field name of the
    `#[derive(Parse)]` struct, as `CRStr::new_unchecked("<field>\\0")`
    (ingot-macros/src/parse.rs:36-50; ingot-examples/src/packets.rs:18-60).
    A Rust binding keeps a static CRStr table equal to these strings
    (INTEGRATION.md §2), indexed by the record's err_layer."""
    from ingot_amd import _lib
    from ingot_amd.abi import Chain

    macro = MACRO.read_text()
    # the label literal is the field name plus a NUL terminator
    assert 'format!("{}\\0", self.fname)' in macro
    assert "CRStr::new_unchecked(#fname_str)" in macro
    text = PACKETS.read_text()
    structs = {}
    for m in re.finditer(r"#\[derive\(Parse\)\]\s*pub struct (\w+)<[^>]*>\s*\{(.*?)\n\}", text,
                         re.S):
        structs[m.group(1)] = re.findall(r"^\s*pub (\w+):", m.group(2), re.M)
    assert set(structs) >= {"UdpParser", "GenericUlp", "GeneveOverV6Tunnel"}
    lib = _lib.load()
    for name, chain in (("UdpParser", Chain.UdpParser), ("GenericUlp", Chain.GenericUlp),
                        ("GeneveOverV6Tunnel", Chain.GeneveOverV6Tunnel)):
        fields = structs[name]
        n = lib.ingot_chain_layer_count(int(chain))
        assert n == len(fields), name
        got = [lib.ingot_chain_layer_label(int(chain), i) + b"\0" for i in range(n)]
        assert got == [f"{f}\0".encode() for f in fields], name
