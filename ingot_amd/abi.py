"""ctypes / numpy mirrors of the C ABI types in include/ingot_gpu.h.

These are plain data layouts (no behaviour); `tests/test_abi.py` checks the
sizes and offsets against the header with a compiled probe.
"""
from __future__ import annotations

import ctypes
import enum

import numpy as np

ABI_VERSION = 3


class ParseError(enum.IntEnum):
    """ingot_types::ParseError (ingot-types/src/error.rs:22-44); value = status byte.

    The record stores 1 + the Rust discriminant so that 0 can mean Ok.
    """

    Unwanted = 1
    NeedsHint = 2
    TooSmall = 3
    StraddledHeader = 4
    NoRemainingChunks = 5
    CannotAccept = 6
    Reject = 7
    IllegalValue = 8


STATUS_OK = 0


class Chain(enum.IntEnum):
    """Parse chains (include/ingot_gpu.h enum ingot_chain)."""

    UdpParser = 0    # ingot-examples/src/packets.rs:18-24
    GenericUlp = 1   # ingot-examples/src/packets.rs:54-60
    VlanUlp = 2      # build-defined (VlanBody, ethernet.rs:57-65)
    GeneveOverV6Tunnel = 3  # ingot-examples/src/packets.rs:27-40


CHAIN_LABELS = {
    Chain.UdpParser: ("eth", "l3", "l4"),
    Chain.GenericUlp: ("inner_eth", "inner_l3", "inner_ulp"),
    Chain.VlanUlp: ("eth", "vlan", "l3", "l4"),
    Chain.GeneveOverV6Tunnel: ("outer_eth", "outer_v6", "outer_udp", "outer_encap", "inner_eth",
                               "inner_l3", "inner_ulp"),
}


class L3Kind(enum.IntEnum):
    NONE = 0
    IPV4 = 1
    IPV6 = 2


class L4Kind(enum.IntEnum):
    NONE = 0
    TCP = 1
    UDP = 2
    ICMPV4 = 3
    ICMPV6 = 4


REC_ACCEPTED = 0x01
REC_INNER = 0x02
MAX_EH_FIELDS = 4
MAX_GENEVE_OPT_FIELDS = 4

# ingot_gpu_ctx_set_tuning keys
TUNE_WINDOW_INDEXED = 1
TUNE_WINDOW_STRIDED = 2
TUNE_MAX_BLOCKS = 3
TUNE_PIPELINE = 4
TUNE_CACHE_POLICY = 5
TUNE_PIPE_DEPTH = 6
TUNE_WRITEBACK = 7
TUNE_FLOW_TABLE = 8
TUNE_SLOW_PATH = 9
TUNE_READ_PLAN = 10
TUNE_FLOW_KERNEL = 11
TUNE_RING_GRID = 12
TUNE_RING_GROUPS = 13
TUNE_XCD_REMAP = 14


class IngotRec(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_uint8),
        ("err_layer", ctypes.c_uint8),
        ("l3_kind", ctypes.c_uint8),
        ("l4_kind", ctypes.c_uint8),
        ("n_vlan", ctypes.c_uint8),
        ("n_v6ext", ctypes.c_uint8),
        ("l4_proto", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
        ("l3_off", ctypes.c_uint16),
        ("l4_off", ctypes.c_uint16),
        ("payload_off", ctypes.c_uint16),
        ("ethertype", ctypes.c_uint16),
    ]


class IngotRec8(ctypes.Structure):
    _fields_ = [
        ("status_layer_l3", ctypes.c_uint8),
        ("l4_vlan_flags", ctypes.c_uint8),
        ("n_v6ext", ctypes.c_uint8),
        ("l4_proto", ctypes.c_uint8),
        ("l4_off", ctypes.c_uint16),
        ("payload_off", ctypes.c_uint16),
    ]


class IngotV6Eh(ctypes.Structure):
    _fields_ = [
        ("ident", ctypes.c_uint32),
        ("frag_offset", ctypes.c_uint16),
        ("off", ctypes.c_uint16),
        ("kind", ctypes.c_uint8),
        ("next_header", ctypes.c_uint8),
        ("ext_len", ctypes.c_uint8),
        ("frag_res_more", ctypes.c_uint8),
    ]


U8, U16, U32 = ctypes.c_uint8, ctypes.c_uint16, ctypes.c_uint32


class IngotFields(ctypes.Structure):
    _fields_ = [
        ("rec", IngotRec),
        ("v6_flow_label", U32),
        ("tcp_sequence", U32),
        ("tcp_acknowledgement", U32),
        ("eth_ethertype", U16),
        ("vlan_vid", U16 * 2),
        ("vlan_ethertype", U16 * 2),
        ("v4_total_len", U16),
        ("v4_identification", U16),
        ("v4_fragment_offset", U16),
        ("v4_checksum", U16),
        ("v4_options_off", U16),
        ("v4_options_len", U16),
        ("v6_payload_len", U16),
        ("v6_ext_off", U16),
        ("v6_ext_len", U16),
        ("l4_source", U16),
        ("l4_destination", U16),
        ("tcp_window_size", U16),
        ("tcp_checksum", U16),
        ("tcp_urgent_ptr", U16),
        ("tcp_options_off", U16),
        ("tcp_options_len", U16),
        ("udp_length", U16),
        ("udp_checksum", U16),
        ("icmp_checksum", U16),
        ("eth_destination", U8 * 6),
        ("eth_source", U8 * 6),
        ("vlan_priority", U8 * 2),
        ("vlan_dei", U8 * 2),
        ("v4_version", U8),
        ("v4_ihl", U8),
        ("v4_dscp", U8),
        ("v4_ecn_raw", U8),
        ("v4_ecn", U8),
        ("v4_flags", U8),
        ("v4_hop_limit", U8),
        ("v4_protocol", U8),
        ("v4_source", U8 * 4),
        ("v4_destination", U8 * 4),
        ("v6_version", U8),
        ("v6_dscp", U8),
        ("v6_ecn_raw", U8),
        ("v6_ecn", U8),
        ("v6_next_header", U8),
        ("v6_hop_limit", U8),
        ("v6_source", U8 * 16),
        ("v6_destination", U8 * 16),
        ("tcp_data_offset", U8),
        ("tcp_reserved", U8),
        ("tcp_flags", U8),
        ("icmp_ty", U8),
        ("icmp_code", U8),
        ("icmp_rest_of_hdr", U8 * 4),
        ("_pad0", U8),
        ("v6_eh", IngotV6Eh * MAX_EH_FIELDS),
        ("_pad1", U8 * 52),
    ]


class IngotGeneveOpt(ctypes.Structure):
    _fields_ = [
        ("opt_class", U16),
        ("data_off", U16),
        ("option_type", U8),
        ("reserved", U8),
        ("length", U8),
        ("_pad", U8),
    ]


class IngotTunnelFields(ctypes.Structure):
    _fields_ = [
        ("outer_eth_destination", U8 * 6),
        ("outer_eth_source", U8 * 6),
        ("outer_eth_ethertype", U16),
        ("outer_udp_off", U16),
        ("outer_v6_source", U8 * 16),
        ("outer_v6_destination", U8 * 16),
        ("outer_v6_flow_label", U32),
        ("outer_v6_payload_len", U16),
        ("outer_v6_ext_len", U16),
        ("outer_v6_version", U8),
        ("outer_v6_dscp", U8),
        ("outer_v6_ecn_raw", U8),
        ("outer_v6_ecn", U8),
        ("outer_v6_next_header", U8),
        ("outer_v6_hop_limit", U8),
        ("outer_v6_n_ext", U8),
        ("outer_l4_proto", U8),
        ("outer_udp_source", U16),
        ("outer_udp_destination", U16),
        ("outer_udp_length", U16),
        ("outer_udp_checksum", U16),
        ("geneve_off", U16),
        ("inner_eth_off", U16),
        ("geneve_vni", U32),
        ("geneve_protocol_type", U16),
        ("geneve_version", U8),
        ("geneve_opt_len", U8),
        ("geneve_flags", U8),
        ("geneve_reserved", U8),
        ("geneve_n_opts", U8),
        ("geneve_critical", U8),
        ("geneve_opt", IngotGeneveOpt * MAX_GENEVE_OPT_FIELDS),
        ("_pad", U8 * 8),
    ]


class IngotGeneveFields(ctypes.Structure):
    _fields_ = [("inner", IngotFields), ("outer", IngotTunnelFields)]


assert ctypes.sizeof(IngotRec) == 16
assert ctypes.sizeof(IngotRec8) == 8
assert ctypes.sizeof(IngotV6Eh) == 12
assert ctypes.sizeof(IngotFields) == 256
assert ctypes.sizeof(IngotGeneveOpt) == 8
assert ctypes.sizeof(IngotTunnelFields) == 128
assert ctypes.sizeof(IngotGeneveFields) == 384

class HeaderKind(enum.IntEnum):
    """Single-header parse kinds (include/ingot_gpu.h enum ingot_header_kind)."""

    Ethernet = 0      # ethernet.rs:46-55
    VlanBody = 1      # ethernet.rs:57-65
    Ipv4 = 2          # ip.rs:63-93
    Ipv6 = 3          # ip.rs:159-182 (+ extension headers)
    Tcp = 4           # tcp.rs:9-30
    Udp = 5           # udp.rs:8-15
    Icmp = 6          # icmp.rs:42-50
    RepeatedUdp = 7   # Repeated<Udp> (util.rs:189-228)
    Geneve = 8        # geneve.rs:16-44
    L3 = 16           # choice, ingot-examples/src/choices.rs:17-21
    L4 = 17           # choices.rs:25-29
    Ulp = 18          # choices.rs:32-38


HINT_NONE = 0xFFFFFFFF


class IngotHdr(ctypes.Structure):
    _fields_ = [("status", ctypes.c_uint8), ("kind", ctypes.c_uint8), ("used", ctypes.c_uint16),
                ("hint", ctypes.c_uint32)]


REC_DTYPE = np.dtype(IngotRec)
HDR_DTYPE = np.dtype(IngotHdr)
FIELDS_DTYPE = np.dtype(IngotFields)
REC8_DTYPE = np.dtype(IngotRec8)
GENEVE_FIELDS_DTYPE = np.dtype(IngotGeneveFields)
REC_BYTES = REC_DTYPE.itemsize
REC8_BYTES = REC8_DTYPE.itemsize


def rec16_to_rec8(rec: np.ndarray) -> np.ndarray:
    """The ingot_rec8 encoding of ingot_rec records (include/ingot_gpu.h)."""
    out = np.zeros(rec.shape, dtype=REC8_DTYPE)
    st = rec["status"].astype(np.uint32)
    layer = np.where(st != 0, rec["err_layer"].astype(np.uint32) & 3, 0)
    out["status_layer_l3"] = ((st & 15) | (layer << 4) | (rec["l3_kind"].astype(np.uint32) << 6)
                              ).astype(np.uint8)
    out["l4_vlan_flags"] = (rec["l4_kind"].astype(np.uint32) | (rec["n_vlan"].astype(np.uint32)
                            << 3) | ((rec["flags"].astype(np.uint32) & 1) << 5)).astype(np.uint8)
    out["n_v6ext"] = rec["n_v6ext"]
    out["l4_proto"] = rec["l4_proto"]
    out["l4_off"] = rec["l4_off"]
    out["payload_off"] = rec["payload_off"]
    return out


FIELDS_BYTES = FIELDS_DTYPE.itemsize


_FIELD_NAMES = """ETH_ETHERTYPE VLAN_PRIORITY VLAN_DEI VLAN_VID VLAN_ETHERTYPE
V4_VERSION V4_IHL V4_DSCP V4_ECN V4_TOTAL_LEN V4_IDENTIFICATION V4_FLAGS V4_FRAGMENT_OFFSET
V4_HOP_LIMIT V4_PROTOCOL V4_CHECKSUM V4_SOURCE V4_DESTINATION
V6_VERSION V6_DSCP V6_ECN V6_FLOW_LABEL V6_PAYLOAD_LEN V6_NEXT_HEADER V6_HOP_LIMIT
TCP_SOURCE TCP_DESTINATION TCP_SEQUENCE TCP_ACKNOWLEDGEMENT TCP_DATA_OFFSET TCP_RESERVED
TCP_FLAGS TCP_WINDOW_SIZE TCP_CHECKSUM TCP_URGENT_PTR
UDP_SOURCE UDP_DESTINATION UDP_LENGTH UDP_CHECKSUM ICMP_TY ICMP_CODE ICMP_CHECKSUM
GENEVE_VERSION GENEVE_OPT_LEN GENEVE_FLAGS GENEVE_PROTOCOL_TYPE GENEVE_VNI
GENEVE_RESERVED""".split()
# enum ingot_field (include/ingot_gpu.h): setter targets of ingot_gpu_parse_modify
Field = enum.IntEnum("Field", [(n, i) for i, n in enumerate(_FIELD_NAMES)])


class EditOp(enum.IntEnum):
    SET = 0
    ADD = 1
    SUB = 2
    AND = 3
    OR = 4
    XOR = 5


MAX_EDITS = 16


class IngotEdit(ctypes.Structure):
    _fields_ = [("layer", U8), ("field", U8), ("op", U8), ("index", U8), ("value", U32)]


assert ctypes.sizeof(IngotEdit) == 8
EDIT_DTYPE = np.dtype(IngotEdit)


def edits_array(edits) -> np.ndarray:
    """[(layer, Field, EditOp, value[, index]), ...] -> ingot_edit array."""
    a = np.zeros(len(edits), dtype=EDIT_DTYPE)
    for k, e in enumerate(edits):
        a[k]["layer"], a[k]["field"], a[k]["op"], a[k]["value"] = e[0], int(e[1]), int(e[2]), e[3]
        a[k]["index"] = e[4] if len(e) > 4 else 0
    return a


class EmitSource(enum.IntEnum):
    """enum ingot_emit_source: where a per-packet setter's value comes from."""

    LENGTH = 0  # the packet's emitted bytes from the header's start to its end, + add
    U16 = 1     # a u16 per packet (device array) + add
    U32 = 2     # a u32 per packet (device array) + add
    VALUE = 3   # `add` for every packet


MAX_EMIT_SETS = 8
MAX_EMIT_HDR = 256


class IngotEmitSet(ctypes.Structure):
    _fields_ = [("at", U16), ("field", U8), ("source", U8), ("add", ctypes.c_int32),
                ("d_values", ctypes.c_void_p)]


assert ctypes.sizeof(IngotEmitSet) == 16
EMIT_SET_DTYPE = np.dtype(IngotEmitSet)


def emit_sets_array(sets) -> np.ndarray:
    """[(at, Field, EmitSource, add[, values pointer]), ...] -> ingot_emit_set
    array (values: a device address for U16 / U32 sources, else 0)."""
    a = np.zeros(len(sets), dtype=EMIT_SET_DTYPE)
    for k, e in enumerate(sets):
        add = ((int(e[3]) + (1 << 31)) % (1 << 32)) - (1 << 31)  # modulo 2^32, as the C int32
        a[k]["at"], a[k]["field"], a[k]["source"], a[k]["add"] = e[0], int(e[1]), int(e[2]), add
        a[k]["d_values"] = e[4] if len(e) > 4 and e[4] is not None else 0
    return a


class GenProfile(enum.IntEnum):
    """Synthetic traffic profiles (include/ingot_pktgen.h)."""

    ADVERSARIAL = 0
    V4UDP64 = 2
    MIXED = 3
    VLAN_V6EH = 4
    FLOWS = 5
    GENEVE = 6              # OPTE-style Geneve-over-IPv6 tunnel traffic
    GENEVE_ADVERSARIAL = 7  # tunnel-shaped frames with every outer/inner defect


GEN_SEED = 20250808
