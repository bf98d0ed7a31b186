/*
 * ingot_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Scalar CPU restatement of ingot's single-slice parse path.  Each function
 * cites the reference file:line whose behaviour it restates; paths are
 * relative to the reference checkout (oxidecomputer/ingot @ 2025-08-08).
 * Nothing here is shipped: the product path (ingot_amd/, include/) never
 * links this file, and bench.py times it only as the "port" CPU baseline.
 *
 * Parity pinning: tests/golden/kats.json holds the reference's own
 * known-answer vectors (ingot/src/tests.rs, ingot-examples/src/tests.rs,
 * ingot-examples/benches/packet.rs) and tests/test_oracle_golden.py checks
 * this file against every one of them.
 */
#define _GNU_SOURCE
#include "ingot_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

/* Static contiguous partition of [0, n) over nthreads pthreads (the calling
 * thread takes the first range); defined with the batch driver below. */
typedef void (*range_fn)(void* ctx, uint64_t lo, uint64_t hi);
static int parallel_ranges(uint64_t n, int nthreads, range_fn fn, void* ctx);

/* ParseError discriminants + 1 (ingot-types/src/error.rs:22-44). */
enum {
    PE_OK = INGOT_OK,
    PE_UNWANTED = INGOT_ERR_UNWANTED,
    PE_NEEDS_HINT = INGOT_ERR_NEEDS_HINT,
    PE_TOO_SMALL = INGOT_ERR_TOO_SMALL,
    PE_STRADDLED = INGOT_ERR_STRADDLED_HEADER,
    PE_CANNOT_ACCEPT = INGOT_ERR_CANNOT_ACCEPT
};

/* Ethertype constants (ingot/src/ethernet.rs:12-20). */
#define ET_IPV4 0x0800u
#define ET_ARP 0x0806u
#define ET_VLAN 0x8100u
#define ET_IPV6 0x86ddu
#define ET_QINQ 0x9100u

/* IpProtocol constants (ingot/src/ip.rs:20-38). */
#define IPP_ICMP 1u
#define IPP_TCP 6u
#define IPP_UDP 17u
#define IPP_ICMP_V6 58u

/* ------------------------------------------------------------------------
 * Field layout tables — a restatement of the ingot-macros layout rules
 * (packet/mod.rs:547-821): fields in declaration order, packed, widths from
 * the declared primitive (u4, u13be, u16be, [u8; 6] ...).  (bit offset, bits)
 * ---------------------------------------------------------------------- */
/* Ethernet (ethernet.rs:46-55): destination [u8;6], source [u8;6], ethertype u16be */
#define ETH_LEN 14u
/* VlanBody (ethernet.rs:57-65): priority u3, dei u1, vid u12be, ethertype u16be */
#define VLAN_LEN 4u
#define VLAN_PRIORITY 0, 3
#define VLAN_DEI 3, 1
#define VLAN_VID 4, 12
#define VLAN_ETHERTYPE 16, 16
/* Ipv4 (ip.rs:63-93) */
#define V4_LEN 20u
#define V4_VERSION 0, 4
#define V4_IHL 4, 4
#define V4_DSCP 8, 6
#define V4_ECN 14, 2
#define V4_TOTAL_LEN 16, 16
#define V4_IDENT 32, 16
#define V4_FLAGS 48, 3
#define V4_FRAG_OFF 51, 13
#define V4_HOP_LIMIT 64, 8
#define V4_PROTOCOL 72, 8
#define V4_CHECKSUM 80, 16
/* Ipv6 (ip.rs:159-182) */
#define V6_LEN 40u
#define V6_VERSION 0, 4
#define V6_DSCP 4, 6
#define V6_ECN 10, 2
#define V6_FLOW 12, 20
#define V6_PAYLOAD_LEN 32, 16
#define V6_NEXT_HEADER 48, 8
#define V6_HOP_LIMIT 56, 8
/* IpV6ExtFragment (ip.rs:190-200): next_header u8, reserved u8,
 * fragment_offset u13be, res u2, more_frags u1, ident u32be */
#define FRAG_LEN 8u
#define FRAG_OFFSET 16, 13
#define FRAG_RES 29, 2
#define FRAG_MORE 31, 1
#define FRAG_IDENT 32, 32
/* IpV6Ext6564 (ip.rs:202-211): next_header u8, ext_len u8, data var_len */
#define EH6564_FIXED 2u
/* Tcp (tcp.rs:9-30) */
#define TCP_LEN 20u
#define TCP_DATA_OFFSET 96, 4
#define TCP_RESERVED 100, 4
/* Udp (udp.rs:8-15), IcmpV4/IcmpV6 (icmp.rs:42-50, 114-122) */
#define UDP_LEN 8u
#define ICMP_LEN 8u
/* Geneve (geneve.rs:16-44): version u2, opt_len u6, flags u8,
 * protocol_type u16be, vni [u8;3], reserved u8, options var_len */
#define GENEVE_LEN 8u
#define GENEVE_VERSION 0, 2
#define GENEVE_OPT_LEN_F 2, 6
/* GeneveOpt (geneve.rs:80-102): class u16be, option_type u8, reserved u3,
 * length u5, data var_len */
#define GENEVE_OPT_LEN 4u
#define GOPT_RESERVED 24, 3
#define GOPT_LENGTH 27, 5

uint64_t oracle_be_bits(const uint8_t* hdr, uint32_t first_bit, uint32_t n_bits) {
    /* bitfield.rs:40-186: the covering bytes, read as a big-endian integer,
     * shifted right by the bits after the field's end in its last byte and
     * masked to n_bits. */
    uint32_t fb = first_bit / 8u;
    uint32_t lb = (first_bit + n_bits + 7u) / 8u;
    unsigned __int128 acc = 0;
    for (uint32_t b = fb; b < lb; ++b) acc = (acc << 8) | hdr[b];
    uint32_t right = (8u - ((first_bit + n_bits) % 8u)) % 8u;
    acc >>= right;
    uint64_t mask = (n_bits >= 64) ? ~(uint64_t)0 : (((uint64_t)1 << n_bits) - 1u);
    return (uint64_t)acc & mask;
}

#define BITS(h, spec) ((uint32_t)oracle_be_bits((h), spec))

static uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* Ecn::from_network (ip.rs:111-119): 3 maps to Capable0. */
static uint8_t ecn_from_network(uint32_t raw) { return (uint8_t)(raw == 3 ? 1 : raw); }

int oracle_v6eh_class(uint8_t proto) {
    /* IpProtocol::class (ip.rs:40-54) */
    switch (proto) {
    case 44:
        return INGOT_EH_FRAGMENT;
    case 0: case 43: case 60: case 135: case 139: case 140: case 253: case 254:
        return INGOT_EH_RFC6564;
    default:
        return 0;
    }
}

/* ------------------------------------------------------------------------
 * Per-header parse bodies: the generated `HeaderParse::parse_choice`
 * (packet/mod.rs:1831-2005).  Each fixed chunk is an
 * `Accessor::read_from_prefix` (accessor.rs:30-67: len >= size else TooSmall);
 * each var_len chunk is `from.split_at(chunk_len)` else TooSmall
 * (mod.rs:1867-1875).  `n` = bytes left in the slice.
 * ---------------------------------------------------------------------- */
static int parse_eth(const uint8_t* s, uint32_t n, uint32_t* used, uint32_t* hint) {
    if (n < ETH_LEN) return PE_TOO_SMALL;
    *used = ETH_LEN;
    *hint = be16(s + 12); /* next_layer ethertype (ethernet.rs:53) */
    return PE_OK;
}

static int parse_vlan(const uint8_t* s, uint32_t n, uint32_t* used, uint32_t* hint) {
    if (n < VLAN_LEN) return PE_TOO_SMALL;
    *used = VLAN_LEN;
    *hint = be16(s + 2); /* next_layer ethertype (ethernet.rs:63) */
    return PE_OK;
}

static int parse_ipv4(const uint8_t* s, uint32_t n, uint32_t* used, uint32_t* hint) {
    if (n < V4_LEN) return PE_TOO_SMALL;
    uint32_t ihl = BITS(s, V4_IHL);
    uint32_t opt = ihl * 4 > 20 ? ihl * 4 - 20 : 0; /* saturating_sub, ip.rs:91 */
    if (n - V4_LEN < opt) return PE_TOO_SMALL;
    *used = V4_LEN + opt;
    *hint = s[9]; /* next_layer protocol (ip.rs:80-81) */
    return PE_OK;
}

/* LowRentV6Eh::parse_choice (ip.rs:184-188; choice.rs:193-246 with
 * map_on = IpProtocol::class). */
static int parse_v6eh(const uint8_t* s, uint32_t n, uint32_t hint, uint32_t* used,
                      uint32_t* hint_out, int* kind) {
    int c = oracle_v6eh_class((uint8_t)hint);
    *kind = c;
    if (c == 0) return PE_UNWANTED;
    if (c == INGOT_EH_FRAGMENT) {
        if (n < FRAG_LEN) return PE_TOO_SMALL;
        *used = FRAG_LEN;
    } else {
        if (n < EH6564_FIXED) return PE_TOO_SMALL;
        uint32_t data = 6u + (uint32_t)s[1] * 8u; /* ip.rs:209 */
        if (n - EH6564_FIXED < data) return PE_TOO_SMALL;
        *used = EH6564_FIXED + data;
    }
    *hint_out = s[0];
    return PE_OK;
}

static void fill_eh(ingot_v6eh* e, const uint8_t* s, int kind, uint32_t off) {
    memset(e, 0, sizeof *e);
    e->kind = (uint8_t)kind;
    e->off = (uint16_t)off;
    e->next_header = s[0];
    e->ext_len = s[1];
    if (kind == INGOT_EH_FRAGMENT) {
        e->frag_offset = (uint16_t)BITS(s, FRAG_OFFSET);
        e->frag_res_more = (uint8_t)((BITS(s, FRAG_RES) << 1) | BITS(s, FRAG_MORE));
        e->ident = BITS(s, FRAG_IDENT);
    }
}

/* Ipv6 body: 40-B chunk, then the `subparse(on_next_layer)` Repeated<LowRentV6Eh>
 * over the rest of the slice (mod.rs:1933-1975) = RepeatedView::parse_choice
 * (util.rs:189-228): loop while bytes remain; Unwanted ends the chain, any
 * other error is the header's error; the last EH's next_header is the hint. */
static int parse_ipv6(const uint8_t* s, uint32_t n, uint32_t frame_off, uint32_t* used,
                      uint32_t* hint, uint32_t* n_eh, ingot_fields* F) {
    if (n < V6_LEN) return PE_TOO_SMALL;
    uint32_t h = s[6];
    const uint8_t* rest = s + V6_LEN;
    uint32_t rn = n - V6_LEN;
    uint32_t read = 0;
    while (read < rn) {
        uint32_t u = 0, h2 = 0;
        int kind = 0;
        int r = parse_v6eh(rest + read, rn - read, h, &u, &h2, &kind);
        if (r == PE_UNWANTED) break;
        if (r != PE_OK) return r;
        if (F && *n_eh < INGOT_MAX_EH_FIELDS)
            fill_eh(&F->v6_eh[*n_eh], rest + read, kind, frame_off + V6_LEN + read);
        *n_eh += 1;
        read += u;
        h = h2;
    }
    *used = V6_LEN + read;
    *hint = h;
    return PE_OK;
}

static int parse_tcp(const uint8_t* s, uint32_t n, uint32_t* used) {
    if (n < TCP_LEN) return PE_TOO_SMALL;
    uint32_t doff = BITS(s, TCP_DATA_OFFSET);
    uint32_t opt = doff * 4 > 20 ? doff * 4 - 20 : 0; /* tcp.rs:28 */
    if (n - TCP_LEN < opt) return PE_TOO_SMALL;
    *used = TCP_LEN + opt;
    return PE_OK;
}

static int parse_fixed(uint32_t n, uint32_t size, uint32_t* used) {
    if (n < size) return PE_TOO_SMALL;
    *used = size;
    return PE_OK;
}

/* ------------------------------------------------------------------------
 * Getter materialisation (generated XRef getters, packet/mod.rs:1183-1479).
 * ---------------------------------------------------------------------- */
static void fields_eth(ingot_fields* F, const uint8_t* s) {
    memcpy(F->eth_destination, s, 6);
    memcpy(F->eth_source, s + 6, 6);
    F->eth_ethertype = (uint16_t)be16(s + 12);
}

static void fields_vlan(ingot_fields* F, int i, const uint8_t* s) {
    F->vlan_priority[i] = (uint8_t)BITS(s, VLAN_PRIORITY);
    F->vlan_dei[i] = (uint8_t)BITS(s, VLAN_DEI);
    F->vlan_vid[i] = (uint16_t)BITS(s, VLAN_VID);
    F->vlan_ethertype[i] = (uint16_t)BITS(s, VLAN_ETHERTYPE);
}

static void fields_ipv4(ingot_fields* F, const uint8_t* s, uint32_t off, uint32_t used) {
    F->v4_version = (uint8_t)BITS(s, V4_VERSION);
    F->v4_ihl = (uint8_t)BITS(s, V4_IHL);
    F->v4_dscp = (uint8_t)BITS(s, V4_DSCP);
    F->v4_ecn_raw = (uint8_t)BITS(s, V4_ECN);
    F->v4_ecn = ecn_from_network(F->v4_ecn_raw);
    F->v4_total_len = (uint16_t)BITS(s, V4_TOTAL_LEN);
    F->v4_identification = (uint16_t)BITS(s, V4_IDENT);
    F->v4_flags = (uint8_t)BITS(s, V4_FLAGS); /* from_bits_truncate keeps all 3 */
    F->v4_fragment_offset = (uint16_t)BITS(s, V4_FRAG_OFF);
    F->v4_hop_limit = (uint8_t)BITS(s, V4_HOP_LIMIT);
    F->v4_protocol = (uint8_t)BITS(s, V4_PROTOCOL);
    F->v4_checksum = (uint16_t)BITS(s, V4_CHECKSUM);
    memcpy(F->v4_source, s + 12, 4);
    memcpy(F->v4_destination, s + 16, 4);
    F->v4_options_off = (uint16_t)(off + V4_LEN);
    F->v4_options_len = (uint16_t)(used - V4_LEN);
}

static void fields_ipv6(ingot_fields* F, const uint8_t* s, uint32_t off, uint32_t used) {
    F->v6_version = (uint8_t)BITS(s, V6_VERSION);
    F->v6_dscp = (uint8_t)BITS(s, V6_DSCP);
    F->v6_ecn_raw = (uint8_t)BITS(s, V6_ECN);
    F->v6_ecn = ecn_from_network(F->v6_ecn_raw);
    F->v6_flow_label = BITS(s, V6_FLOW);
    F->v6_payload_len = (uint16_t)BITS(s, V6_PAYLOAD_LEN);
    F->v6_next_header = (uint8_t)BITS(s, V6_NEXT_HEADER);
    F->v6_hop_limit = (uint8_t)BITS(s, V6_HOP_LIMIT);
    memcpy(F->v6_source, s + 8, 16);
    memcpy(F->v6_destination, s + 24, 16);
    F->v6_ext_off = (uint16_t)(off + V6_LEN);
    F->v6_ext_len = (uint16_t)(used - V6_LEN);
}

static void fields_tcp(ingot_fields* F, const uint8_t* s, uint32_t off, uint32_t used) {
    F->l4_source = (uint16_t)be16(s);
    F->l4_destination = (uint16_t)be16(s + 2);
    F->tcp_sequence = (uint32_t)oracle_be_bits(s, 32, 32);
    F->tcp_acknowledgement = (uint32_t)oracle_be_bits(s, 64, 32);
    F->tcp_data_offset = (uint8_t)BITS(s, TCP_DATA_OFFSET);
    F->tcp_reserved = (uint8_t)BITS(s, TCP_RESERVED);
    F->tcp_flags = s[13];
    F->tcp_window_size = (uint16_t)be16(s + 14);
    F->tcp_checksum = (uint16_t)be16(s + 16);
    F->tcp_urgent_ptr = (uint16_t)be16(s + 18);
    F->tcp_options_off = (uint16_t)(off + TCP_LEN);
    F->tcp_options_len = (uint16_t)(used - TCP_LEN);
}

static void fields_udp(ingot_fields* F, const uint8_t* s) {
    F->l4_source = (uint16_t)be16(s);
    F->l4_destination = (uint16_t)be16(s + 2);
    F->udp_length = (uint16_t)be16(s + 4);
    F->udp_checksum = (uint16_t)be16(s + 6);
}

static void fields_icmp(ingot_fields* F, const uint8_t* s) {
    F->icmp_ty = s[0];
    F->icmp_code = s[1];
    F->icmp_checksum = (uint16_t)be16(s + 2);
    memcpy(F->icmp_rest_of_hdr, s + 4, 4);
}

/* ------------------------------------------------------------------------
 * Chain driver: generated `parse_slice` (parse.rs:496-509) running the layer
 * fragments (parse.rs:292-416): layer 0 via parse, later layers via
 * parse_choice(slice, prev_hint), errors tagged with the layer label,
 * `from=` conversion after the parse (parse.rs:196-200), control fn after
 * the layer (parse.rs:229-254), Option<> layers skipped once accepted.
 * ---------------------------------------------------------------------- */
typedef struct {
    const uint8_t* f;
    uint32_t len; /* end of the current chunk (the whole frame for parse_slice) */
    uint32_t p;   /* bytes consumed */
    ingot_rec* r;
    ingot_fields* F;
    /* parse_read over chunks (parse.rs:511-537): f is the chunks
     * concatenated (copied in as the walk reaches them), chunk k spans
     * sum(seglen[0..k)) .. + seglen[k]; seglen NULL for parse_slice. */
    const uint16_t* seglen;
    uint32_t nseg, k;
    const uint8_t* arena;
    const uint64_t* seg_off;
    uint8_t* buf;
} walk_t;

/* Append chunk k of a parse_read packet to the concatenation (bytes past
 * 65535 are dropped: record offsets are u16). */
static void pull_chunk(walk_t* w) {
    uint32_t l = w->seglen[w->k];
    if (w->len + l > 65535u) l = 65535u - w->len;
    memcpy(w->buf + w->len, w->arena + w->seg_off[w->k], l);
    w->len += l;
}

static int more_chunks(const walk_t* w) { return w->seglen && w->k + 1 < w->nseg; }

static void fail(walk_t* w, int layer, int code) {
    /* parse_read: a header that does not fit its chunk is StraddledHeader when
     * another chunk exists, else TooSmall (ParseError::convert_read_parse,
     * error.rs:65-72, applied to every layer's parse error, parse.rs:296-347). */
    if (code == PE_TOO_SMALL && more_chunks(w)) code = PE_STRADDLED;
    w->r->status = (uint8_t)code;
    w->r->err_layer = (uint8_t)layer;
}

/* parse_read's step between a layer and the next (parse.rs:205-218): if the
 * layer left the chunk empty, the next chunk becomes the slice; with none
 * left that is TooSmall at this layer's label.  No-op for parse_slice and
 * after the last layer. */
static int next_slice(walk_t* w, int layer) {
    if (!w->seglen || w->p != w->len) return PE_OK;
    if (!more_chunks(w)) {
        fail(w, layer, PE_TOO_SMALL);
        return PE_TOO_SMALL;
    }
    w->k++;
    pull_chunk(w);
    return PE_OK;
}

/* L3 choice (ingot-examples/src/choices.rs:17-21; choice.rs:231-246). */
static int layer_l3(walk_t* w, int layer, uint32_t et, uint32_t* proto) {
    ingot_rec* r = w->r;
    const uint8_t* s = w->f + w->p;
    uint32_t n = w->len - w->p, used = 0, n_eh = 0;
    int e;
    if (et == ET_IPV4) {
        r->l3_kind = INGOT_L3_IPV4;
        r->l3_off = (uint16_t)w->p;
        e = parse_ipv4(s, n, &used, proto);
        if (e == PE_OK && w->F) fields_ipv4(w->F, s, w->p, used);
    } else if (et == ET_IPV6) {
        r->l3_kind = INGOT_L3_IPV6;
        r->l3_off = (uint16_t)w->p;
        e = parse_ipv6(s, n, w->p, &used, proto, &n_eh, w->F);
        r->n_v6ext = (uint8_t)(n_eh > 255 ? 255 : n_eh);
        if (w->F) {
            if (e == PE_OK) fields_ipv6(w->F, s, w->p, used);
            else memset(w->F->v6_eh, 0, sizeof w->F->v6_eh);
        }
    } else {
        e = PE_UNWANTED;
    }
    if (e != PE_OK) {
        fail(w, layer, e);
        return e;
    }
    w->p += used;
    r->payload_off = (uint16_t)w->p;
    r->l4_proto = (uint8_t)*proto;
    return PE_OK;
}

/* L4 choice (choices.rs:25-29) when ulp == 0, Ulp (choices.rs:32-38) when 1;
 * udp_only applies UdpParser's `from = "L4<Q>"` conversion to UdpPacket. */
static int layer_l4(walk_t* w, int layer, uint32_t proto, int ulp, int udp_only) {
    ingot_rec* r = w->r;
    const uint8_t* s = w->f + w->p;
    uint32_t n = w->len - w->p, used = 0;
    int e, kind;
    if (proto == IPP_TCP) {
        kind = INGOT_L4_TCP;
    } else if (proto == IPP_UDP) {
        kind = INGOT_L4_UDP;
    } else if (ulp && proto == IPP_ICMP) {
        kind = INGOT_L4_ICMPV4;
    } else if (ulp && proto == IPP_ICMP_V6) {
        kind = INGOT_L4_ICMPV6;
    } else {
        fail(w, layer, PE_UNWANTED);
        return PE_UNWANTED;
    }
    r->l4_kind = (uint8_t)kind;
    r->l4_off = (uint16_t)w->p;
    if (kind == INGOT_L4_TCP) {
        e = parse_tcp(s, n, &used);
        if (e == PE_OK && w->F) fields_tcp(w->F, s, w->p, used);
    } else if (kind == INGOT_L4_UDP) {
        e = parse_fixed(n, UDP_LEN, &used);
        if (e == PE_OK && w->F) fields_udp(w->F, s);
    } else {
        e = parse_fixed(n, ICMP_LEN, &used);
        if (e == PE_OK && w->F) fields_icmp(w->F, s);
    }
    if (e != PE_OK) {
        fail(w, layer, e);
        return e;
    }
    w->p += used;
    r->payload_off = (uint16_t)w->p;
    if (udp_only && kind != INGOT_L4_UDP) {
        /* TryFrom<ValidL4> for ValidUdp: wrong variant -> Unwanted
         * (choice.rs:153-187), reported at the l4 label. */
        fail(w, layer, PE_UNWANTED);
        return PE_UNWANTED;
    }
    return PE_OK;
}

static int layer_eth(walk_t* w, uint32_t* et) {
    uint32_t used = 0;
    int e = parse_eth(w->f, w->len, &used, et);
    if (e != PE_OK) {
        fail(w, 0, e);
        return e;
    }
    if (w->F) fields_eth(w->F, w->f);
    w->p = used;
    w->r->payload_off = (uint16_t)used;
    w->r->ethertype = (uint16_t)*et;
    return PE_OK;
}

/* Geneve (geneve.rs:16-44) as its generated parse_choice (mod.rs:1846-1957):
 * the 8-B fixed chunk (Accessor, else TooSmall), then `options`:
 * var_len = opt_len*4 cut with split_at (else TooSmall) and subparsed as
 * Repeated<GeneveOpt> with no hint = RepeatedView::parse_choice
 * (util.rs:199-216) over exactly that span.  GeneveOpt (geneve.rs:80-102) is a
 * 4-B chunk + data var_len length*4; it never returns Unwanted, so an option
 * that overruns the span is TooSmall for the whole header. */
static int parse_geneve(const uint8_t* s, uint32_t n, uint32_t frame_off, uint32_t* used,
                        ingot_tunnel_fields* T) {
    if (n < GENEVE_LEN) return PE_TOO_SMALL;
    uint32_t span = (s[0] & 0x3fu) * 4u;
    if (n - GENEVE_LEN < span) return PE_TOO_SMALL;
    uint32_t read = 0, n_opt = 0, crit = 0;
    while (read < span) {
        const uint8_t* o = s + GENEVE_LEN + read;
        uint32_t rem = span - read;
        if (rem < GENEVE_OPT_LEN) goto small;
        uint32_t data = BITS(o, GOPT_LENGTH) * 4u;
        if (rem - GENEVE_OPT_LEN < data) goto small;
        if (T && n_opt < INGOT_MAX_GENEVE_OPT_FIELDS) {
            ingot_geneve_opt* g = &T->geneve_opt[n_opt];
            g->opt_class = (uint16_t)be16(o);
            g->option_type = o[2];
            g->reserved = (uint8_t)BITS(o, GOPT_RESERVED);
            g->length = (uint8_t)BITS(o, GOPT_LENGTH);
            g->data_off = (uint16_t)(frame_off + GENEVE_LEN + read + GENEVE_OPT_LEN);
        }
        if (o[2] & 0x80u) crit = 1; /* GeneveOptionType::is_critical, geneve.rs:72-76 */
        n_opt++;
        read += GENEVE_OPT_LEN + data;
    }
    *used = GENEVE_LEN + span;
    if (T) {
        T->geneve_version = (uint8_t)BITS(s, GENEVE_VERSION);
        T->geneve_opt_len = (uint8_t)BITS(s, GENEVE_OPT_LEN_F);
        T->geneve_flags = (uint8_t)(s[1] & 0xc0u); /* GeneveFlags::from_bits_truncate */
        T->geneve_protocol_type = (uint16_t)be16(s + 2);
        T->geneve_vni = ((uint32_t)s[4] << 16) | ((uint32_t)s[5] << 8) | s[6];
        T->geneve_reserved = s[7];
        T->geneve_n_opts = (uint8_t)(n_opt > 255 ? 255 : n_opt);
        T->geneve_critical = (uint8_t)crit;
    }
    return PE_OK;
small:
    if (T) memset(T->geneve_opt, 0, sizeof T->geneve_opt);
    return PE_TOO_SMALL;
}

/* GeneveOverV6Tunnel (ingot-examples/src/packets.rs:27-40) after outer_eth:
 *   outer_v6:    #[ingot(from = "L3<Q>")] Ipv6 — the L3 choice parses, then
 *                TryFrom<ValidL3> keeps only the Ipv6 variant (choice.rs:153-187);
 *   outer_udp:   #[ingot(from = "L4<Q>")] Udp, likewise;
 *   outer_encap: Geneve (parse, no hint needed);
 *   inner_eth:   control = exit_on_arp (packets.rs:45-51); the Option<> sled
 *                after it allows Accept there (parse.rs:144-156, 221-254);
 *   inner_l3: Option<L3>, inner_ulp: Option<Ulp>. */
static void geneve_chain(walk_t* w, uint32_t et, ingot_fields* inner, ingot_tunnel_fields* T) {
    ingot_rec* r = w->r;
    const uint8_t* f = w->f;
    uint32_t proto = 0, used = 0, iet = 0;
    int e;
    if (T) {
        memcpy(T->outer_eth_destination, f, 6);
        memcpy(T->outer_eth_source, f + 6, 6);
        T->outer_eth_ethertype = (uint16_t)et;
    }
    if (next_slice(w, 0) != PE_OK) return;
    if (layer_l3(w, 1, et, &proto) != PE_OK) return;
    if (T && r->l3_kind == INGOT_L3_IPV6) {
        const uint8_t* s = f + r->l3_off;
        T->outer_v6_version = (uint8_t)BITS(s, V6_VERSION);
        T->outer_v6_dscp = (uint8_t)BITS(s, V6_DSCP);
        T->outer_v6_ecn_raw = (uint8_t)BITS(s, V6_ECN);
        T->outer_v6_ecn = ecn_from_network(T->outer_v6_ecn_raw);
        T->outer_v6_flow_label = BITS(s, V6_FLOW);
        T->outer_v6_payload_len = (uint16_t)BITS(s, V6_PAYLOAD_LEN);
        T->outer_v6_next_header = s[6];
        T->outer_v6_hop_limit = s[7];
        memcpy(T->outer_v6_source, s + 8, 16);
        memcpy(T->outer_v6_destination, s + 24, 16);
        T->outer_v6_ext_len = (uint16_t)(w->p - r->l3_off - V6_LEN);
        T->outer_v6_n_ext = r->n_v6ext;
        T->outer_l4_proto = (uint8_t)proto;
    }
    /* The generated layer is parse_choice -> control -> slice step -> from=
     * conversion (parse.rs:402-407): under parse_read an IPv4 outer header
     * that ends the last chunk is TooSmall here (parse.rs:208-219,
     * ingot-types/src/lib.rs:172-173) before TryFrom can say Unwanted. */
    if (next_slice(w, 1) != PE_OK) return;
    if (r->l3_kind != INGOT_L3_IPV6) {
        fail(w, 1, PE_UNWANTED);
        return;
    }
    if (layer_l4(w, 2, proto, 0, 0) != PE_OK) return;
    if (T && r->l4_kind == INGOT_L4_UDP) {
        const uint8_t* s = f + r->l4_off;
        T->outer_udp_off = r->l4_off;
        T->outer_udp_source = (uint16_t)be16(s);
        T->outer_udp_destination = (uint16_t)be16(s + 2);
        T->outer_udp_length = (uint16_t)be16(s + 4);
        T->outer_udp_checksum = (uint16_t)be16(s + 6);
    }
    /* likewise: slice step, then TryFrom<ValidL4> keeps only Udp */
    if (next_slice(w, 2) != PE_OK) return;
    if (r->l4_kind != INGOT_L4_UDP) {
        fail(w, 2, PE_UNWANTED);
        return;
    }
    e = parse_geneve(f + w->p, w->len - w->p, w->p, &used, T);
    if (e != PE_OK) {
        fail(w, 3, e);
        return;
    }
    if (T) T->geneve_off = (uint16_t)w->p;
    w->p += used;
    r->payload_off = (uint16_t)w->p;
    if (next_slice(w, 3) != PE_OK) return;

    e = parse_eth(f + w->p, w->len - w->p, &used, &iet);
    if (e != PE_OK) {
        fail(w, 4, e);
        return;
    }
    /* the record now describes the inner frame */
    r->flags |= INGOT_REC_INNER;
    r->l3_kind = r->l4_kind = 0;
    r->l3_off = r->l4_off = 0;
    r->n_v6ext = 0;
    r->l4_proto = 0;
    r->ethertype = (uint16_t)iet;
    if (T) T->inner_eth_off = (uint16_t)w->p;
    w->F = inner;
    if (inner) fields_eth(inner, f + w->p);
    w->p += used;
    r->payload_off = (uint16_t)w->p;
    if (iet == ET_ARP) {
        /* accepted: inner_l3 / inner_ulp are None, but parse_read still
         * steps the slice after each non-final layer */
        r->flags |= INGOT_REC_ACCEPTED;
        if (next_slice(w, 4) == PE_OK) next_slice(w, 5);
        return;
    }
    if (next_slice(w, 4) != PE_OK) return;
    if (layer_l3(w, 5, iet, &proto) != PE_OK) return;
    if (next_slice(w, 5) != PE_OK) return;
    layer_l4(w, 6, proto, 1, 0);
}

static void walk_chain(walk_t* w, int chain, ingot_fields* fields, ingot_tunnel_fields* tunnel) {
    ingot_rec* rec = w->r;
    const uint8_t* frame = w->f;
    uint32_t et = 0, proto = 0;
    rec->err_layer = 0xff;

    if (layer_eth(w, &et) != PE_OK) goto out;

    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        /* UdpParser { eth, l3: L3, #[ingot(from = "L4<Q>")] l4: UdpPacket }
         * (ingot-examples/src/packets.rs:18-24) */
        if (next_slice(w, 0) != PE_OK) goto out;
        if (layer_l3(w, 1, et, &proto) != PE_OK) goto out;
        if (next_slice(w, 1) != PE_OK) goto out;
        layer_l4(w, 2, proto, 0, 1);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        /* GenericUlp { #[ingot(control = exit_on_arp)] inner_eth,
         *              inner_l3: Option<L3>, inner_ulp: Option<Ulp> }
         * (packets.rs:45-60).  The trailing Option<> sled makes
         * accept_allowed_from = 0 (parse.rs:144-156), so Accept on the eth
         * layer is allowed and skips both optional layers. */
        if (et == ET_ARP) {
            rec->flags |= INGOT_REC_ACCEPTED;
            if (next_slice(w, 0) == PE_OK) next_slice(w, 1);
            break;
        }
        if (next_slice(w, 0) != PE_OK) goto out;
        if (layer_l3(w, 1, et, &proto) != PE_OK) goto out;
        if (next_slice(w, 1) != PE_OK) goto out;
        layer_l4(w, 2, proto, 1, 0);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        /* Build-defined chain (no reference chain uses VlanBody); under
         * parse_read each tag is a header followed by the slice step. */
        if (next_slice(w, 0) != PE_OK) goto out;
        while ((et == ET_VLAN || et == ET_QINQ) && rec->n_vlan < 2) {
            uint32_t used = 0;
            const uint8_t* s = frame + w->p;
            if (parse_vlan(s, w->len - w->p, &used, &et) != PE_OK) {
                fail(w, 1, PE_TOO_SMALL);
                goto out;
            }
            if (fields) fields_vlan(fields, rec->n_vlan, s);
            rec->n_vlan++;
            w->p += used;
            rec->payload_off = (uint16_t)w->p;
            rec->ethertype = (uint16_t)et;
            if (next_slice(w, 1) != PE_OK) goto out;
        }
        if (layer_l3(w, 2, et, &proto) != PE_OK) goto out;
        if (next_slice(w, 2) != PE_OK) goto out;
        layer_l4(w, 3, proto, 1, 0);
        break;
    case INGOT_CHAIN_GENEVE_OVER_V6:
        geneve_chain(w, et, fields, tunnel);
        break;
    default:
        fail(w, 0, PE_UNWANTED);
        break;
    }
out:
    if (rec->status == PE_OK) rec->err_layer = 0xff;
    if (fields) fields->rec = *rec;
}

static void parse_one(const uint8_t* frame, uint32_t len, int chain, ingot_rec* rec,
                      ingot_fields* fields, ingot_tunnel_fields* tunnel) {
    memset(rec, 0, sizeof *rec);
    if (fields) memset(fields, 0, sizeof *fields);
    if (tunnel) memset(tunnel, 0, sizeof *tunnel);
    const int tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    /* the tunnel's outer layers have no ingot_fields slots */
    walk_t w = {frame, len, 0, rec, tun ? 0 : fields, 0, 0, 0, 0, 0, 0};
    walk_chain(&w, chain, fields, tunnel);
}

/* parse_read: the chunks are concatenated as the walk steps into them and
 * walked with chunk-end bounds. */
static void parse_read_one(const uint8_t* arena, const uint64_t* seg_off,
                           const uint16_t* seg_len, uint32_t nseg, int chain, ingot_rec* rec,
                           ingot_fields* fields, ingot_tunnel_fields* tunnel, uint16_t* chunk) {
    static __thread uint8_t buf[65536 + 16];
    memset(rec, 0, sizeof *rec);
    if (fields) memset(fields, 0, sizeof *fields);
    if (tunnel) memset(tunnel, 0, sizeof *tunnel);
    const int tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    /* next_chunk() for the first slice: no chunks -> TooSmall (lib.rs:169-175),
     * which the eth layer then reports (a zero-length first slice). */
    walk_t w = {buf, 0, 0, rec, tun ? 0 : fields, seg_len, nseg, 0, arena, seg_off, buf};
    if (nseg) pull_chunk(&w);
    walk_chain(&w, chain, fields, tunnel);
    if (chunk) *chunk = (uint16_t)w.k;
}

void oracle_parse_one(const uint8_t* frame, uint32_t len, int chain, ingot_rec* rec,
                      ingot_fields* fields) {
    parse_one(frame, len, chain, rec, fields, 0);
}

typedef struct {
    const uint8_t* arena;
    const uint64_t* seg_off;
    const uint16_t* seg_len;
    const uint32_t* pkt_seg;
    int chain;
    ingot_rec* rec;
    ingot_fields* fields;
    ingot_geneve_fields* gfields;
    uint16_t* chunk;
} read_job_t;

static void read_range(void* ctx, uint64_t lo, uint64_t hi) {
    const read_job_t* j = (const read_job_t*)ctx;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint32_t a = j->pkt_seg[i], b = j->pkt_seg[i + 1];
        ingot_rec* r = j->gfields ? &j->gfields[i].inner.rec : &j->rec[i];
        parse_read_one(j->arena, j->seg_off + a, j->seg_len + a, b - a, j->chain, r,
                       j->gfields ? &j->gfields[i].inner : j->fields ? &j->fields[i] : 0,
                       j->gfields ? &j->gfields[i].outer : 0, j->chunk ? &j->chunk[i] : 0);
        if (j->gfields) j->rec[i] = *r;
    }
}

int oracle_parse_read_batch(const uint8_t* arena, const uint64_t* seg_off, const uint16_t* seg_len,
                            const uint32_t* pkt_seg, uint64_t n, int chain, ingot_rec* rec,
                            ingot_fields* fields, ingot_geneve_fields* gfields, uint16_t* chunk,
                            int nthreads) {
    if ((!rec && n) || !pkt_seg || chain < 0 || chain >= INGOT_CHAIN_COUNT) return -1;
    if (fields && gfields) return -1;
    read_job_t j = {arena, seg_off, seg_len, pkt_seg, chain, rec, fields, gfields, chunk};
    return parallel_ranges(n, nthreads, read_range, &j);
}

void oracle_parse_geneve(const uint8_t* frame, uint32_t len, ingot_geneve_fields* out) {
    parse_one(frame, len, INGOT_CHAIN_GENEVE_OVER_V6, &out->inner.rec, &out->inner,
              &out->outer);
}

int oracle_geneve_fields_batch(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                               uint32_t stride, uint64_t n, ingot_geneve_fields* out) {
    if ((!arena && n) || (!out && n) || (!off && stride == 0 && n)) return -1;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t o = off ? off[i] : i * (uint64_t)stride;
        uint32_t l = len ? len[i] : stride;
        if (!off && l > stride) l = stride;
        oracle_parse_geneve(arena + o, l, &out[i]);
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * Setters (packet/mod.rs:2097-2255; BE bitfield set paths bitfield.rs:188-315):
 * write n_bits at first_bit, MSB first, leaving every other bit of the
 * covering bytes unchanged.
 * ---------------------------------------------------------------------- */
void oracle_be_set_bits(uint8_t* hdr, uint32_t first_bit, uint32_t n_bits, uint64_t value) {
    for (uint32_t k = 0; k < n_bits; ++k) {
        const uint32_t bit = first_bit + k;                   /* MSB-first position */
        const uint64_t v = (value >> (n_bits - 1u - k)) & 1u;  /* k-th bit from the top */
        const uint8_t m = (uint8_t)(0x80u >> (bit % 8u));
        hdr[bit / 8u] = (uint8_t)(v ? (hdr[bit / 8u] | m) : (hdr[bit / 8u] & ~m));
    }
}

/* ingot_field -> (header kind, first bit, width), restated from the header
 * declarations (ethernet.rs:46-65, ip.rs:63-93, 159-182, tcp.rs:9-30,
 * udp.rs:8-15, icmp.rs:42-50, geneve.rs:16-44). */
enum { HK_ETH, HK_VLAN, HK_V4, HK_V6, HK_TCP, HK_UDP, HK_ICMP, HK_GENEVE };
static const struct { uint8_t kind; uint16_t bit; uint8_t bits; } FIELD_GEO[INGOT_F_COUNT] = {
    [INGOT_F_ETH_ETHERTYPE] = {HK_ETH, 96, 16},
    [INGOT_F_VLAN_PRIORITY] = {HK_VLAN, VLAN_PRIORITY}, [INGOT_F_VLAN_DEI] = {HK_VLAN, VLAN_DEI},
    [INGOT_F_VLAN_VID] = {HK_VLAN, VLAN_VID}, [INGOT_F_VLAN_ETHERTYPE] = {HK_VLAN, VLAN_ETHERTYPE},
    [INGOT_F_V4_VERSION] = {HK_V4, V4_VERSION}, [INGOT_F_V4_IHL] = {HK_V4, V4_IHL},
    [INGOT_F_V4_DSCP] = {HK_V4, V4_DSCP}, [INGOT_F_V4_ECN] = {HK_V4, V4_ECN},
    [INGOT_F_V4_TOTAL_LEN] = {HK_V4, V4_TOTAL_LEN}, [INGOT_F_V4_IDENTIFICATION] = {HK_V4, V4_IDENT},
    [INGOT_F_V4_FLAGS] = {HK_V4, V4_FLAGS}, [INGOT_F_V4_FRAGMENT_OFFSET] = {HK_V4, V4_FRAG_OFF},
    [INGOT_F_V4_HOP_LIMIT] = {HK_V4, V4_HOP_LIMIT}, [INGOT_F_V4_PROTOCOL] = {HK_V4, V4_PROTOCOL},
    [INGOT_F_V4_CHECKSUM] = {HK_V4, V4_CHECKSUM}, [INGOT_F_V4_SOURCE] = {HK_V4, 96, 32},
    [INGOT_F_V4_DESTINATION] = {HK_V4, 128, 32},
    [INGOT_F_V6_VERSION] = {HK_V6, V6_VERSION}, [INGOT_F_V6_DSCP] = {HK_V6, V6_DSCP},
    [INGOT_F_V6_ECN] = {HK_V6, V6_ECN}, [INGOT_F_V6_FLOW_LABEL] = {HK_V6, V6_FLOW},
    [INGOT_F_V6_PAYLOAD_LEN] = {HK_V6, V6_PAYLOAD_LEN},
    [INGOT_F_V6_NEXT_HEADER] = {HK_V6, V6_NEXT_HEADER}, [INGOT_F_V6_HOP_LIMIT] = {HK_V6, V6_HOP_LIMIT},
    [INGOT_F_TCP_SOURCE] = {HK_TCP, 0, 16}, [INGOT_F_TCP_DESTINATION] = {HK_TCP, 16, 16},
    [INGOT_F_TCP_SEQUENCE] = {HK_TCP, 32, 32}, [INGOT_F_TCP_ACKNOWLEDGEMENT] = {HK_TCP, 64, 32},
    [INGOT_F_TCP_DATA_OFFSET] = {HK_TCP, TCP_DATA_OFFSET}, [INGOT_F_TCP_RESERVED] = {HK_TCP, TCP_RESERVED},
    [INGOT_F_TCP_FLAGS] = {HK_TCP, 104, 8}, [INGOT_F_TCP_WINDOW_SIZE] = {HK_TCP, 112, 16},
    [INGOT_F_TCP_CHECKSUM] = {HK_TCP, 128, 16}, [INGOT_F_TCP_URGENT_PTR] = {HK_TCP, 144, 16},
    [INGOT_F_UDP_SOURCE] = {HK_UDP, 0, 16}, [INGOT_F_UDP_DESTINATION] = {HK_UDP, 16, 16},
    [INGOT_F_UDP_LENGTH] = {HK_UDP, 32, 16}, [INGOT_F_UDP_CHECKSUM] = {HK_UDP, 48, 16},
    [INGOT_F_ICMP_TY] = {HK_ICMP, 0, 8}, [INGOT_F_ICMP_CODE] = {HK_ICMP, 8, 8},
    [INGOT_F_ICMP_CHECKSUM] = {HK_ICMP, 16, 16},
    [INGOT_F_GENEVE_VERSION] = {HK_GENEVE, GENEVE_VERSION},
    [INGOT_F_GENEVE_OPT_LEN] = {HK_GENEVE, GENEVE_OPT_LEN_F},
    [INGOT_F_GENEVE_FLAGS] = {HK_GENEVE, 8, 8}, [INGOT_F_GENEVE_PROTOCOL_TYPE] = {HK_GENEVE, 16, 16},
    [INGOT_F_GENEVE_VNI] = {HK_GENEVE, 32, 24}, [INGOT_F_GENEVE_RESERVED] = {HK_GENEVE, 56, 8},
};

static int l3_hk(const ingot_rec* r) {
    return r->l3_kind == INGOT_L3_IPV4 ? HK_V4 : r->l3_kind == INGOT_L3_IPV6 ? HK_V6 : -1;
}
static int l4_hk(const ingot_rec* r) {
    switch (r->l4_kind) {
    case INGOT_L4_TCP: return HK_TCP;
    case INGOT_L4_UDP: return HK_UDP;
    case INGOT_L4_ICMPV4: case INGOT_L4_ICMPV6: return HK_ICMP;
    default: return -1;
    }
}

int oracle_parse_modify(uint8_t* frame, uint32_t len, int chain, const ingot_edit* edits,
                        uint32_t n_edits, ingot_rec* rec) {
    ingot_geneve_fields g;
    ingot_rec* r = &g.inner.rec;
    if (chain == INGOT_CHAIN_GENEVE_OVER_V6) oracle_parse_geneve(frame, len, &g);
    else parse_one(frame, len, chain, r, 0, 0);
    if (rec) *rec = *r;
    if (r->status != PE_OK) return 0;
    for (uint32_t k = 0; k < n_edits; ++k) {
        const ingot_edit* e = &edits[k];
        if (e->field >= INGOT_F_COUNT) return -1;
        int have = -1;
        uint32_t h = 0;
        const int L = e->layer;
        if (chain == INGOT_CHAIN_GENEVE_OVER_V6) {
            const ingot_tunnel_fields* t = &g.outer;
            if (L == 0) have = HK_ETH;
            else if (L == 1) { have = HK_V6; h = ETH_LEN; }
            else if (L == 2) { have = HK_UDP; h = t->outer_udp_off; }
            else if (L == 3) { have = HK_GENEVE; h = t->geneve_off; }
            else if (L == 4) { have = HK_ETH; h = t->inner_eth_off; }
            else if (L == 5) { have = l3_hk(r); h = r->l3_off; }
            else if (L == 6) { have = l4_hk(r); h = r->l4_off; }
        } else if (chain == INGOT_CHAIN_VLAN_ULP) {
            if (L == 0) have = HK_ETH;
            else if (L == 1) { if (e->index < r->n_vlan) have = HK_VLAN; h = ETH_LEN + VLAN_LEN * e->index; }
            else if (L == 2) { have = l3_hk(r); h = r->l3_off; }
            else if (L == 3) { have = l4_hk(r); h = r->l4_off; }
        } else {
            if (L == 0) have = HK_ETH;
            else if (L == 1) { have = l3_hk(r); h = r->l3_off; }
            else if (L == 2) { have = l4_hk(r); h = r->l4_off; }
        }
        if (have != FIELD_GEO[e->field].kind) continue;
        const uint32_t bit = FIELD_GEO[e->field].bit, bits = FIELD_GEO[e->field].bits;
        const uint64_t m = (bits >= 64) ? ~0ull : ((1ull << bits) - 1u);
        const uint64_t cur = oracle_be_bits(frame + h, bit, bits);
        uint64_t v;
        switch (e->op) {
        case INGOT_OP_SET: v = e->value; break;
        case INGOT_OP_ADD: v = cur + e->value; break;  /* wrapping (release-mode Rust) */
        case INGOT_OP_SUB: v = cur - e->value; break;
        case INGOT_OP_AND: v = cur & e->value; break;
        case INGOT_OP_OR: v = cur | e->value; break;
        case INGOT_OP_XOR: v = cur ^ e->value; break;
        default: return -1;
        }
        oracle_be_set_bits(frame + h, bit, bits, v & m);
    }
    return 0;
}

typedef struct {
    uint8_t* arena;
    const uint64_t* off;
    const uint16_t* len;
    uint32_t stride;
    int chain;
    const ingot_edit* edits;
    uint32_t n_edits;
    ingot_rec* rec;
    int bad;
} modify_job_t;

static void modify_range(void* ctx, uint64_t lo, uint64_t hi) {
    modify_job_t* j = (modify_job_t*)ctx;
    for (uint64_t i = lo; i < hi; ++i) {
        uint64_t o = j->off ? j->off[i] : i * (uint64_t)j->stride;
        uint32_t l = j->len ? j->len[i] : j->stride;
        if (!j->off && l > j->stride) l = j->stride;
        if (oracle_parse_modify(j->arena + o, l, j->chain, j->edits, j->n_edits,
                                j->rec ? &j->rec[i] : 0) != 0)
            j->bad = 1;
    }
}

int oracle_parse_modify_batch(uint8_t* arena, const uint64_t* off, const uint16_t* len,
                              uint32_t stride, uint64_t n, int chain, const ingot_edit* edits,
                              uint32_t n_edits, ingot_rec* rec, int nthreads) {
    if ((!off && stride == 0 && n) || chain < 0 || chain >= INGOT_CHAIN_COUNT) return -1;
    modify_job_t j = {arena, off, len, stride, chain, edits, n_edits, rec, 0};
    if (parallel_ranges(n, nthreads, modify_range, &j) != 0) return -1;
    return j.bad ? -1 : 0;
}

/* ------------------------------------------------------------------------
 * Batched Emit (ingot_gpu_emit_packets / _headers semantics): per packet the
 * owned header block as given (Emit::emit_raw of the caller's header stack,
 * ingot-types/src/emit.rs:8-120), then each setter in order through the BE
 * set path (packet/mod.rs:2097-2255, bitfield.rs:188-315), then the payload
 * bytes (a `&[u8]` member of the emitted tuple: a plain copy).  U16 / U32
 * sources read host arrays here.  copy = 0: header blocks only, at
 * dst_off[i] or i * stride.
 * ---------------------------------------------------------------------- */
typedef struct {
    const uint8_t* hdr;
    uint32_t hdr_len;
    const ingot_emit_set* sets;
    uint32_t n_sets;
    const uint8_t* src;
    const uint64_t* off;
    const uint16_t* len;
    uint8_t* dst;
    const uint64_t* dst_off;
    uint32_t stride;
    int copy;
} emit_job_t;

static void emit_range(void* ctx, uint64_t lo, uint64_t hi) {
    const emit_job_t* j = (const emit_job_t*)ctx;
    uint8_t buf[INGOT_MAX_EMIT_HDR];
    for (uint64_t i = lo; i < hi; ++i) {
        const uint32_t total = j->hdr_len + j->len[i];
        memcpy(buf, j->hdr, j->hdr_len);
        for (uint32_t k = 0; k < j->n_sets; ++k) {
            const ingot_emit_set* e = &j->sets[k];
            uint32_t v;
            switch (e->source) {
            case INGOT_EMIT_LENGTH: v = total - e->at + (uint32_t)e->add; break;
            case INGOT_EMIT_U16: v = (uint32_t)((const uint16_t*)e->d_values)[i] + (uint32_t)e->add; break;
            case INGOT_EMIT_U32: v = ((const uint32_t*)e->d_values)[i] + (uint32_t)e->add; break;
            default: v = (uint32_t)e->add; break;
            }
            const uint32_t bits = FIELD_GEO[e->field].bits;
            const uint64_t m = bits >= 32 ? 0xffffffffull : ((1ull << bits) - 1u);
            oracle_be_set_bits(buf + e->at, FIELD_GEO[e->field].bit, bits, v & m);
        }
        uint8_t* d = j->dst + (j->dst_off ? j->dst_off[i] : i * (uint64_t)j->stride);
        memcpy(d, buf, j->hdr_len);
        if (j->copy) memcpy(d + j->hdr_len, j->src + j->off[i], j->len[i]);
    }
}

int oracle_emit_batch(const uint8_t* hdr, uint32_t hdr_len, const ingot_emit_set* sets,
                      uint32_t n_sets, const uint8_t* src, const uint64_t* off,
                      const uint16_t* len, uint64_t n, uint8_t* dst, const uint64_t* dst_off,
                      uint32_t stride, int copy, int nthreads) {
    if (hdr_len > INGOT_MAX_EMIT_HDR || n_sets > INGOT_MAX_EMIT_SETS) return -1;
    for (uint32_t k = 0; k < n_sets; ++k) {
        const ingot_emit_set* e = &sets[k];
        if (e->field >= INGOT_F_COUNT || e->source > INGOT_EMIT_VALUE) return -1;
        const uint32_t bit = FIELD_GEO[e->field].bit, bits = FIELD_GEO[e->field].bits;
        if (e->at + (bit + bits + 7u) / 8u > hdr_len) return -1;
    }
    emit_job_t j = {hdr, hdr_len, sets, n_sets, src, off, len, dst, dst_off, stride, copy};
    return parallel_ranges(n, nthreads, emit_range, &j) != 0 ? -1 : 0;
}

/* ------------------------------------------------------------------------
 * Batch driver (pthreads, static contiguous partition).
 * ---------------------------------------------------------------------- */
typedef struct {
    range_fn fn;
    void* ctx;
    uint64_t lo, hi;
} range_job_t;

/* Passes each worker makes over its range per batch call (default 1).  A
 * throughput measurement only: >1 amortises thread start-up over more work
 * (bench.py's all-core CPU baseline); results are those of one pass. */
static int g_passes = 1;

void oracle_set_passes(int passes) { g_passes = passes < 1 ? 1 : passes; }

/* CPUs the workers are pinned to (bench.py's CPU baseline: one thread per
 * CPU the process may use, worker t on cpus[t % n]); none = unpinned. */
static int* g_cpus = 0;
static int g_ncpus = 0;

void oracle_set_affinity(const int* cpus, int n) {
    free(g_cpus);
    g_cpus = 0;
    g_ncpus = 0;
    if (!cpus || n <= 0) return;
    g_cpus = (int*)malloc((size_t)n * sizeof(int));
    if (!g_cpus) return;
    memcpy(g_cpus, cpus, (size_t)n * sizeof(int));
    g_ncpus = n;
}

static void pin_set(int t, cpu_set_t* set) {
    CPU_ZERO(set);
    CPU_SET(g_cpus[t % g_ncpus], set);
}

static void* run_range(void* arg) {
    range_job_t* j = (range_job_t*)arg;
    for (int k = 0; k < g_passes; ++k) j->fn(j->ctx, j->lo, j->hi);
    return 0;
}

static int parallel_ranges(uint64_t n, int nthreads, range_fn fn, void* ctx) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    range_job_t* jobs = (range_job_t*)calloc((size_t)nthreads, sizeof(range_job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    uint64_t per = (n + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t lo = per * (uint64_t)t, hi = lo + per;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        range_job_t j = {fn, ctx, lo, hi};
        jobs[t] = j;
    }
    int started = 0;
    for (int t = 1; t < nthreads; ++t) {
        pthread_attr_t attr;
        pthread_attr_t* ap = 0;
        if (g_ncpus && pthread_attr_init(&attr) == 0) {
            cpu_set_t set;
            pin_set(t, &set);
            pthread_attr_setaffinity_np(&attr, sizeof(set), &set);
            ap = &attr;
        }
        const int rc = pthread_create(&th[t], ap, run_range, &jobs[t]);
        if (ap) pthread_attr_destroy(ap);
        if (rc != 0) break;
        started = t;
    }
    /* worker 0 is the calling thread: pinned for the call, then restored */
    cpu_set_t saved;
    const int repin = g_ncpus && pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) == 0;
    if (repin) {
        cpu_set_t set;
        pin_set(0, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    run_range(&jobs[0]);
    if (repin) pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    for (int t = 1; t <= started; ++t) pthread_join(th[t], 0);
    /* any range whose thread failed to start runs here */
    for (int t = started + 1; t < nthreads; ++t) run_range(&jobs[t]);
    free(jobs);
    free(th);
    return 0;
}

typedef struct {
    const uint8_t* arena;
    const uint64_t* off;
    const uint16_t* len;
    uint32_t stride;
    int chain;
    ingot_rec* rec;
    ingot_fields* fields;
} slice_job_t;

static void slice_range(void* ctx, uint64_t lo, uint64_t hi) {
    const slice_job_t* j = (const slice_job_t*)ctx;
    for (uint64_t i = lo; i < hi; ++i) {
        uint64_t o = j->off ? j->off[i] : i * (uint64_t)j->stride;
        uint32_t l = j->len ? j->len[i] : j->stride;
        if (!j->off && l > j->stride) l = j->stride; /* a slot holds one frame */
        oracle_parse_one(j->arena + o, l, j->chain, &j->rec[i], j->fields ? &j->fields[i] : 0);
    }
}

int oracle_parse_batch(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                       uint32_t stride, uint64_t n, int chain, ingot_rec* rec,
                       ingot_fields* fields, int nthreads) {
    if ((!arena && n) || (!rec && n) || chain < 0 || chain >= INGOT_CHAIN_COUNT) return -1;
    if (!off && stride == 0 && n) return -1;
    slice_job_t j = {arena, off, len, stride, chain, rec, fields};
    return parallel_ranges(n, nthreads, slice_range, &j);
}

/* ------------------------------------------------------------------------
 * Toeplitz hash (Microsoft RSS definition): for every set bit of the input,
 * MSB first, XOR in the 32-bit window of the key starting at that bit.
 * ---------------------------------------------------------------------- */
uint32_t oracle_toeplitz(const uint8_t* key, uint32_t key_len, const uint8_t* data,
                         uint32_t n) {
    uint32_t result = 0;
    if (key_len < n + 4) return 0;
    uint64_t window = ((uint64_t)key[0] << 24) | ((uint64_t)key[1] << 16) |
                      ((uint64_t)key[2] << 8) | key[3];
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t next = key[i + 4];
        for (int b = 7; b >= 0; --b) {
            if (data[i] & (1u << b)) result ^= (uint32_t)(window >> 0);
            window = ((window << 1) | ((next >> b) & 1u)) & 0xffffffffu;
        }
    }
    return result;
}

/* ------------------------------------------------------------------------
 * Header-level entry (single `ValidX::parse`), for the reference's
 * header-level known-answer tests.  kind: 0 Ethernet, 1 VlanBody, 2 Ipv4,
 * 3 Ipv6, 4 Tcp, 5 Udp, 6 IcmpV4/V6, 7 RepeatedView<Udp> (util.rs:189-228
 * over a fixed 8-B header with a unit hint), 8 Geneve.  Returns the status; *used and
 * *hint_out (0xffffffff = None) on Ok.
 * ---------------------------------------------------------------------- */
int oracle_parse_header(int kind, const uint8_t* s, uint32_t n, uint32_t* used,
                        uint32_t* hint_out) {
    uint32_t u = 0, h = 0xffffffffu, n_eh = 0;
    int e;
    switch (kind) {
    case 0: e = parse_eth(s, n, &u, &h); break;
    case 1: e = parse_vlan(s, n, &u, &h); break;
    case 2: e = parse_ipv4(s, n, &u, &h); break;
    case 3: e = parse_ipv6(s, n, 0, &u, &h, &n_eh, 0); break;
    case 4: e = parse_tcp(s, n, &u); break;
    case 5: e = parse_fixed(n, UDP_LEN, &u); break;
    case 6: e = parse_fixed(n, ICMP_LEN, &u); break;
    case 7: {
        uint32_t read = 0;
        e = PE_OK;
        while (read < n) {
            uint32_t uu = 0;
            int r = parse_fixed(n - read, UDP_LEN, &uu);
            if (r == PE_UNWANTED) break;
            if (r != PE_OK) { e = r; break; }
            read += uu;
        }
        u = read;
        break;
    }
    case 8: e = parse_geneve(s, n, 0, &u, 0); break;
    default: return PE_UNWANTED;
    }
    if (e == PE_OK) {
        *used = u;
        *hint_out = h;
    }
    return e;
}

/* Choices (ingot-macros/src/choice.rs:231-246): `hint None -> NeedsHint`;
 * variants tried in declaration order (choice.rs:104-112); no match ->
 * Unwanted.  L3 (choices.rs:17-21): IPV4 -> Ipv4, IPV6 -> Ipv6.  L4
 * (choices.rs:25-29): TCP -> Tcp, UDP -> Udp.  Ulp (choices.rs:32-38): + ICMP
 * and ICMPv6 (one 8-B layout, icmp.rs:42-50). */
int oracle_parse_choice(int kind, uint32_t hint, const uint8_t* s, uint32_t n, uint32_t* used,
                        uint32_t* hint_out, uint32_t* variant) {
    *variant = (uint32_t)kind;
    if (hint == 0xffffffffu) return PE_NEEDS_HINT;
    int v = -1;
    if (kind == 16) {
        if (hint == 0x0800) v = 2;
        else if (hint == 0x86dd) v = 3;
    } else if (kind == 17 || kind == 18) {
        if (hint == 6) v = 4;
        else if (hint == 17) v = 5;
        else if (kind == 18 && (hint == 1 || hint == 58)) v = 6;
    } else {
        return PE_UNWANTED;
    }
    if (v < 0) return PE_UNWANTED;
    *variant = (uint32_t)v;
    return oracle_parse_header(v, s, n, used, hint_out);
}

int oracle_parse_header_batch(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                              uint32_t stride, uint64_t n, int kind, const uint32_t* hints,
                              uint32_t hint, ingot_hdr* out) {
    if (!off && !stride) return -1;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t o = off ? off[i] : i * (uint64_t)stride;
        uint32_t l = len ? len[i] : stride;
        if (!off && l > stride) l = stride;
        uint32_t used = 0, h = 0xffffffffu, variant = (uint32_t)kind;
        int st;
        if (kind >= 16) st = oracle_parse_choice(kind, hints ? hints[i] : hint, arena + o, l,
                                                 &used, &h, &variant);
        else st = oracle_parse_header(kind, arena + o, l, &used, &h);
        ingot_hdr* r = &out[i];
        r->status = (uint8_t)st;
        r->kind = (uint8_t)variant;
        r->used = st ? 0 : (uint16_t)used;
        r->hint = st ? 0xffffffffu : h;
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * Flow classification (build-defined; ingot has no flow hash): Toeplitz over
 * src | dst (| sport | dport for TCP/UDP) of frames that parse Ok with an L3.
 * ---------------------------------------------------------------------- */
int oracle_flow_hash(const uint8_t* frame, uint32_t len, int chain, const uint8_t* key,
                     uint32_t* hash) {
    ingot_rec r;
    oracle_parse_one(frame, len, chain, &r, 0);
    *hash = 0;
    if (r.status != INGOT_OK || r.l3_kind == INGOT_L3_NONE) return 0;
    uint8_t in[36];
    uint32_t n = 0;
    if (r.l3_kind == INGOT_L3_IPV4) {
        memcpy(in, frame + r.l3_off + 12, 8);
        n = 8;
    } else {
        memcpy(in, frame + r.l3_off + 8, 32);
        n = 32;
    }
    if (r.l4_kind == INGOT_L4_TCP || r.l4_kind == INGOT_L4_UDP) {
        memcpy(in + n, frame + r.l4_off, 4);
        n += 4;
    }
    *hash = oracle_toeplitz(key, 40, in, n);
    return 1;
}

int oracle_flow_hist(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                     uint32_t stride, uint64_t n, int chain, const uint8_t* key, uint32_t* hist,
                     uint32_t bins, uint32_t* hash_out, uint32_t* flow_out) {
    if (!bins || (bins & (bins - 1))) return -1;
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t o = off ? off[i] : i * (uint64_t)stride;
        uint32_t l = len ? len[i] : stride;
        if (!off && l > stride) l = stride;
        uint32_t h = 0;
        int counted = oracle_flow_hash(arena + o, l, chain, key, &h);
        if (counted) hist[h & (bins - 1)] += 1;
        if (hash_out) hash_out[i] = h;
        if (flow_out) flow_out[i] = counted ? (h & (bins - 1)) : INGOT_FLOW_NONE;
    }
    return 0;
}
