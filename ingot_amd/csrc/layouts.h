// layouts.h — kernel-side metadata: ingot-macros field layouts as constexpr
// tables.
//
// ingot decides each header's wire layout at compile time in
// `#[derive(Ingot)]` (ingot-macros/src/packet/mod.rs:547-821): fields in
// declaration order, `repr(C, packed)`; byte-aligned power-of-two ints become
// zerocopy big-endian words, runs of sub-byte / odd-width fields become one
// `[u8; n]` bitfield read MSB-first (bitfield.rs:40-315), `[u8; N]` and
// zerocopy fields are byte arrays.  Every field is therefore fully described
// by (first bit, width) from the header start, read big-endian.  This file
// restates those layouts for the headers on the parse path so the kernels can
// extract any getter with one generic, constant-folded BE bit read.
#pragma once

#include <stdint.h>

namespace ingot_gpu {
namespace layout {

struct Field {
    uint16_t bit;   // first bit, MSB-first from the header start
    uint8_t bits;   // width
    constexpr uint32_t byte0() const { return bit / 8u; }
    constexpr uint32_t nbytes() const { return (bit % 8u + bits + 7u) / 8u; }
    constexpr uint32_t rshift() const { return (8u - ((bit + bits) % 8u)) % 8u; }
    constexpr uint32_t mask() const { return bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u); }
};

// Ethernet (ingot/src/ethernet.rs:46-55) — 14 B
namespace eth {
constexpr uint32_t LEN = 14;
constexpr Field ethertype{96, 16};
}  // namespace eth

// VlanBody (ethernet.rs:57-65) — 4 B: one 2-B bitfield + ethertype
namespace vlan {
constexpr uint32_t LEN = 4;
constexpr Field priority{0, 3}, dei{3, 1}, vid{4, 12}, ethertype{16, 16};
}  // namespace vlan

// Ipv4 (ingot/src/ip.rs:63-93) — 20 B + options ((ihl*4).saturating_sub(20))
namespace ipv4 {
constexpr uint32_t LEN = 20;
constexpr Field version{0, 4}, ihl{4, 4}, dscp{8, 6}, ecn{14, 2}, total_len{16, 16},
    identification{32, 16}, flags{48, 3}, fragment_offset{51, 13}, hop_limit{64, 8},
    protocol{72, 8}, checksum{80, 16}, source{96, 32}, destination{128, 32};
}  // namespace ipv4

// Ipv6 (ip.rs:159-182) — 40 B + Repeated<LowRentV6Eh>
namespace ipv6 {
constexpr uint32_t LEN = 40;
constexpr Field version{0, 4}, dscp{4, 6}, ecn{10, 2}, flow_label{12, 20}, payload_len{32, 16},
    next_header{48, 8}, hop_limit{56, 8};
constexpr uint32_t SOURCE_BYTE = 8, DESTINATION_BYTE = 24;
}  // namespace ipv6

// IpV6ExtFragment (ip.rs:190-200) — 8 B
namespace v6frag {
constexpr uint32_t LEN = 8;
constexpr Field next_header{0, 8}, reserved{8, 8}, fragment_offset{16, 13}, res{29, 2},
    more_frags{31, 1}, ident{32, 32};
}  // namespace v6frag

// IpV6Ext6564 (ip.rs:202-211) — 2 B fixed + data (6 + ext_len*8)
namespace v6ext6564 {
constexpr uint32_t FIXED = 2;
constexpr Field next_header{0, 8}, ext_len{8, 8};
}  // namespace v6ext6564

// Tcp (ingot/src/tcp.rs:9-30) — 20 B + options ((data_offset*4).saturating_sub(20))
namespace tcp {
constexpr uint32_t LEN = 20;
constexpr Field source{0, 16}, destination{16, 16}, sequence{32, 32}, acknowledgement{64, 32},
    data_offset{96, 4}, reserved{100, 4}, flags{104, 8}, window_size{112, 16}, checksum{128, 16},
    urgent_ptr{144, 16};
}  // namespace tcp

// Udp (ingot/src/udp.rs:8-15) — 8 B
namespace udp {
constexpr uint32_t LEN = 8;
constexpr Field source{0, 16}, destination{16, 16}, length{32, 16}, checksum{48, 16};
}  // namespace udp

// IcmpV4 / IcmpV6 (ingot/src/icmp.rs:42-50, 114-122) — 8 B
namespace icmp {
constexpr uint32_t LEN = 8;
constexpr Field ty{0, 8}, code{8, 8}, checksum{16, 16}, rest_of_hdr{32, 32};
}  // namespace icmp

// Geneve (ingot/src/geneve.rs:16-44) — 8 B + options (opt_len*4)
namespace geneve {
constexpr uint32_t LEN = 8;
constexpr Field version{0, 2}, opt_len{2, 6}, flags{8, 8}, protocol_type{16, 16}, vni{32, 24},
    reserved{56, 8};
constexpr uint32_t FLAGS_KNOWN = 0xc0;  // GeneveFlags bits (geneve.rs:47-53)
}  // namespace geneve

// GeneveOpt (geneve.rs:80-102) — 4 B + data (length*4)
namespace geneve_opt {
constexpr uint32_t LEN = 4;
constexpr Field opt_class{0, 16}, option_type{16, 8}, reserved{24, 3}, length{27, 5};
}  // namespace geneve_opt

// Protocol constants (ethernet.rs:12-20, ip.rs:20-38).
constexpr uint32_t ET_IPV4 = 0x0800, ET_ARP = 0x0806, ET_VLAN = 0x8100, ET_IPV6 = 0x86dd,
                   ET_QINQ = 0x9100;
constexpr uint32_t IPP_ICMP = 1, IPP_TCP = 6, IPP_UDP = 17, IPP_ICMP_V6 = 58;

// IpProtocol::class (ip.rs:40-54) as two 256-bit membership masks:
// 44 -> FragmentHeader; {0, 43, 60, 135, 139, 140, 253, 254} -> Rfc6564.
constexpr uint32_t EH_NONE = 0, EH_FRAGMENT = 1, EH_RFC6564 = 2;

}  // namespace layout
}  // namespace ingot_gpu
