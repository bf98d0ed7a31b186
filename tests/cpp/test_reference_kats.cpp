// test_reference_kats.cpp — the reference's own chain-level tests, restated
// against the C++ mirror (include/ingot_amd.hpp); every parse runs on the GPU.
//
// Each TEST follows one test of oxidecomputer/ingot @ 2025-08-08 (file:line in
// its comment): the same frame construction and the same assertions.
// Built by __graft_entry__.build() into tests/cpp/build/, run by
// tests/test_cpp_mirror.py (pytest -m gpu).
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "ingot_amd.hpp"

using namespace ingot;
using namespace ingot::examples;
using ingot::types::ParseError;

static int g_failed = 0, g_run = 0;

#define ASSERT_EQ(a, b)                                                                  \
    do {                                                                                 \
        if (!((a) == (b))) {                                                             \
            std::fprintf(stderr, "  %s:%d: ASSERT_EQ(%s, %s) failed\n", __FILE__, __LINE__, \
                         #a, #b);                                                        \
            throw std::runtime_error("assertion");                                       \
        }                                                                                \
    } while (0)
#define ASSERT_TRUE(a) ASSERT_EQ(!!(a), true)

static std::vector<std::pair<const char*, std::function<void()>>>& registry() {
    static std::vector<std::pair<const char*, std::function<void()>>> r;
    return r;
}
struct Reg {
    Reg(const char* n, std::function<void()> f) { registry().push_back({n, f}); }
};
#define TEST(name)                          \
    static void name();                     \
    static Reg reg_##name(#name, name);     \
    static void name()

static const MacAddr6 ABCDEF{0xa, 0xb, 0xc, 0xd, 0xe, 0xf};
static const MacAddr6 BROADCAST{0xff, 0xff, 0xff, 0xff, 0xff, 0xff};

static void put16(std::vector<uint8_t>& b, size_t at, uint16_t v) {
    b[at] = (uint8_t)(v >> 8);
    b[at + 1] = (uint8_t)v;
}

// ingot-examples/src/tests.rs:22-54
TEST(parse_header_chain_with_narrowing) {
    std::vector<uint8_t> buf2(14 + 20 + 8, 0);
    for (int i = 0; i < 6; ++i) buf2[i] = BROADCAST[i], buf2[6 + i] = ABCDEF[i];
    put16(buf2, 12, ethernet::Ethertype::IPV4);
    buf2[14 + 9] = ip::IpProtocol::UDP;
    const uint8_t src[4] = {192, 168, 0, 1}, dst[4] = {192, 168, 0, 255};
    std::memcpy(&buf2[14 + 12], src, 4);
    std::memcpy(&buf2[14 + 16], dst, 4);

    auto [mystack, hint, rest] = UdpParser::parse(buf2).unwrap();
    (void)hint;
    ASSERT_TRUE(mystack.l3.ipv4.has_value());
    (void)mystack.l3.ipv4->hop_limit();
    ASSERT_EQ(mystack.eth.source(), ABCDEF);
    ASSERT_EQ(rest.size(), 0u);
}

// ingot-examples/src/tests.rs:56-118
TEST(variable_len_fields_in_header_chain) {
    const size_t V4_EXTRA = 12;
    std::vector<uint8_t> buf2(14 + 20 + V4_EXTRA + 8, 0);
    for (int i = 0; i < 6; ++i) buf2[i] = BROADCAST[i], buf2[6 + i] = ABCDEF[i];
    put16(buf2, 12, ethernet::Ethertype::IPV4);
    buf2[14] = (uint8_t)(5 + V4_EXTRA / 4);  // set_ihl
    buf2[14 + 9] = ip::IpProtocol::UDP;
    const uint8_t src[4] = {192, 168, 0, 1}, dst[4] = {192, 168, 0, 255};
    std::memcpy(&buf2[14 + 12], src, 4);
    std::memcpy(&buf2[14 + 16], dst, 4);
    for (size_t i = 0; i < V4_EXTRA; ++i) buf2[34 + i] = (uint8_t)i;
    const size_t l = buf2.size();
    put16(buf2, l - 8, 6082);
    put16(buf2, l - 6, 6081);
    put16(buf2, l - 4, 0);
    put16(buf2, l - 2, 0xffff);

    auto [mystack, hint, rest] = UdpParser::parse(buf2).unwrap();
    (void)hint;
    (void)rest;
    ASSERT_EQ(mystack.eth.source(), ABCDEF);
    ASSERT_EQ(mystack.eth.destination(), BROADCAST);
    ASSERT_EQ(mystack.eth.ethertype(), ethernet::Ethertype::IPV4);
    ASSERT_TRUE(mystack.l3.ipv4.has_value());
    const auto& v4 = *mystack.l3.ipv4;
    ASSERT_EQ(v4.protocol(), ip::IpProtocol::UDP);
    ASSERT_EQ(v4.source(), (Ipv4Addr{192, 168, 0, 1}));
    ASSERT_EQ(v4.destination(), (Ipv4Addr{192, 168, 0, 255}));
    ASSERT_EQ(v4.ihl(), 8);
    ASSERT_EQ(v4.options_ref(), (std::vector<uint8_t>{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11}));
    ASSERT_EQ(mystack.l4.source(), 6082);
    ASSERT_EQ(mystack.l4.destination(), 6081);
    ASSERT_EQ(mystack.l4.length(), 0);
    ASSERT_EQ(mystack.l4.checksum(), 0xffff);
}

// ingot-examples/src/tests.rs:120-187 (values; chunks concatenated)
TEST(parse_header_chain_multichunk_values) {
    std::vector<uint8_t> f(14 + 40 + 8, 0);
    for (int i = 0; i < 6; ++i) f[i] = BROADCAST[i], f[6 + i] = ABCDEF[i];
    put16(f, 12, ethernet::Ethertype::IPV6);
    f[14 + 6] = ip::IpProtocol::UDP;
    f[14 + 8 + 15] = 1;  // Ipv6Addr::LOCALHOST
    put16(f, 54, 6082);
    put16(f, 56, 6081);
    put16(f, 58, 128);
    put16(f, 60, 0xffff);
    f.insert(f.end(), 128, 0xaa);

    auto [hdr, hint, rest] = UdpParser::parse(f).unwrap();
    (void)hint;
    ASSERT_EQ(hdr.eth.source(), ABCDEF);
    ASSERT_EQ(hdr.eth.destination(), BROADCAST);
    ASSERT_EQ(hdr.eth.ethertype(), ethernet::Ethertype::IPV6);
    ASSERT_TRUE(hdr.l3.ipv6.has_value());
    const auto& v6 = *hdr.l3.ipv6;
    ASSERT_EQ(v6.next_header(), ip::IpProtocol::UDP);
    ASSERT_EQ(v6.next_layer(), ip::IpProtocol::UDP);
    Ipv6Addr lo{};
    lo[15] = 1;
    ASSERT_EQ(v6.source(), lo);
    ASSERT_EQ(v6.destination(), Ipv6Addr{});
    ASSERT_EQ(hdr.l4.source(), 6082);
    ASSERT_EQ(hdr.l4.destination(), 6081);
    ASSERT_EQ(hdr.l4.length(), 128);
    ASSERT_EQ(hdr.l4.checksum(), 0xffff);
    ASSERT_EQ(rest.size(), 128u);
    for (auto b : rest) ASSERT_EQ(b, 0xaa);
}

static std::vector<uint8_t> would_be_valid() {
    return {0xAA, 0x00, 0x04, 0x00, 0xFF, 0x10, 0xAA, 0x00, 0x04, 0x00, 0xFF, 0x01, 0x08, 0x00,
            0x45, 0x00, 0x00, 28 + 8, 0x00, 0x00, 0x00, 0x00, 0xf0, 0x11, 0x00, 0x00,
            8, 8, 8, 8, 192, 168, 0, 5,
            0x00, 0x80, 0x00, 53, 0x00, 0x08, 0x00, 0x00};
}

// ingot-examples/src/tests.rs:307-379
TEST(parse_reports_error_location) {
    const auto v = would_be_valid();
    auto cut = [&](size_t n) { return std::vector<uint8_t>(v.begin(), v.begin() + n); };
    auto e = GenericUlp::parse_slice(cut(4)).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::TooSmall);
    ASSERT_EQ(std::string(e.header()), "inner_eth");
    e = GenericUlp::parse_slice(cut(14)).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::TooSmall);
    ASSERT_EQ(std::string(e.header()), "inner_l3");
    e = GenericUlp::parse_slice(cut(v.size() - 1)).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::TooSmall);
    ASSERT_EQ(std::string(e.header()), "inner_ulp");

    auto u = v;
    u[14 + 9] = 0x59;  // OSPF
    e = GenericUlp::parse_slice(u).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::Unwanted);
    ASSERT_EQ(std::string(e.header()), "inner_ulp");
}

// ingot-examples/src/tests.rs:277-305 (single-slice half)
TEST(chunks_present_on_early_accept) {
    std::vector<uint8_t> pkt = {0xA8, 0x40, 0x25, 0x77, 0x77, 0x76, 0xA8, 0x40, 0x25, 0x77, 0x77,
                                0x77, 0x08, 0x06, 0, 1, 2, 3, 4, 5, 6, 7};
    auto [g, hint, b] = GenericUlp::parse(pkt).unwrap();
    (void)hint;
    ASSERT_TRUE(!g.inner_l3.has_value());
    ASSERT_TRUE(!g.inner_ulp.has_value());
    ASSERT_EQ(b.size(), 8u);
}

// ingot-examples/src/tests.rs:416-423 (single chunk of the straddle test)
TEST(straddle_failure_single_chunk) {
    const auto v = would_be_valid();
    auto e = GenericUlp::parse_slice(std::vector<uint8_t>(v.begin(), v.begin() + 16)).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::TooSmall);
    ASSERT_EQ(std::string(e.header()), "inner_l3");
}

// ingot/src/tests.rs:296-369, through a chain (Ethernet prefix, UDP suffix)
TEST(v6_repeat_extension_headers) {
    std::vector<uint8_t> f(14, 0);
    put16(f, 12, ethernet::Ethertype::IPV6);
    const uint8_t v6[] = {0x6A, 0x61, 0xe2, 0x40, 0x00, 0x10, 0x00, 0xf0,
                          0xFD, 0, 0, 0, 0, 0xF7, 1, 1, 0, 0, 0, 0, 0, 0, 0, 2,
                          0xFD, 0, 0, 0, 0, 0xF7, 1, 1, 0, 0, 0, 0, 0, 0, 0, 1,
                          44, 0x00, 0, 0, 0, 0, 0, 0,
                          253, 0, 0, 0, 0, 0, 0, 0,
                          0x11, 0x04};
    f.insert(f.end(), std::begin(v6), std::end(v6));
    f.insert(f.end(), 38, 0);
    const uint8_t udp[] = {0, 1, 0, 2, 0, 8, 0, 0};
    f.insert(f.end(), std::begin(udp), std::end(udp));

    auto [s, hint, rest] = UdpParser::parse(f).unwrap();
    (void)hint;
    (void)rest;
    ASSERT_TRUE(s.l3.ipv6.has_value());
    const auto& x = *s.l3.ipv6;
    ASSERT_EQ(x.next_layer(), ip::IpProtocol::UDP);
    ASSERT_EQ(x.extension_header_count(), 3u);
    ASSERT_EQ(x.extension_header(0).kind, INGOT_EH_RFC6564);
    ASSERT_EQ(x.extension_header(0).next_header, ip::IpProtocol::IPV6_FRAGMENT);
    ASSERT_EQ(x.extension_header(0).ext_len, 0);
    ASSERT_EQ(x.extension_header(1).kind, INGOT_EH_FRAGMENT);
    ASSERT_EQ(x.extension_header(1).next_header, ip::IpProtocol::IPV6_EXPERIMENT0);
    ASSERT_EQ(x.extension_header(2).kind, INGOT_EH_RFC6564);
    ASSERT_EQ(x.extension_header(2).next_header, ip::IpProtocol::UDP);
    ASSERT_EQ(x.extension_header(2).ext_len, 4);
    // bitset_fields_do_not_disturb_neighbours (ingot/src/tests.rs:223-294)
    ASSERT_EQ(x.version(), 6);
    ASSERT_EQ(x.dscp(), 41);
    ASSERT_EQ(x.ecn(), ip::Ecn::Capable1);
    ASSERT_EQ(x.flow_label(), 123456u);
}

// ingot-examples/benches/packet.rs:15-34, 136-138 (batched: the bench loop)
TEST(bench_parse_stack_v4_batch) {
    std::vector<uint8_t> v4 = {0, 0, 0, 0, 0, 0, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0x08, 0x00,
                               0x45, 0x00, 0x00, 28 + 8, 0, 0, 0, 0, 0xf0, 0x11, 0, 0,
                               192, 168, 0, 1, 192, 168, 0, 255,
                               0x00, 0x80, 0x17, 0xc1, 0x00, 0x08, 0x00, 0x00,
                               0, 1, 2, 3, 4, 5, 6, 7};
    std::vector<std::vector<uint8_t>> batch(1000, v4);
    auto res = UdpParser::parse_all(batch);
    ASSERT_EQ(res.size(), 1000u);
    for (auto& r : res) {
        auto& [s, hint, rest] = r.unwrap();
        (void)hint;
        ASSERT_EQ(s.l4.destination(), 0x17c1);
        ASSERT_EQ(rest.size(), 8u);
    }
}

static std::vector<uint8_t> opte_in_pkt() {
    // ingot-examples/src/tests.rs:192-261 (== ingot-examples/benches/packet.rs:59-128)
    std::vector<uint8_t> p = {
        0xA8, 0x40, 0x25, 0x77, 0x77, 0x76, 0xA8, 0x40, 0x25, 0x77, 0x77, 0x77, 0x86, 0xdd,
        0x60, 0x00, 0x00, 0x00, 0x00, 0x10, 0x11, 0xf0,
        0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01, 0, 0, 0, 0, 0, 0, 0, 0x02,
        0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01, 0, 0, 0, 0, 0, 0, 0, 0x01,
        0x1E, 0x61, 0x17, 0xC1, 0x00, 0x14, 0x00, 0x00,
        0x01, 0x00, 0x65, 0x58, 0x00, 0x04, 0xD2, 0x00,
        0x01, 0x29, 0x00, 0x00};
    const auto inner = would_be_valid();
    p.insert(p.end(), inner.begin(), inner.end());
    for (uint8_t b = 0; b < 8; ++b) p.push_back(b);
    return p;
}

// ingot-examples/src/tests.rs:189-275
TEST(test_tunnelled_unconditionals) {
    auto pkt = opte_in_pkt();
    {
        auto [opte_in, hint, rest] = GeneveOverV6Tunnel::parse(pkt).unwrap();
        (void)hint;
        ASSERT_EQ(opte_in.outer_encap.options_ref().size(), 4u);
        ASSERT_EQ(opte_in.inner_eth.ethertype(), ethernet::Ethertype::IPV4);
        ASSERT_TRUE(opte_in.inner_l3.has_value());
        ASSERT_TRUE(opte_in.inner_ulp.has_value());
        ASSERT_EQ(opte_in.outer_encap.vni(), 0x0004D2u);
        ASSERT_EQ(rest.size(), 8u);
    }
    // Now, try out pretending we're ARP and early exiting.
    put16(pkt, 74 + 12, ethernet::Ethertype::ARP);
    auto [opte_in, hint, rest] = GeneveOverV6Tunnel::parse(pkt).unwrap();
    (void)hint;
    (void)rest;
    ASSERT_TRUE(!opte_in.inner_l3.has_value());
    ASSERT_TRUE(!opte_in.inner_ulp.has_value());
}

// ingot/src/tests.rs:384-419 (to_owned of g_opt, here the tunnel's outer_encap)
TEST(geneve_to_owned_in_tunnel) {
    auto [t, hint, rest] = GeneveOverV6Tunnel::parse(opte_in_pkt()).unwrap();
    (void)hint;
    (void)rest;
    const auto& g = t.outer_encap;
    ASSERT_EQ(g.version(), 0);
    ASSERT_EQ(g.opt_len(), 1);
    ASSERT_EQ(g.flags(), 0);
    ASSERT_EQ(g.protocol_type(), 0x6558);
    ASSERT_EQ(g.vni(), 0x0004d2u);
    ASSERT_EQ(g.reserved(), 0);
    ASSERT_EQ(g.packet_length(), 12u);
    auto opts = g.options();
    ASSERT_EQ(opts.size(), 1u);
    ASSERT_EQ(opts[0].class_, 0x0129);
    ASSERT_EQ(opts[0].option_type, 0);
    ASSERT_EQ(opts[0].length, 0);
    ASSERT_TRUE(opts[0].data.empty());
}

// ingot-examples/src/tests.rs:120-187 (the parse_read half)
TEST(parse_header_chain_multichunk) {
    std::vector<uint8_t> eth(14, 0), v6(40, 0), udp(8, 0), body(128, 0xaa);
    for (int i = 0; i < 6; ++i) eth[i] = 0xff;
    const uint8_t src[] = {0xa, 0xb, 0xc, 0xd, 0xe, 0xf};
    std::memcpy(&eth[6], src, 6);
    put16(eth, 12, ethernet::Ethertype::IPV6);
    v6[6] = ip::IpProtocol::UDP;
    v6[8 + 15] = 1;  // source = ::1
    put16(udp, 0, 6082);
    put16(udp, 2, 6081);
    put16(udp, 4, 128);
    put16(udp, 6, 0xffff);
    auto res = UdpParser::parse_read({eth, v6, udp, body});
    auto& mystack = res.unwrap();
    const auto& hdr = mystack.headers;
    ASSERT_EQ(hdr.eth.source(), (MacAddr6{0xa, 0xb, 0xc, 0xd, 0xe, 0xf}));
    ASSERT_EQ(hdr.eth.destination(), (MacAddr6{0xff, 0xff, 0xff, 0xff, 0xff, 0xff}));
    ASSERT_EQ(hdr.eth.ethertype(), ethernet::Ethertype::IPV6);
    ASSERT_TRUE(hdr.l3.ipv6.has_value());
    ASSERT_EQ(hdr.l3.ipv6->next_header(), ip::IpProtocol::UDP);
    ASSERT_EQ(hdr.l3.ipv6->next_layer(), ip::IpProtocol::UDP);
    ASSERT_EQ(hdr.l3.ipv6->source()[15], 1);
    ASSERT_EQ(hdr.l4.source(), 6082);
    ASSERT_EQ(hdr.l4.destination(), 6081);
    ASSERT_EQ(hdr.l4.length(), 128);
    ASSERT_EQ(hdr.l4.checksum(), 0xffff);
    ASSERT_TRUE(!mystack.last_chunk.has_value());
    ASSERT_EQ(mystack.data.size(), 1u);
    ASSERT_EQ(mystack.data[0].size(), 128u);
    ASSERT_TRUE(std::all_of(mystack.data[0].begin(), mystack.data[0].end(),
                            [](uint8_t v) { return v == 0xaa; }));
}

// ingot-examples/src/tests.rs:277-305 (the parse_read half)
TEST(chunks_present_on_early_accept_read) {
    std::vector<uint8_t> eth = {0xA8, 0x40, 0x25, 0x77, 0x77, 0x76, 0xA8,
                                0x40, 0x25, 0x77, 0x77, 0x77, 0x08, 0x06};
    std::vector<uint8_t> rest = {0, 1, 2, 3, 4, 5, 6, 7};
    auto res = GenericUlp::parse_read({eth, rest});
    auto& parsed = res.unwrap();
    ASSERT_TRUE(parsed.last_chunk.has_value());
    ASSERT_EQ(parsed.last_chunk->size(), 8u);
    ASSERT_EQ(parsed.data.size(), 0u);
}

// ingot-examples/src/tests.rs:381-423
TEST(straddle_failure) {
    const auto v = would_be_valid();
    const std::vector<uint8_t> a(v.begin(), v.begin() + 16), b(v.begin() + 16, v.end());
    auto e = GenericUlp::parse_read({a, b}).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::StraddledHeader);
    ASSERT_EQ(std::string(e.header()), "inner_l3");
    e = GenericUlp::parse_read({a}).unwrap_err();
    ASSERT_EQ(e.error(), ParseError::TooSmall);
    ASSERT_EQ(std::string(e.header()), "inner_l3");
}

// ingot-examples/benches/packet.rs:15-35 (pkt_body_v4) and :139-145
// (parse-and-decr-v4: l4.set_destination(l4.destination() - 1)), over a batch.
static std::vector<uint8_t> pkt_body_v4() {
    std::vector<uint8_t> f(14, 0);
    for (int i = 6; i < 12; ++i) f[i] = 0xff;
    f[12] = 0x08;
    const uint8_t v4[20] = {0x45, 0, 0, 28 + 8, 0, 0, 0, 0, 0xf0, 0x11, 0, 0,
                            192, 168, 0, 1, 192, 168, 0, 255};
    const uint8_t udp[8] = {0x00, 0x80, 0x17, 0xc1, 0x00, 0x08, 0x00, 0x00};
    f.insert(f.end(), v4, v4 + 20);
    f.insert(f.end(), udp, udp + 8);
    for (uint8_t b = 0; b < 8; ++b) f.push_back(b);
    return f;
}

TEST(parse_and_decr_v4) {
    const auto f = pkt_body_v4();
    std::vector<std::vector<uint8_t>> batch(1000, f);
    auto out = gpu::modify_batch(
        gpu::default_context(), batch, UdpParser::CHAIN,
        {gpu::edit(UdpParser::L4_LAYER, INGOT_F_UDP_DESTINATION, INGOT_OP_SUB, 1)});
    ASSERT_EQ(out.size(), 1000u);
    for (const auto& m : out) {
        ASSERT_EQ((int)m.rec.status, (int)INGOT_OK);
        auto [h, hint, rest] = UdpParser::parse(m.frame).unwrap();
        (void)hint;
        (void)rest;
        ASSERT_EQ(h.l4.destination(), 0x17c0);
        ASSERT_EQ(h.l4.source(), 0x0080);
        std::vector<uint8_t> want = f;
        want[37] = 0xc0;
        ASSERT_EQ(m.frame, want);
    }
}

// ingot/src/tests.rs:223-294 — setting each bitfield of the IPv6 header to
// the value it already holds (cumulatively, iterations 0..4) leaves every
// other field, and the bytes, unchanged.
TEST(bitset_fields_do_not_disturb_neighbours) {
    const uint8_t golden[4] = {0x6A, 0x61, 0xe2, 0x40};
    const uint8_t v6[40] = {0x6A, 0x61, 0xe2, 0x40, 0x00, 0x10, 0x11, 0xf0,
                            0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01,
                            0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x02,
                            0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01,
                            0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x01};
    std::vector<uint8_t> pkt(14, 0);
    put16(pkt, 12, ethernet::Ethertype::IPV6);
    pkt.insert(pkt.end(), v6, v6 + 40);
    pkt.insert(pkt.end(), {0, 7, 0, 9, 0, 8, 0, 0});  // UDP (v6 next_header 0x11)
    const uint8_t L = UdpParser::L3_LAYER;
    const std::vector<ingot_edit> setters = {
        gpu::edit(L, INGOT_F_V6_VERSION, INGOT_OP_SET, 6),
        gpu::edit(L, INGOT_F_V6_DSCP, INGOT_OP_SET, 41),
        gpu::edit(L, INGOT_F_V6_ECN, INGOT_OP_SET, (uint32_t)ip::Ecn::Capable1),
        gpu::edit(L, INGOT_F_V6_FLOW_LABEL, INGOT_OP_SET, 123456),
    };
    for (size_t i = 0; i < 5; ++i) {
        std::vector<ingot_edit> upto(setters.begin(), setters.begin() + (i ? i : 0));
        auto m = gpu::modify_batch(gpu::default_context(), {pkt}, UdpParser::CHAIN, upto)[0];
        auto [h, hint, rest] = UdpParser::parse(m.frame).unwrap();
        (void)hint;
        (void)rest;
        ASSERT_TRUE(h.l3.ipv6.has_value());
        ASSERT_EQ(h.l3.ipv6->version(), 6);
        ASSERT_EQ(h.l3.ipv6->dscp(), 41);
        ASSERT_EQ(h.l3.ipv6->ecn(), ip::Ecn::Capable1);
        ASSERT_EQ(h.l3.ipv6->flow_label(), 123456u);
        for (int k = 0; k < 4; ++k) ASSERT_EQ(m.frame[14 + k], golden[k]);
        ASSERT_EQ(m.frame, pkt);
    }
}

// ingot-examples/src/tests.rs:189-268: the reference tunnel frame's outer
// stack emitted in front of its inner frame (batched, with OPTE's per-packet
// setters) parses back as GeneveOverV6Tunnel with those values.
TEST(encapsulate_and_parse_back) {
    static const uint8_t frame[] = {
        0xA8, 0x40, 0x25, 0x77, 0x77, 0x76, 0xA8, 0x40, 0x25, 0x77, 0x77, 0x77, 0x86, 0xDD,
        0x60, 0x00, 0x00, 0x00, 0x00, 0x10, 0x11, 0xF0,
        0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01, 0, 0, 0, 0, 0, 0, 0, 0x02,
        0xFD, 0x00, 0x00, 0x00, 0x00, 0xF7, 0x01, 0x01, 0, 0, 0, 0, 0, 0, 0, 0x01,
        0x1E, 0x61, 0x17, 0xC1, 0x00, 0x14, 0x00, 0x00,
        0x01, 0x00, 0x65, 0x58, 0x00, 0x04, 0xD2, 0x00, 0x01, 0x29, 0x00, 0x00,
        0xAA, 0x00, 0x04, 0x00, 0xFF, 0x10, 0xAA, 0x00, 0x04, 0x00, 0xFF, 0x01, 0x08, 0x00,
        0x45, 0x00, 0x00, 36, 0x00, 0x00, 0x00, 0x00, 0xF0, 0x11, 0x00, 0x00,
        8, 8, 8, 8, 192, 168, 0, 5,
        0x00, 0x80, 0x00, 53, 0x00, 0x08, 0x00, 0x00, 0, 1, 2, 3, 4, 5, 6, 7};
    const std::vector<uint8_t> hdr(frame, frame + 74), inner(frame + 74, frame + sizeof(frame));
    std::vector<std::vector<uint8_t>> payloads;
    std::vector<uint32_t> ports, vnis;
    for (uint32_t i = 0; i < 300; ++i) {
        payloads.push_back(inner);
        payloads.back().resize(inner.size() + i % 37, (uint8_t)i);  // varied lengths
        ports.push_back(0xC000 | i);
        vnis.push_back(0x100000 + i);
    }
    auto pkts = gpu::emit_batch(
        gpu::default_context(), hdr,
        {{14, INGOT_F_V6_PAYLOAD_LEN, INGOT_EMIT_LENGTH, -40, {}},
         {54, INGOT_F_UDP_LENGTH, INGOT_EMIT_LENGTH, 0, {}},
         {54, INGOT_F_UDP_SOURCE, INGOT_EMIT_U16, 0, ports},
         {62, INGOT_F_GENEVE_VNI, INGOT_EMIT_U32, 0, vnis}},
        payloads);
    for (uint32_t i = 0; i < 300; ++i) {
        const auto& p = pkts[i];
        ASSERT_EQ(p.size(), 74 + payloads[i].size());
        ASSERT_TRUE(std::equal(payloads[i].begin(), payloads[i].end(), p.begin() + 74));
        auto [h, hint, rest] = GeneveOverV6Tunnel::parse(p).unwrap();
        (void)hint;
        (void)rest;
        ASSERT_EQ(h.outer_v6.payload_len(), (uint16_t)(p.size() - 54));
        ASSERT_EQ(h.outer_udp.length(), (uint16_t)(p.size() - 54));
        ASSERT_EQ(h.outer_udp.source(), (uint16_t)(0xC000 | i));
        ASSERT_EQ(h.outer_encap.vni(), 0x100000u + i);
        ASSERT_EQ(h.outer_udp.destination(), 6081);
    }
}

int main() {
    for (auto& [name, fn] : registry()) {
        ++g_run;
        try {
            fn();
            std::printf("ok   %s\n", name);
        } catch (const std::exception& e) {
            ++g_failed;
            std::printf("FAIL %s: %s\n", name, e.what());
        }
    }
    std::printf("%d run, %d failed\n", g_run, g_failed);
    return g_failed ? 1 : 0;
}
