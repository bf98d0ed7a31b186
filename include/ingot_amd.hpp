// ingot_amd.hpp — C++17 host-side mirror of ingot's parse interface, over the
// C ABI in ingot_gpu.h.  Header-only; link libingot_gpu.so and amdhip64.
//
// The reference (Rust) exposes, per `#[derive(Parse)]` chain,
//   Chain::parse(slice) -> Result<(Chain, Option<Hint>, Remainder), PacketParseError>
// (ingot-macros/src/parse.rs:475-509, ingot-types/src/lib.rs:137-147, 208),
// with one view per layer whose generated getters read the wire fields
// (packet/mod.rs:1183-1479), and `PacketParseError{label, inner}`
// (ingot-types/src/error.rs:119-171).  This header keeps those names and
// meanings — UdpParser / GenericUlp (ingot-examples/src/packets.rs:18-24,
// 54-60), ValidEthernet / ValidIpv4 / ValidIpv6 / ValidTcp / ValidUdp getters,
// ParseError / PacketParseError — but every parse runs on the GPU: a
// `gpu::BatchParser` uploads frames, runs the batched kernels and hands back
// per-packet results.  `Chain::parse(bytes)` is the one-packet convenience
// form (a batch of one), for tests that read like the reference's.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <tuple>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "ingot_gpu.h"

namespace ingot {

// ---------------------------------------------------------------------------
// ingot_types::{ParseError, PacketParseError} (error.rs:21-44, 119-171)
// ---------------------------------------------------------------------------
namespace types {

enum class ParseError : uint8_t {
    Unwanted = INGOT_ERR_UNWANTED,
    NeedsHint = INGOT_ERR_NEEDS_HINT,
    TooSmall = INGOT_ERR_TOO_SMALL,
    StraddledHeader = INGOT_ERR_STRADDLED_HEADER,
    NoRemainingChunks = INGOT_ERR_NO_REMAINING_CHUNKS,
    CannotAccept = INGOT_ERR_CANNOT_ACCEPT,
    Reject = INGOT_ERR_REJECT,
    IllegalValue = INGOT_ERR_ILLEGAL_VALUE,
};

inline const char* as_cstr(ParseError e) { return ingot_parse_error_name((int)e); }

class PacketParseError {
   public:
    PacketParseError(const char* label, ParseError inner) : label_(label), inner_(inner) {}
    const char* header() const { return label_; }  // the failing layer's label
    ParseError error() const { return inner_; }
    std::string to_string() const { return std::string(label_) + ": " + as_cstr(inner_); }

   private:
    const char* label_;
    ParseError inner_;
};

// Result<T, PacketParseError>
template <class T>
class ParseResult {
   public:
    static ParseResult ok(T v) { return ParseResult(std::move(v)); }
    static ParseResult err(PacketParseError e) { return ParseResult(e); }
    bool is_ok() const { return value_.has_value(); }
    bool is_err() const { return !is_ok(); }
    T& unwrap() {
        if (!value_) throw std::runtime_error("unwrap on Err: " + error_->to_string());
        return *value_;
    }
    const PacketParseError& unwrap_err() const {
        if (!error_) throw std::runtime_error("unwrap_err on Ok");
        return *error_;
    }

   private:
    explicit ParseResult(T v) : value_(std::move(v)) {}
    explicit ParseResult(PacketParseError e) : error_(e) {}
    std::optional<T> value_;
    std::optional<PacketParseError> error_;
};

}  // namespace types

using MacAddr6 = std::array<uint8_t, 6>;
using Ipv4Addr = std::array<uint8_t, 4>;
using Ipv6Addr = std::array<uint8_t, 16>;

namespace ethernet {
// ingot/src/ethernet.rs:9-20
struct Ethertype {
    uint16_t v;
    static constexpr uint16_t IPV4 = 0x0800, ARP = 0x0806, ETHERNET = 0x6558, VLAN = 0x8100,
                              IPV6 = 0x86dd, LLDP = 0x88cc, QINQ = 0x9100;
};
}  // namespace ethernet

namespace ip {
// ingot/src/ip.rs:20-38, 95-135
struct IpProtocol {
    static constexpr uint8_t ICMP = 1, IGMP = 2, TCP = 6, UDP = 17, ICMP_V6 = 58,
                             IPV6_NO_NH = 59, IPV6_HOP_BY_HOP = 0, IPV6_ROUTE = 43,
                             IPV6_FRAGMENT = 44, IPV6_DEST_OPTS = 60, IPV6_EXPERIMENT0 = 253,
                             IPV6_EXPERIMENT1 = 254;
};
enum class Ecn : uint8_t { NotCapable = 0, Capable0 = 1, Capable1 = 2, CongestionExperienced = 3 };
}  // namespace ip

// ---------------------------------------------------------------------------
// Layer views: the generated getters (values from the device field block).
// ---------------------------------------------------------------------------
namespace detail {
template <size_t N>
std::array<uint8_t, N> arr(const uint8_t* p) {
    std::array<uint8_t, N> a{};
    std::memcpy(a.data(), p, N);
    return a;
}
}  // namespace detail

class ValidEthernet {
   public:
    explicit ValidEthernet(const ingot_fields* f)
        : dst_(f->eth_destination), src_(f->eth_source), et_(f->eth_ethertype) {}
    // GeneveOverV6Tunnel's outer_eth
    explicit ValidEthernet(const ingot_tunnel_fields* t)
        : dst_(t->outer_eth_destination), src_(t->outer_eth_source), et_(t->outer_eth_ethertype) {}
    MacAddr6 destination() const { return detail::arr<6>(dst_); }
    MacAddr6 source() const { return detail::arr<6>(src_); }
    uint16_t ethertype() const { return et_; }

   private:
    const uint8_t* dst_;
    const uint8_t* src_;
    uint16_t et_;
};

class ValidVlanBody {
   public:
    ValidVlanBody(const ingot_fields* f, int i) : f_(f), i_(i) {}
    uint8_t priority() const { return f_->vlan_priority[i_]; }
    uint8_t dei() const { return f_->vlan_dei[i_]; }
    uint16_t vid() const { return f_->vlan_vid[i_]; }
    uint16_t ethertype() const { return f_->vlan_ethertype[i_]; }

   private:
    const ingot_fields* f_;
    int i_;
};

class ValidIpv4 {
   public:
    ValidIpv4(const ingot_fields* f, const std::vector<uint8_t>* frame) : f_(f), frame_(frame) {}
    uint8_t version() const { return f_->v4_version; }
    uint8_t ihl() const { return f_->v4_ihl; }
    uint8_t dscp() const { return f_->v4_dscp; }
    ip::Ecn ecn() const { return (ip::Ecn)f_->v4_ecn; }
    uint16_t total_len() const { return f_->v4_total_len; }
    uint16_t identification() const { return f_->v4_identification; }
    uint8_t flags() const { return f_->v4_flags; }
    uint16_t fragment_offset() const { return f_->v4_fragment_offset; }
    uint8_t hop_limit() const { return f_->v4_hop_limit; }
    uint8_t protocol() const { return f_->v4_protocol; }
    uint16_t checksum() const { return f_->v4_checksum; }
    Ipv4Addr source() const { return detail::arr<4>(f_->v4_source); }
    Ipv4Addr destination() const { return detail::arr<4>(f_->v4_destination); }
    std::vector<uint8_t> options_ref() const {
        auto b = frame_->begin() + f_->v4_options_off;
        return std::vector<uint8_t>(b, b + f_->v4_options_len);
    }
    uint8_t next_layer() const { return f_->v4_protocol; }

   private:
    const ingot_fields* f_;
    const std::vector<uint8_t>* frame_;
};

class ValidIpv6 {
   public:
    ValidIpv6(const ingot_fields* f, uint8_t hint) : f_(f), hint_(hint) {}
    uint8_t version() const { return f_->v6_version; }
    uint8_t dscp() const { return f_->v6_dscp; }
    ip::Ecn ecn() const { return (ip::Ecn)f_->v6_ecn; }
    uint32_t flow_label() const { return f_->v6_flow_label; }
    uint16_t payload_len() const { return f_->v6_payload_len; }
    uint8_t next_header() const { return f_->v6_next_header; }
    uint8_t hop_limit() const { return f_->v6_hop_limit; }
    Ipv6Addr source() const { return detail::arr<16>(f_->v6_source); }
    Ipv6Addr destination() const { return detail::arr<16>(f_->v6_destination); }
    // next_layer(): the last extension header's next_header (ip.rs:180-181)
    uint8_t next_layer() const { return hint_; }
    size_t extension_header_count() const { return f_->rec.n_v6ext; }
    const ingot_v6eh& extension_header(size_t i) const { return f_->v6_eh[i]; }

   private:
    const ingot_fields* f_;
    uint8_t hint_;
};

class ValidTcp {
   public:
    ValidTcp(const ingot_fields* f, const std::vector<uint8_t>* frame) : f_(f), frame_(frame) {}
    uint16_t source() const { return f_->l4_source; }
    uint16_t destination() const { return f_->l4_destination; }
    uint32_t sequence() const { return f_->tcp_sequence; }
    uint32_t acknowledgement() const { return f_->tcp_acknowledgement; }
    uint8_t data_offset() const { return f_->tcp_data_offset; }
    uint8_t flags() const { return f_->tcp_flags; }
    uint16_t window_size() const { return f_->tcp_window_size; }
    uint16_t checksum() const { return f_->tcp_checksum; }
    uint16_t urgent_ptr() const { return f_->tcp_urgent_ptr; }
    std::vector<uint8_t> options_ref() const {
        auto b = frame_->begin() + f_->tcp_options_off;
        return std::vector<uint8_t>(b, b + f_->tcp_options_len);
    }

   private:
    const ingot_fields* f_;
    const std::vector<uint8_t>* frame_;
};

class ValidUdp {
   public:
    explicit ValidUdp(const ingot_fields* f)
        : src_(f->l4_source), dst_(f->l4_destination), len_(f->udp_length),
          csum_(f->udp_checksum) {}
    // GeneveOverV6Tunnel's outer_udp
    explicit ValidUdp(const ingot_tunnel_fields* t)
        : src_(t->outer_udp_source), dst_(t->outer_udp_destination), len_(t->outer_udp_length),
          csum_(t->outer_udp_checksum) {}
    uint16_t source() const { return src_; }
    uint16_t destination() const { return dst_; }
    uint16_t length() const { return len_; }
    uint16_t checksum() const { return csum_; }

   private:
    uint16_t src_, dst_, len_, csum_;
};

// GeneveOverV6Tunnel's outer_v6 (ingot/src/ip.rs:159-182 getters).
class ValidOuterIpv6 {
   public:
    explicit ValidOuterIpv6(const ingot_tunnel_fields* t) : t_(t) {}
    uint8_t version() const { return t_->outer_v6_version; }
    uint8_t dscp() const { return t_->outer_v6_dscp; }
    ip::Ecn ecn() const { return (ip::Ecn)t_->outer_v6_ecn; }
    uint32_t flow_label() const { return t_->outer_v6_flow_label; }
    uint16_t payload_len() const { return t_->outer_v6_payload_len; }
    uint8_t next_header() const { return t_->outer_v6_next_header; }
    uint8_t hop_limit() const { return t_->outer_v6_hop_limit; }
    Ipv6Addr source() const { return detail::arr<16>(t_->outer_v6_source); }
    Ipv6Addr destination() const { return detail::arr<16>(t_->outer_v6_destination); }
    uint8_t next_layer() const { return t_->outer_l4_proto; }
    size_t extension_header_count() const { return t_->outer_v6_n_ext; }

   private:
    const ingot_tunnel_fields* t_;
};

// ingot::geneve::GeneveOpt (geneve.rs:80-102) with its data bytes.
struct GeneveOpt {
    uint16_t class_;
    uint8_t option_type;
    uint8_t reserved;
    uint8_t length;
    std::vector<uint8_t> data;
    bool is_critical() const { return (option_type >> 7) == 1; }
};

// ingot::geneve::ValidGeneve getters (geneve.rs:16-44).
class ValidGeneve {
   public:
    ValidGeneve(const ingot_tunnel_fields* t, const std::vector<uint8_t>* frame)
        : t_(t), frame_(frame) {}
    uint8_t version() const { return t_->geneve_version; }
    uint8_t opt_len() const { return t_->geneve_opt_len; }
    uint8_t flags() const { return t_->geneve_flags; }
    uint16_t protocol_type() const { return t_->geneve_protocol_type; }
    uint32_t vni() const { return t_->geneve_vni; }
    uint8_t reserved() const { return t_->geneve_reserved; }
    size_t packet_length() const { return 8u + 4u * t_->geneve_opt_len; }
    std::vector<uint8_t> options_ref() const {
        auto b = frame_->begin() + t_->geneve_off + 8;
        return std::vector<uint8_t>(b, b + 4 * t_->geneve_opt_len);
    }
    size_t option_count() const { return t_->geneve_n_opts; }
    // the first INGOT_MAX_GENEVE_OPT_FIELDS options
    std::vector<GeneveOpt> options() const {
        std::vector<GeneveOpt> out;
        const size_t n = option_count() < INGOT_MAX_GENEVE_OPT_FIELDS ? option_count()
                                                                      : INGOT_MAX_GENEVE_OPT_FIELDS;
        for (size_t i = 0; i < n; ++i) {
            const ingot_geneve_opt& g = t_->geneve_opt[i];
            auto b = frame_->begin() + g.data_off;
            out.push_back(GeneveOpt{g.opt_class, g.option_type, g.reserved, g.length,
                                    std::vector<uint8_t>(b, b + 4 * g.length)});
        }
        return out;
    }

   private:
    const ingot_tunnel_fields* t_;
    const std::vector<uint8_t>* frame_;
};

// L3 choice (ingot-examples/src/choices.rs:17-21) and L4 / Ulp choices.
struct L3 {
    std::optional<ValidIpv4> ipv4;
    std::optional<ValidIpv6> ipv6;
};
struct L4 {
    std::optional<ValidTcp> tcp;
    std::optional<ValidUdp> udp;
    bool icmpv4 = false, icmpv6 = false;
};

// One parsed packet: owns its frame bytes and device field block so the views
// stay valid.
struct Packet {
    std::vector<uint8_t> frame;
    ingot_fields fields;
    ingot_tunnel_fields outer;  // GENEVE_OVER_V6 only (zero otherwise)
};

namespace gpu {

inline void check(int rc, const char* what) {
    if (rc != INGOT_GPU_SUCCESS)
        throw std::runtime_error(std::string(what) + ": " + ingot_gpu_strerror(rc));
}
inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class Context {
   public:
    explicit Context(int device = 0) { check(ingot_gpu_ctx_create(device, &h_), "ctx_create"); }
    ~Context() { ingot_gpu_ctx_destroy(h_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    ingot_gpu_ctx* get() const { return h_; }

   private:
    ingot_gpu_ctx* h_ = nullptr;
};

// Config 5's reduce: one rank's RCCL communicator (ingot_gpu_comm_*).  Rank 0
// calls Comm::unique_id() and the host carries the bytes to every rank;
// allreduce_hist sums a device histogram (bins x u32) over the ranks on
// `stream`, after the work already enqueued there.
class Comm {
   public:
    using Id = std::array<uint8_t, INGOT_COMM_ID_BYTES>;
    static Id unique_id() {
        Id id{};
        check(ingot_gpu_comm_unique_id(id.data()), "comm_unique_id");
        return id;
    }
    Comm(Context& ctx, int nranks, int rank, const Id& id) {
        check(ingot_gpu_comm_create(ctx.get(), nranks, rank, id.data(), &h_), "comm_create");
    }
    // The host's own RCCL communicator (an ncclComm_t), borrowed: it stays
    // the host's and must outlive this object.
    Comm(Context& ctx, void* nccl_comm) {
        check(ingot_gpu_comm_wrap(ctx.get(), nccl_comm, &h_), "comm_wrap");
    }
    ~Comm() {
        if (h_) (void)ingot_gpu_comm_destroy(h_);
    }
    Comm(const Comm&) = delete;
    Comm& operator=(const Comm&) = delete;
    int size() const { return ingot_gpu_comm_size(h_); }
    int rank() const { return ingot_gpu_comm_rank(h_); }
    void allreduce_hist(uint32_t* d_hist, uint32_t bins, hipStream_t stream = nullptr) {
        check(ingot_gpu_flow_hist_allreduce(h_, d_hist, bins, stream), "flow_hist_allreduce");
    }

   private:
    ingot_gpu_comm* h_ = nullptr;
};

// Uploads host frames into a packed device arena, runs the records + field
// kernels for `chain`, copies the per-packet field blocks back.
inline std::vector<Packet> parse_batch(Context& ctx, const std::vector<std::vector<uint8_t>>& frames,
                                       int chain) {
    const size_t n = frames.size();
    std::vector<uint64_t> off(n);
    std::vector<uint16_t> len(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        if (frames[i].size() > 65535) throw std::length_error("frame longer than 65535 bytes");
        off[i] = total;
        len[i] = (uint16_t)frames[i].size();
        total += (frames[i].size() + 15) / 16 * 16 + 16;
    }
    std::vector<uint8_t> arena(total + 64, 0);
    for (size_t i = 0; i < n; ++i)
        if (!frames[i].empty()) std::memcpy(arena.data() + off[i], frames[i].data(), frames[i].size());
    uint8_t* d_arena = nullptr;
    uint64_t* d_off = nullptr;
    uint16_t* d_len = nullptr;
    const bool tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    const size_t blk = tun ? sizeof(ingot_geneve_fields) : sizeof(ingot_fields);
    uint8_t* d_f = nullptr;
    hip_check(hipMalloc(&d_arena, arena.size()), "hipMalloc");
    hip_check(hipMalloc(&d_off, n * 8 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_len, n * 2 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_f, n * blk + 512), "hipMalloc");
    hip_check(hipMemcpy(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_len, len.data(), n * 2, hipMemcpyHostToDevice), "H2D");
    if (tun)
        check(ingot_gpu_geneve_fields(ctx.get(), d_arena, d_off, d_len, 0, n,
                                      reinterpret_cast<ingot_geneve_fields*>(d_f), nullptr),
              "ingot_gpu_geneve_fields");
    else
        check(ingot_gpu_fields(ctx.get(), d_arena, d_off, d_len, 0, n, chain,
                               reinterpret_cast<ingot_fields*>(d_f), nullptr),
              "ingot_gpu_fields");
    std::vector<Packet> out(n);
    std::vector<uint8_t> f(n * blk);
    hip_check(hipMemcpy(f.data(), d_f, n * blk, hipMemcpyDeviceToHost), "D2H");
    for (size_t i = 0; i < n; ++i) {
        out[i].frame = frames[i];
        std::memcpy(&out[i].fields, f.data() + i * blk, sizeof(ingot_fields));
        if (tun)
            std::memcpy(&out[i].outer, f.data() + i * blk + sizeof(ingot_fields),
                        sizeof(ingot_tunnel_fields));
        else
            std::memset(&out[i].outer, 0, sizeof(ingot_tunnel_fields));
    }
    (void)hipFree(d_arena);
    (void)hipFree(d_off);
    (void)hipFree(d_len);
    (void)hipFree(d_f);
    return out;
}

// parse_read over chunk lists: packet i = chunks[i] (a `Read` of byte chunks,
// ingot-types/src/lib.rs:151-166).  The Packet's frame is the chunks
// concatenated (record offsets are logical); `chunk` = the chunk holding the
// remainder; `ends` = each chunk's logical end.
using Chunks = std::vector<std::vector<uint8_t>>;
struct ReadResult {
    Packet pkt;
    uint16_t chunk;
    std::vector<size_t> ends;
};

inline std::vector<ReadResult> parse_read_batch(Context& ctx, const std::vector<Chunks>& packets,
                                                int chain) {
    const size_t n = packets.size();
    std::vector<uint64_t> seg_off;
    std::vector<uint16_t> seg_len;
    std::vector<uint32_t> pkt_seg{0};
    std::vector<uint8_t> arena;
    for (const auto& chunks : packets) {
        for (const auto& c : chunks) {
            if (c.size() > 65535) throw std::length_error("chunk longer than 65535 bytes");
            seg_off.push_back(arena.size());
            seg_len.push_back((uint16_t)c.size());
            arena.insert(arena.end(), c.begin(), c.end());
            arena.resize((arena.size() + 15) / 16 * 16 + 16, 0);  // chunks apart in memory
        }
        pkt_seg.push_back((uint32_t)seg_off.size());
    }
    seg_off.push_back(arena.size());  // keeps the tables non-empty
    seg_len.push_back(0);
    arena.resize(arena.size() + 64, 0);
    const bool tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    const size_t blk = tun ? sizeof(ingot_geneve_fields) : sizeof(ingot_fields);
    uint8_t *d_arena = nullptr, *d_f = nullptr;
    uint64_t* d_off = nullptr;
    uint16_t *d_len = nullptr, *d_chunk = nullptr;
    uint32_t* d_ps = nullptr;
    hip_check(hipMalloc(&d_arena, arena.size()), "hipMalloc");
    hip_check(hipMalloc(&d_off, seg_off.size() * 8), "hipMalloc");
    hip_check(hipMalloc(&d_len, seg_len.size() * 2), "hipMalloc");
    hip_check(hipMalloc(&d_ps, pkt_seg.size() * 4), "hipMalloc");
    hip_check(hipMalloc(&d_f, n * blk + 512), "hipMalloc");
    hip_check(hipMalloc(&d_chunk, n * 2 + 8), "hipMalloc");
    hip_check(hipMemcpy(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_off, seg_off.data(), seg_off.size() * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_len, seg_len.data(), seg_len.size() * 2, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_ps, pkt_seg.data(), pkt_seg.size() * 4, hipMemcpyHostToDevice), "H2D");
    if (tun)
        check(ingot_gpu_geneve_fields_read(ctx.get(), d_arena, d_off, d_len, d_ps, n,
                                           reinterpret_cast<ingot_geneve_fields*>(d_f), d_chunk,
                                           nullptr),
              "ingot_gpu_geneve_fields_read");
    else
        check(ingot_gpu_fields_read(ctx.get(), d_arena, d_off, d_len, d_ps, n, chain,
                                    reinterpret_cast<ingot_fields*>(d_f), d_chunk, nullptr),
              "ingot_gpu_fields_read");
    std::vector<uint8_t> f(n * blk);
    std::vector<uint16_t> chunk(n);
    hip_check(hipMemcpy(f.data(), d_f, n * blk, hipMemcpyDeviceToHost), "D2H");
    hip_check(hipMemcpy(chunk.data(), d_chunk, n * 2, hipMemcpyDeviceToHost), "D2H");
    std::vector<ReadResult> out(n);
    for (size_t i = 0; i < n; ++i) {
        ReadResult& r = out[i];
        for (const auto& c : packets[i]) {
            r.pkt.frame.insert(r.pkt.frame.end(), c.begin(), c.end());
            r.ends.push_back(r.pkt.frame.size());
        }
        std::memcpy(&r.pkt.fields, f.data() + i * blk, sizeof(ingot_fields));
        if (tun)
            std::memcpy(&r.pkt.outer, f.data() + i * blk + sizeof(ingot_fields),
                        sizeof(ingot_tunnel_fields));
        else
            std::memset(&r.pkt.outer, 0, sizeof(ingot_tunnel_fields));
        r.chunk = chunk[i];
    }
    for (void* p : {(void*)d_arena, (void*)d_off, (void*)d_len, (void*)d_ps, (void*)d_f,
                    (void*)d_chunk})
        (void)hipFree(p);
    return out;
}

// ingot's generated setters (`set_<field>`, packet/mod.rs:2097-2255; BE
// bitfield set paths, bitfield.rs:188-315), batched: every frame is parsed as
// `chain` and, when Ok, the edit list is applied in order in place
// (ingot_gpu_parse_modify).  Returns the rewritten frames and their records.
inline ingot_edit edit(uint8_t layer, int field, int op, uint32_t value, uint8_t index = 0) {
    ingot_edit e;
    e.layer = layer;
    e.field = (uint8_t)field;
    e.op = (uint8_t)op;
    e.index = index;
    e.value = value;
    return e;
}

struct Modified {
    std::vector<uint8_t> frame;
    ingot_rec rec;
};

inline std::vector<Modified> modify_batch(Context& ctx,
                                          const std::vector<std::vector<uint8_t>>& frames,
                                          int chain, const std::vector<ingot_edit>& edits) {
    const size_t n = frames.size();
    std::vector<uint64_t> off(n);
    std::vector<uint16_t> len(n);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        if (frames[i].size() > 65535) throw std::length_error("frame longer than 65535 bytes");
        off[i] = total;
        len[i] = (uint16_t)frames[i].size();
        total += (frames[i].size() + 15) / 16 * 16 + 16;
    }
    std::vector<uint8_t> arena(total + 64, 0);
    for (size_t i = 0; i < n; ++i)
        if (!frames[i].empty()) std::memcpy(arena.data() + off[i], frames[i].data(), frames[i].size());
    uint8_t* d_arena = nullptr;
    uint64_t* d_off = nullptr;
    uint16_t* d_len = nullptr;
    ingot_rec* d_rec = nullptr;
    hip_check(hipMalloc(&d_arena, arena.size()), "hipMalloc");
    hip_check(hipMalloc(&d_off, n * 8 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_len, n * 2 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_rec, n * sizeof(ingot_rec) + 16), "hipMalloc");
    hip_check(hipMemcpy(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_len, len.data(), n * 2, hipMemcpyHostToDevice), "H2D");
    check(ingot_gpu_parse_modify(ctx.get(), d_arena, d_off, d_len, 0, n, chain, edits.data(),
                                 (uint32_t)edits.size(), d_rec, nullptr),
          "ingot_gpu_parse_modify");
    std::vector<ingot_rec> rec(n);
    hip_check(hipMemcpy(arena.data(), d_arena, arena.size(), hipMemcpyDeviceToHost), "D2H");
    hip_check(hipMemcpy(rec.data(), d_rec, n * sizeof(ingot_rec), hipMemcpyDeviceToHost), "D2H");
    std::vector<Modified> out(n);
    for (size_t i = 0; i < n; ++i) {
        out[i].frame.assign(arena.begin() + (long)off[i], arena.begin() + (long)(off[i] + len[i]));
        out[i].rec = rec[i];
    }
    for (void* p : {(void*)d_arena, (void*)d_off, (void*)d_len, (void*)d_rec}) (void)hipFree(p);
    return out;
}

// Batched Emit (ingot_gpu_emit_packets): `hdr` = an owned header stack
// emitted once (ingot's emit_vec on the host), the setters applied per packet
// (values per packet for INGOT_EMIT_U16 / U32 sources), then each payload.
// Returns the emitted packets.
struct EmitSet {
    uint16_t at;
    int field;
    int source;
    int32_t add;
    std::vector<uint32_t> values;  // U16 / U32 sources: one per payload
};

inline std::vector<std::vector<uint8_t>> emit_batch(Context& ctx, const std::vector<uint8_t>& hdr,
                                                    const std::vector<EmitSet>& sets,
                                                    const std::vector<std::vector<uint8_t>>& payloads) {
    const size_t n = payloads.size();
    std::vector<uint64_t> off(n), doff(n);
    std::vector<uint16_t> len(n);
    size_t total = 0, dtotal = 0;
    for (size_t i = 0; i < n; ++i) {
        if (payloads[i].size() + hdr.size() > 65535) throw std::length_error("packet too long");
        off[i] = total;
        doff[i] = dtotal;
        len[i] = (uint16_t)payloads[i].size();
        total += (payloads[i].size() + 15) / 16 * 16 + 16;
        dtotal += hdr.size() + payloads[i].size();
    }
    std::vector<uint8_t> arena(total + 64, 0), out(dtotal + 64, 0);
    for (size_t i = 0; i < n; ++i)
        if (!payloads[i].empty()) std::memcpy(arena.data() + off[i], payloads[i].data(), payloads[i].size());
    uint8_t *d_arena = nullptr, *d_dst = nullptr;
    uint64_t *d_off = nullptr, *d_doff = nullptr;
    uint16_t* d_len = nullptr;
    std::vector<void*> d_vals;
    std::vector<ingot_emit_set> es(sets.size());
    hip_check(hipMalloc(&d_arena, arena.size()), "hipMalloc");
    hip_check(hipMalloc(&d_dst, out.size()), "hipMalloc");
    hip_check(hipMalloc(&d_off, n * 8 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_doff, n * 8 + 8), "hipMalloc");
    hip_check(hipMalloc(&d_len, n * 2 + 8), "hipMalloc");
    for (size_t k = 0; k < sets.size(); ++k) {
        const EmitSet& s = sets[k];
        es[k] = ingot_emit_set{s.at, (uint8_t)s.field, (uint8_t)s.source, s.add, nullptr};
        if (s.source == INGOT_EMIT_U16 || s.source == INGOT_EMIT_U32) {
            if (s.values.size() != n) throw std::invalid_argument("one set value per payload");
            void* d = nullptr;
            hip_check(hipMalloc(&d, n * 4 + 8), "hipMalloc");
            if (s.source == INGOT_EMIT_U16) {
                std::vector<uint16_t> v(s.values.begin(), s.values.end());
                hip_check(hipMemcpy(d, v.data(), n * 2, hipMemcpyHostToDevice), "H2D");
            } else {
                hip_check(hipMemcpy(d, s.values.data(), n * 4, hipMemcpyHostToDevice), "H2D");
            }
            es[k].d_values = d;
            d_vals.push_back(d);
        }
    }
    hip_check(hipMemcpy(d_arena, arena.data(), arena.size(), hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_off, off.data(), n * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_doff, doff.data(), n * 8, hipMemcpyHostToDevice), "H2D");
    hip_check(hipMemcpy(d_len, len.data(), n * 2, hipMemcpyHostToDevice), "H2D");
    check(ingot_gpu_emit_packets(ctx.get(), hdr.data(), (uint32_t)hdr.size(), es.data(),
                                 (uint32_t)es.size(), d_arena, d_off, d_len, n, d_dst, d_doff,
                                 nullptr),
          "ingot_gpu_emit_packets");
    hip_check(hipMemcpy(out.data(), d_dst, out.size(), hipMemcpyDeviceToHost), "D2H");
    std::vector<std::vector<uint8_t>> pkts(n);
    for (size_t i = 0; i < n; ++i)
        pkts[i].assign(out.begin() + (long)doff[i],
                       out.begin() + (long)(doff[i] + hdr.size() + len[i]));
    for (void* p : {(void*)d_arena, (void*)d_dst, (void*)d_off, (void*)d_doff, (void*)d_len})
        (void)hipFree(p);
    for (void* p : d_vals) (void)hipFree(p);
    return pkts;
}

inline Context& default_context() {
    static Context ctx(0);
    return ctx;
}

}  // namespace gpu

namespace examples {

template <class Chain>
using Success = std::tuple<Chain, std::optional<uint8_t>, std::vector<uint8_t>>;

// ingot_types::Parsed (parse_read's result, parse.rs:525-535): the headers,
// the chunks not yet read, and the rest of the chunk holding the remainder
// (None when that chunk was consumed exactly).
template <class Chain>
struct Parsed {
    Chain headers;
    gpu::Chunks data;
    std::optional<std::vector<uint8_t>> last_chunk;
};

// Shared by every chain's parse_read: run the batch, build each Ok packet's
// headers with Chain::build, attach Parsed's chunk bookkeeping.
template <class Chain>
std::vector<types::ParseResult<Parsed<Chain>>> parse_read_all(const std::vector<gpu::Chunks>& pk,
                                                              gpu::Context& ctx) {
    std::vector<types::ParseResult<Parsed<Chain>>> out;
    auto res = gpu::parse_read_batch(ctx, pk, Chain::CHAIN);
    for (size_t i = 0; i < res.size(); ++i) {
        auto& r = res[i];
        const ingot_rec rec = r.pkt.fields.rec;
        if (rec.status != INGOT_OK) {
            out.push_back(types::ParseResult<Parsed<Chain>>::err(types::PacketParseError(
                ingot_chain_layer_label(Chain::CHAIN, rec.err_layer),
                (types::ParseError)rec.status)));
            continue;
        }
        const size_t end = r.ends.empty() ? 0 : r.ends[r.chunk];
        std::optional<std::vector<uint8_t>> last;
        if (end > rec.payload_off)
            last = std::vector<uint8_t>(r.pkt.frame.begin() + rec.payload_off,
                                        r.pkt.frame.begin() + end);
        gpu::Chunks data(pk[i].begin() + std::min(pk[i].size(), (size_t)r.chunk + 1),
                         pk[i].end());
        auto sp = std::make_shared<const Packet>(std::move(r.pkt));
        out.push_back(types::ParseResult<Parsed<Chain>>::ok(
            Parsed<Chain>{Chain::build(sp), std::move(data), std::move(last)}));
    }
    return out;
}

namespace detail {
inline types::PacketParseError error_of(int chain, const ingot_rec& r) {
    return types::PacketParseError(ingot_chain_layer_label(chain, r.err_layer),
                                   (types::ParseError)r.status);
}
inline L3 l3_of(const Packet& p) {
    L3 l3;
    if (p.fields.rec.l3_kind == INGOT_L3_IPV4) l3.ipv4.emplace(&p.fields, &p.frame);
    if (p.fields.rec.l3_kind == INGOT_L3_IPV6) l3.ipv6.emplace(&p.fields, p.fields.rec.l4_proto);
    return l3;
}
inline L4 l4_of(const Packet& p) {
    L4 l4;
    switch (p.fields.rec.l4_kind) {
    case INGOT_L4_TCP: l4.tcp.emplace(&p.fields, &p.frame); break;
    case INGOT_L4_UDP: l4.udp.emplace(&p.fields); break;
    case INGOT_L4_ICMPV4: l4.icmpv4 = true; break;
    case INGOT_L4_ICMPV6: l4.icmpv6 = true; break;
    default: break;
    }
    return l4;
}
inline std::vector<uint8_t> remainder(const Packet& p) {
    return std::vector<uint8_t>(p.frame.begin() + p.fields.rec.payload_off, p.frame.end());
}
}  // namespace detail

// ingot-examples/src/packets.rs:18-24 — eth, l3: L3, l4: from L4 -> Udp.
// The Packet is shared so the views outlive the temporary batch.
struct UdpParser {
    static constexpr int CHAIN = INGOT_CHAIN_UDP_PARSER;
    // edit layers = label indices (eth, l3, l4)
    static constexpr uint8_t ETH_LAYER = 0, L3_LAYER = 1, L4_LAYER = 2;
    std::shared_ptr<const Packet> pkt;
    ValidEthernet eth;
    L3 l3;
    ValidUdp l4;

    static std::vector<types::ParseResult<Success<UdpParser>>> parse_all(
        const std::vector<std::vector<uint8_t>>& frames,
        gpu::Context& ctx = gpu::default_context()) {
        std::vector<types::ParseResult<Success<UdpParser>>> out;
        for (auto& p : gpu::parse_batch(ctx, frames, CHAIN)) {
            auto sp = std::make_shared<const Packet>(std::move(p));
            if (sp->fields.rec.status != INGOT_OK) {
                out.push_back(types::ParseResult<Success<UdpParser>>::err(
                    detail::error_of(CHAIN, sp->fields.rec)));
                continue;
            }
            out.push_back(types::ParseResult<Success<UdpParser>>::ok(
                Success<UdpParser>{build(sp), std::nullopt, detail::remainder(*sp)}));
        }
        return out;
    }
    static types::ParseResult<Success<UdpParser>> parse(const std::vector<uint8_t>& frame) {
        return std::move(parse_all({frame})[0]);
    }
    // parse.rs:511-537 over a chunk list
    static types::ParseResult<Parsed<UdpParser>> parse_read(
        const gpu::Chunks& chunks, gpu::Context& ctx = gpu::default_context()) {
        return std::move(parse_read_all<UdpParser>({chunks}, ctx)[0]);
    }
    static UdpParser build(const std::shared_ptr<const Packet>& sp) {
        return UdpParser{sp, ValidEthernet(&sp->fields), detail::l3_of(*sp),
                         ValidUdp(&sp->fields)};
    }
};

// ingot-examples/src/packets.rs:54-60 — inner_eth (control = exit_on_arp),
// inner_l3: Option<L3>, inner_ulp: Option<Ulp>.
struct GenericUlp {
    static constexpr int CHAIN = INGOT_CHAIN_GENERIC_ULP;
    static constexpr uint8_t INNER_ETH_LAYER = 0, INNER_L3_LAYER = 1, INNER_ULP_LAYER = 2;
    std::shared_ptr<const Packet> pkt;
    ValidEthernet inner_eth;
    std::optional<L3> inner_l3;
    std::optional<L4> inner_ulp;

    static std::vector<types::ParseResult<Success<GenericUlp>>> parse_all(
        const std::vector<std::vector<uint8_t>>& frames,
        gpu::Context& ctx = gpu::default_context()) {
        std::vector<types::ParseResult<Success<GenericUlp>>> out;
        for (auto& p : gpu::parse_batch(ctx, frames, CHAIN)) {
            auto sp = std::make_shared<const Packet>(std::move(p));
            if (sp->fields.rec.status != INGOT_OK) {
                out.push_back(types::ParseResult<Success<GenericUlp>>::err(
                    detail::error_of(CHAIN, sp->fields.rec)));
                continue;
            }
            out.push_back(types::ParseResult<Success<GenericUlp>>::ok(
                Success<GenericUlp>{build(sp), std::nullopt, detail::remainder(*sp)}));
        }
        return out;
    }
    static GenericUlp build(const std::shared_ptr<const Packet>& sp) {
        GenericUlp c{sp, ValidEthernet(&sp->fields), std::nullopt, std::nullopt};
        if (!(sp->fields.rec.flags & INGOT_REC_ACCEPTED)) {
            c.inner_l3 = detail::l3_of(*sp);
            c.inner_ulp = detail::l4_of(*sp);
        }
        return c;
    }
    static types::ParseResult<Parsed<GenericUlp>> parse_read(
        const gpu::Chunks& chunks, gpu::Context& ctx = gpu::default_context()) {
        return std::move(parse_read_all<GenericUlp>({chunks}, ctx)[0]);
    }
    static types::ParseResult<Success<GenericUlp>> parse(const std::vector<uint8_t>& frame) {
        return std::move(parse_all({frame})[0]);
    }
    static types::ParseResult<Success<GenericUlp>> parse_slice(const std::vector<uint8_t>& frame) {
        return parse(frame);
    }
};

// ingot-examples/src/packets.rs:27-40 — outer_eth, outer_v6: from L3 -> Ipv6,
// outer_udp: from L4 -> Udp, outer_encap: Geneve, then GenericUlp's layers.
struct GeneveOverV6Tunnel {
    static constexpr int CHAIN = INGOT_CHAIN_GENEVE_OVER_V6;
    static constexpr uint8_t OUTER_ETH_LAYER = 0, OUTER_V6_LAYER = 1, OUTER_UDP_LAYER = 2,
                             OUTER_ENCAP_LAYER = 3, INNER_ETH_LAYER = 4, INNER_L3_LAYER = 5,
                             INNER_ULP_LAYER = 6;
    std::shared_ptr<const Packet> pkt;
    ValidEthernet outer_eth;
    ValidOuterIpv6 outer_v6;
    ValidUdp outer_udp;
    ValidGeneve outer_encap;
    ValidEthernet inner_eth;
    std::optional<L3> inner_l3;
    std::optional<L4> inner_ulp;

    static std::vector<types::ParseResult<Success<GeneveOverV6Tunnel>>> parse_all(
        const std::vector<std::vector<uint8_t>>& frames,
        gpu::Context& ctx = gpu::default_context()) {
        std::vector<types::ParseResult<Success<GeneveOverV6Tunnel>>> out;
        for (auto& p : gpu::parse_batch(ctx, frames, CHAIN)) {
            auto sp = std::make_shared<const Packet>(std::move(p));
            if (sp->fields.rec.status != INGOT_OK) {
                out.push_back(types::ParseResult<Success<GeneveOverV6Tunnel>>::err(
                    detail::error_of(CHAIN, sp->fields.rec)));
                continue;
            }
            out.push_back(types::ParseResult<Success<GeneveOverV6Tunnel>>::ok(
                Success<GeneveOverV6Tunnel>{build(sp), std::nullopt, detail::remainder(*sp)}));
        }
        return out;
    }
    static GeneveOverV6Tunnel build(const std::shared_ptr<const Packet>& sp) {
        GeneveOverV6Tunnel c{sp,
                             ValidEthernet(&sp->outer),
                             ValidOuterIpv6(&sp->outer),
                             ValidUdp(&sp->outer),
                             ValidGeneve(&sp->outer, &sp->frame),
                             ValidEthernet(&sp->fields),
                             std::nullopt,
                             std::nullopt};
        if (!(sp->fields.rec.flags & INGOT_REC_ACCEPTED)) {
            c.inner_l3 = detail::l3_of(*sp);
            c.inner_ulp = detail::l4_of(*sp);
        }
        return c;
    }
    static types::ParseResult<Parsed<GeneveOverV6Tunnel>> parse_read(
        const gpu::Chunks& chunks, gpu::Context& ctx = gpu::default_context()) {
        return std::move(parse_read_all<GeneveOverV6Tunnel>({chunks}, ctx)[0]);
    }
    static types::ParseResult<Success<GeneveOverV6Tunnel>> parse(
        const std::vector<uint8_t>& frame) {
        return std::move(parse_all({frame})[0]);
    }
};

}  // namespace examples
}  // namespace ingot
