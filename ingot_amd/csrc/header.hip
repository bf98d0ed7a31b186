// header.hip — single-header parse, batched (ingot_gpu_parse_header).
//
// `HeaderParse::parse(slice)` of one header kind at the start of every slice
// (ingot-types/src/lib.rs:137-147; generated bodies packet/mod.rs:1831-2005)
// or a choice's `parse_choice(slice, hint)` (ingot-macros/src/choice.rs:
// 231-246).  Not the chain hot path (k_parse): one lane per slice, reads
// straight from L2/HBM, one 8-B ingot_hdr store per lane.  The layer bodies
// follow the same reference lines as walk() in parse.hip.
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "kernels.h"
#include "layouts.h"

namespace ingot_gpu {
namespace {

using namespace layout;

// One lane's slice in global memory: n-byte big-endian reads (n <= 4).
struct Slice {
    const uint8_t* g;
    __device__ __forceinline__ uint32_t be(uint32_t i, uint32_t n) const {
        uint32_t v = 0;
        for (uint32_t k = 0; k < n; ++k) v = (v << 8) | g[i + k];
        return v;
    }
    __device__ __forceinline__ uint32_t get(uint32_t at, Field f) const {
        return (be(at + f.byte0(), f.nbytes()) >> f.rshift()) & f.mask();
    }
};

struct Out {
    uint32_t status = INGOT_OK, kind, used = 0, hint = INGOT_HINT_NONE;
};

// Accessor::read_from_prefix for a fixed-size header (accessor.rs:30-67).
__device__ __forceinline__ void fixed(Out& o, uint32_t len, uint32_t size) {
    if (len < size) o.status = INGOT_ERR_TOO_SMALL;
    else o.used = size;
}

__device__ __forceinline__ void ipv4_body(Out& o, const Slice& s, uint32_t len) {
    // ip.rs:63-93: 20 B, options (ihl*4).saturating_sub(20) (ip.rs:91)
    if (len < ipv4::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
    const uint32_t ihl = s.get(0, ipv4::ihl);
    const uint32_t opt = ihl * 4u > 20u ? ihl * 4u - 20u : 0u;
    if (len - ipv4::LEN < opt) { o.status = INGOT_ERR_TOO_SMALL; return; }
    o.used = ipv4::LEN + opt;
    o.hint = s.get(0, ipv4::protocol);  // next_layer (ip.rs:80-82)
}

__device__ __forceinline__ uint32_t eh_class(uint32_t h) {
    // IpProtocol::class (ip.rs:40-54)
    if (h == 44u) return EH_FRAGMENT;
    const bool r6564 = h == 0u || h == 43u || h == 60u || h == 135u || h == 139u || h == 140u ||
                       h == 253u || h == 254u;
    return r6564 ? EH_RFC6564 : EH_NONE;
}

__device__ __forceinline__ void ipv6_body(Out& o, const Slice& s, uint32_t len) {
    // ip.rs:159-182: 40 B, then Repeated<LowRentV6Eh> over the rest of the
    // slice (util.rs:189-228): Unwanted ends it, other errors are the header's.
    if (len < ipv6::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
    uint32_t h = s.get(0, ipv6::next_header);
    uint32_t q = ipv6::LEN;
    while (q < len) {
        const uint32_t c = eh_class(h);
        if (c == EH_NONE) break;
        uint32_t used;
        if (c == EH_FRAGMENT) {
            if (len - q < v6frag::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
            used = v6frag::LEN;
        } else {
            if (len - q < v6ext6564::FIXED) { o.status = INGOT_ERR_TOO_SMALL; return; }
            used = 8u + 8u * s.get(q, v6ext6564::ext_len);  // ip.rs:209
            if (len - q < used) { o.status = INGOT_ERR_TOO_SMALL; return; }
        }
        h = s.get(q, v6ext6564::next_header);  // both EH kinds start with next_header
        q += used;
    }
    o.used = q;
    o.hint = h;  // the chain's last next_header (ip.rs:180-181)
}

__device__ __forceinline__ void tcp_body(Out& o, const Slice& s, uint32_t len) {
    // tcp.rs:9-30: 20 B, options (data_offset*4).saturating_sub(20) (tcp.rs:28)
    if (len < tcp::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
    const uint32_t doff = s.get(0, tcp::data_offset);
    const uint32_t opt = doff * 4u > 20u ? doff * 4u - 20u : 0u;
    if (len - tcp::LEN < opt) { o.status = INGOT_ERR_TOO_SMALL; return; }
    o.used = tcp::LEN + opt;
}

__device__ __forceinline__ void geneve_body(Out& o, const Slice& s, uint32_t len) {
    // geneve.rs:16-44: 8 B, options split_at(opt_len*4) and subparsed; an
    // option overrunning the span is TooSmall (GeneveOpt never Unwanted).
    if (len < geneve::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
    const uint32_t span = s.get(0, geneve::opt_len) * 4u;
    if (len - geneve::LEN < span) { o.status = INGOT_ERR_TOO_SMALL; return; }
    uint32_t read = 0;
    while (read < span) {
        const uint32_t at = geneve::LEN + read, rem = span - read;
        if (rem < geneve_opt::LEN) { o.status = INGOT_ERR_TOO_SMALL; return; }
        const uint32_t data = s.get(at, geneve_opt::length) * 4u;
        if (rem - geneve_opt::LEN < data) { o.status = INGOT_ERR_TOO_SMALL; return; }
        read += geneve_opt::LEN + data;
    }
    o.used = geneve::LEN + span;
}

__device__ Out parse_one(int kind, const Slice& s, uint32_t len, uint32_t hint) {
    Out o;
    o.kind = (uint32_t)kind;
    switch (kind) {
    case INGOT_HDR_ETHERNET:  // ethernet.rs:46-55
        fixed(o, len, eth::LEN);
        if (!o.status) o.hint = s.get(0, eth::ethertype);
        break;
    case INGOT_HDR_VLAN:  // ethernet.rs:57-65
        fixed(o, len, vlan::LEN);
        if (!o.status) o.hint = s.get(0, vlan::ethertype);
        break;
    case INGOT_HDR_IPV4: ipv4_body(o, s, len); break;
    case INGOT_HDR_IPV6: ipv6_body(o, s, len); break;
    case INGOT_HDR_TCP: tcp_body(o, s, len); break;
    case INGOT_HDR_UDP: fixed(o, len, udp::LEN); break;
    case INGOT_HDR_ICMP: fixed(o, len, icmp::LEN); break;
    case INGOT_HDR_REPEATED_UDP: {
        // RepeatedView::parse_choice over the slice (util.rs:189-228): Udp
        // never returns Unwanted, so a short tail is TooSmall.
        uint32_t read = 0;
        while (read < len) {
            if (len - read < udp::LEN) { o.status = INGOT_ERR_TOO_SMALL; break; }
            read += udp::LEN;
        }
        if (!o.status) o.used = read;
        break;
    }
    case INGOT_HDR_GENEVE: geneve_body(o, s, len); break;
    case INGOT_HDR_L3:  // choices.rs:17-21; choice.rs:231-246
        if (hint == INGOT_HINT_NONE) o.status = INGOT_ERR_NEEDS_HINT;
        else if (hint == ET_IPV4) { o.kind = INGOT_HDR_IPV4; ipv4_body(o, s, len); }
        else if (hint == ET_IPV6) { o.kind = INGOT_HDR_IPV6; ipv6_body(o, s, len); }
        else o.status = INGOT_ERR_UNWANTED;
        break;
    case INGOT_HDR_L4:   // choices.rs:25-29
    case INGOT_HDR_ULP:  // choices.rs:32-38
        if (hint == INGOT_HINT_NONE) o.status = INGOT_ERR_NEEDS_HINT;
        else if (hint == IPP_TCP) { o.kind = INGOT_HDR_TCP; tcp_body(o, s, len); }
        else if (hint == IPP_UDP) { o.kind = INGOT_HDR_UDP; fixed(o, len, udp::LEN); }
        else if (kind == INGOT_HDR_ULP && (hint == IPP_ICMP || hint == IPP_ICMP_V6)) {
            o.kind = INGOT_HDR_ICMP;
            fixed(o, len, icmp::LEN);
        } else o.status = INGOT_ERR_UNWANTED;
        break;
    default: o.status = INGOT_ERR_UNWANTED; break;
    }
    if (o.status) {
        o.used = 0;
        o.hint = INGOT_HINT_NONE;
    }
    return o;
}

__global__ __launch_bounds__(256) void k_header(HeaderArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i >= a.n) return;
    uint64_t off;
    uint32_t len;
    if (a.off) {
        off = a.off[i];
        len = a.len[i];
    } else {
        off = i * a.stride;
        len = a.len ? a.len[i] : a.stride;
        if (len > a.stride) len = a.stride;
    }
    const uint32_t hint = a.hints ? a.hints[i] : a.hint;
    const Out o = parse_one(a.kind, Slice{a.arena + off}, len, hint);
    uint2 w;
    w.x = o.status | (o.kind << 8) | (o.used << 16);
    w.y = o.hint;
    reinterpret_cast<uint2*>(a.out)[i] = w;
}

}  // namespace

hipError_t launch_header(const HeaderArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint64_t blocks = (a.n + 255u) / 256u;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_header, dim3((uint32_t)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace ingot_gpu
