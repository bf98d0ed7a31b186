// walk.h — the device side shared by the parse kernels (parse.hip,
// read.hip, ring.hip): LDS-DMA staging and record stores, the lane's frame
// views (Frame, SegFrameP), the chain walk `walk<CHAIN>()` that
// restates ingot's generated parse_slice / parse_read (see parse.hip's
// header for the reference map), the setters' and the flow hash's helpers,
// and the grid helpers.  Internal; every definition is in an anonymous
// namespace, so each kernel file gets its own copy.
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/ingot_gpu.h"
#include "kernels.h"
#include "layouts.h"

namespace ingot_gpu {
namespace {

using namespace layout;

constexpr uint32_t WAVE = 64;
constexpr uint32_t WAVES = 4;
constexpr uint32_t BLOCK = WAVE * WAVES;

typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) void lds_void;

// Global-address-space views of device pointers.  A load through a generic
// pointer compiles to a FLAT load, which counts in lgkmcnt as well as vmcnt:
// every LDS read issued after it then waits (s_waitcnt lgkmcnt(0)) for the
// HBM round trip too.  The walk reads frame bytes past the window, chunk
// descriptors and the 5-tuple past the window through these instead.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gbl(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl_mut(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

// HBM -> LDS staging of one 16-B chunk per lane (LDS-DMA).  `nt` (uniform,
// INGOT_TUNE_CACHE_POLICY bit 0) marks the frame bytes non-temporal: they are
// read once per launch.
__device__ __forceinline__ void stage16(const uint8_t* src, uint32_t* dst, bool nt) {
    if (nt) __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 16, 0, 2);
    else __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 16, 0, 0);
}
// The same with the policy word: bits 6-8, when non-zero, pick the staging
// loads' cache bits instead of bit 0 (1 sc1, 2 sc1 nt, 3 sc0 sc1, 4 sc0 sc1
// nt, 5 sc0, 6 sc0 nt) — A/B of where the frame lines are allocated.
__device__ __forceinline__ void stage16p(const uint8_t* src, uint32_t* dst, uint32_t pol) {
#define INGOT_LD(bits) __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)dst, 16, 0, bits)
    switch ((pol >> 6) & 7u) {
    case 1: INGOT_LD(16); return;
    case 2: INGOT_LD(18); return;
    case 3: INGOT_LD(17); return;
    case 4: INGOT_LD(19); return;
    case 5: INGOT_LD(1); return;
    case 6: INGOT_LD(3); return;
    default:
        if (pol & 1u) INGOT_LD(2);
        else INGOT_LD(0);
    }
#undef INGOT_LD
}

// One record per lane; `pol` = the INGOT_TUNE_CACHE_POLICY bits: bit 1 stores
// non-temporal; bits 3-5 (when non-zero) pick the store's scope bits instead
// (1 sc1, 2 sc1 nt, 3 sc0 sc1, 4 sc0 sc1 nt, 5 sc0: A/B of where the records'
// dirty lines sit at the end of the kernel).  The stores are written as asm:
// with a plain-store twin in the other branch the compiler merges the two and
// drops the hint.  (An extra store the waitcnt pass cannot see only makes its
// vmcnt waits stricter; the s_nop covers the store-data VGPR hazard the
// hazard recognizer cannot see in asm.)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// Plain stores through the global address space (HIP's vector types have no
// assignment in address space 1; clang's ext vectors do).
__device__ __forceinline__ void st_global(uint4* dst, const uint4& v) {
    *(__attribute__((address_space(1))) u32x4*)dst = u32x4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ void st_global(uint2* dst, const uint2& v) {
    *(__attribute__((address_space(1))) u32x2*)dst = u32x2{v.x, v.y};
}
#define INGOT_ST(op, bits) asm volatile(op " %0, %1, off " bits "\n\ts_nop 1" ::"v"(dst), "v"(x) : "memory")
#define INGOT_ST_SWITCH(op)                                    \
    switch ((pol >> 3) & 7u) {                                 \
    case 1: INGOT_ST(op, "sc1"); return;                       \
    case 2: INGOT_ST(op, "sc1 nt"); return;                    \
    case 3: INGOT_ST(op, "sc0 sc1"); return;                   \
    case 4: INGOT_ST(op, "sc0 sc1 nt"); return;                \
    case 5: INGOT_ST(op, "sc0"); return;                       \
    default: if (pol & 2u) { INGOT_ST(op, "nt"); return; }     \
    }
__device__ __forceinline__ void store_rec(uint4* dst, const uint4& v, uint32_t pol) {
    const u32x4 x{v.x, v.y, v.z, v.w};
    INGOT_ST_SWITCH("global_store_dwordx4")
    st_global(dst, v);
}
__device__ __forceinline__ void store_rec(uint2* dst, const uint2& v, uint32_t pol) {
    const u32x2 x{v.x, v.y};
    INGOT_ST_SWITCH("global_store_dwordx2")
    st_global(dst, v);
}
#undef INGOT_ST_SWITCH
#undef INGOT_ST

// Slot (16-B unit) of chunk c of packet p inside a wave's LDS image.
// NCH = 4: g(p) = (p>>2)&3; NCH = 8: g(p) = (p>>1)&7 (see header comment);
// other NCH: linear.
template <uint32_t NCH>
__device__ __forceinline__ uint32_t swz(uint32_t p) {
    if constexpr (NCH == 4) return (p >> 2) & 3u;
    else if constexpr (NCH == 8) return (p >> 1) & 7u;
    else return 0u;
}

template <uint32_t NCH>
__device__ __forceinline__ uint32_t slot_of(uint32_t p, uint32_t c) {
    return NCH * p + (c ^ swz<NCH>(p));
}

// One lane's view of its frame: LDS window for the first bytes, HBM beyond.
template <uint32_t NCH>
struct Frame {
    static constexpr bool kRead = false;
    const lds_u32* win;  // this wave's LDS image
    uint32_t p;          // packet index within the wave (== lane)
    uint32_t sh;         // frame start inside its first staged chunk (0..15)
    uint32_t avail;      // frame bytes [0, avail) are staged in LDS
    uint32_t len;        // frame length
    const uint8_t* g;    // frame start in HBM

    __device__ __forceinline__ uint32_t dw(uint32_t b) const {
        return win[slot_of<NCH>(p, b >> 4) * 4u + ((b >> 2) & 3u)];
    }

    // n (1..4) bytes at frame offset i as a big-endian integer.
    // Caller guarantees i + n <= len (every read follows its bounds check).
    __device__ __forceinline__ uint32_t be(uint32_t i, uint32_t n) const {
        uint32_t v;
        if (i + n <= avail) {
            const uint32_t b = sh + i;
            const uint32_t a = b & ~3u;
            const uint32_t d0 = dw(a);
            // the second dword only when the bytes straddle it (then it lies
            // inside the staged chunks); clamped so that a speculated read
            // stays inside this packet's slots too
            const uint32_t a1 = a + 4u < 16u * NCH ? a + 4u : a;
            const uint32_t d1 = ((b & 3u) + n > 4u) ? dw(a1) : 0u;
            const uint32_t x = __builtin_amdgcn_alignbyte(d1, d0, b & 3u);  // bytes b.. little-endian
            v = __builtin_bswap32(x) >> (32u - 8u * n);
        } else {
            v = beyond(i, n);
        }
        return v;
    }

    // NW consecutive big-endian words at frame offset i, all from LDS: NW+1
    // aligned dwords and one v_perm each (align + byte swap).  The caller
    // keeps only words below `avail`; reads past it stay inside this packet's
    // image (chunk index clamped) and are discarded.
    template <uint32_t NW>
    __device__ __forceinline__ void be_words(uint32_t i, uint32_t* out) const {
        const uint32_t b = sh + i;
        const uint32_t sel = (b & 3u) * 0x01010101u + 0x00010203u;
        uint32_t d[NW + 1];
#pragma unroll
        for (uint32_t k = 0; k <= NW; ++k) {
            const uint32_t q = (b >> 2) + k;  // dword of the staged bytes
            const uint32_t c = (q >> 2) < NCH - 1u ? (q >> 2) : NCH - 1u;
            d[k] = win[slot_of<NCH>(p, c) * 4u + (q & 3u)];
        }
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k) out[k] = __builtin_amdgcn_perm(d[k + 1], d[k], sel);
    }

    // As be_words, for a block NOT in the window: the 16-B-aligned chunks
    // holding block bytes (at most 3, from L2 — the staging just fetched
    // their 128-B lines) instead of 4 byte loads per word; then a dword
    // select + one v_perm per word.  Only chunks holding block bytes are
    // read, so nothing past the frame's last 16-B chunk is touched.
    __device__ __forceinline__ void be_words_global8(uint32_t i, uint32_t nw,
                                                     uint32_t* out) const {
        const uintptr_t at = (uintptr_t)(g + i);
        const auto* q = (const __attribute__((address_space(1))) u32x4*)(at & ~(uintptr_t)15);
        const uint32_t r = (uint32_t)(at & 15u);
        const uint32_t end = r + 4u * nw;
        const u32x4 z = {0u, 0u, 0u, 0u};
        const u32x4 c0 = q[0];
        const u32x4 c1 = end > 16u ? q[1] : z;
        const u32x4 c2 = end > 32u ? q[2] : z;
        const uint32_t d[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y,
                                c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
        const uint32_t s = r >> 2;
        uint32_t e[9];
#pragma unroll
        for (uint32_t j = 0; j < 9; ++j)
            e[j] = s == 0u ? d[j] : s == 1u ? d[j + 1] : s == 2u ? d[j + 2] : d[j + 3];
        const uint32_t sel = (r & 3u) * 0x01010101u + 0x00010203u;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) out[k] = __builtin_amdgcn_perm(e[k + 1], e[k], sel);
    }

    // A big-endian word at frame offset i (i + 4 <= len): LDS when staged,
    // else one or two aligned dword loads (never past the word's own dwords).
    __device__ __forceinline__ uint32_t be32(uint32_t i) const {
        if (i + 4u <= avail) return be(i, 4);
        const uintptr_t at = (uintptr_t)(g + i);
        const auto* d = gbl(reinterpret_cast<const uint32_t*>(at & ~(uintptr_t)3));
        const uint32_t r = (uint32_t)(at & 3u);
        const uint32_t d0 = d[0];
        const uint32_t d1 = r ? d[1] : 0u;
        return __builtin_amdgcn_perm(d1, d0, r * 0x01010101u + 0x00010203u);
    }

    // Bytes past the staged window (long option / EH chains), read straight
    // from HBM by the lanes that need them.  Byte loads: measured faster on
    // config 3 than aligned 16-B loads + lane selects (566 vs 659 us/step),
    // since scattered per-lane 16-B requests cost 16x the texture-path work
    // for the same one DRAM sector.
    __device__ __forceinline__ uint32_t beyond(uint32_t i, uint32_t n) const {
        uint32_t v = 0;
        const auto* gg = gbl(g);
        for (uint32_t k = 0; k < n; ++k) v = (v << 8) | gg[i + k];
        return v;
    }

    // Getter of a layout field of the header starting at `hdr`.
    __device__ __forceinline__ uint32_t get(uint32_t hdr, Field f) const {
        return (be(hdr + f.byte0(), f.nbytes()) >> f.rshift()) & f.mask();
    }

    // Setter support: byte i of the frame in the staged copy (so a later
    // edit reads the new value) ...
    __device__ __forceinline__ void put_staged(uint32_t i, uint8_t v) const {
        if (i < avail) {
            const uint32_t b = sh + i;
            const uint32_t d = slot_of<NCH>(p, b >> 4) * 4u + ((b >> 2) & 3u);
            typedef __attribute__((address_space(3))) uint8_t lds_u8;
            const_cast<lds_u8*>(reinterpret_cast<const lds_u8*>(win))[d * 4u + (b & 3u)] = v;
        }
    }
    // ... and staged chunk c (16 B from the 16-B-aligned staging base).
    __device__ __forceinline__ uint4 chunk(uint32_t c) const {
        const uint32_t d = slot_of<NCH>(p, c) * 4u;
        return make_uint4(win[d], win[d + 1], win[d + 2], win[d + 3]);
    }
};

// parse_read's view of a multi-chunk packet (k_parse_read, parse.rs:511-537):
// offsets are logical (the chunks concatenated) and `len` is the end of the
// current chunk, so every bounds check in the walk is a chunk bound.  Chunk
// 0 gets CS0 16-B slots per packet in LDS (packet-major, like a frame's
// window: a packet's pieces sit side by side, so the wave's requests for one
// frame coalesce).  A later chunk that lies inside chunk 0's staged window
// (chunks cut from one buffer, like the reference bench's one chunk per
// header) is read from there; other chunks are read from L2/HBM.  The
// descriptors of chunks 1..NPRE, unless a packet's last, are loaded with
// chunk 0's; the last chunk (an mblk chain's payload) and chunks past NPRE
// are looked up when the walk reaches them.
// LAZY (ingot_gpu_parse_read_first with INGOT_TUNE_READ_PLAN 17): the
// packet's chunk bounds (pkt_seg[pi], pkt_seg[pi + 1]) are not loaded up
// front — chunk 0 comes per packet — but on the first more() / advance(),
// i.e. only by a walk that leaves chunk 0 or fails in it (NPRE = 0: no later
// descriptor is prefetched, since they are found through the bounds).
template <int CS0, bool DENSE = false, int NPRE = 3, bool LAZY = false>
struct SegFrameP {
    static_assert(!LAZY || NPRE == 0, "lazy bounds: no descriptor prefetch");
    static constexpr bool kRead = true;
    const lds_u32* win;  // this wave's image: 64 x CS0 slots
    uint32_t p;          // lane
    uint32_t L, len;     // current chunk: logical [L, len)
    uint32_t sh, avail;  // its start in chunk 0's window, its bytes staged there
    const uint8_t* g;    // g[i] = logical byte i of the current chunk
    const uint8_t* arena;
    const uint64_t* seg_off;
    const uint16_t* seg_len;
    mutable uint32_t s0, nseg;  // LAZY: nseg == kUnknown until bounds() loads them
    uint32_t k;
    const uint32_t* pkt_seg;  // LAZY: the bounds array and this packet's index
    uint64_t pi;
    static constexpr uint32_t kUnknown = 0xffffffffu;
    __device__ __forceinline__ void bounds() const {
        if constexpr (LAZY) {
            if (nseg == kUnknown) {
                s0 = gbl(pkt_seg)[pi];
                nseg = gbl(pkt_seg)[pi + 1] - s0;
            }
        }
    }
    uint64_t o0, o1, o2, o3;  // the first four chunks' offsets and lengths
    uint32_t l0, l1, l2, l3;
    int64_t b0;      // chunk 0's window: arena bytes [b0, b0 + span0) staged
    uint32_t span0;

    // staged byte b (window coordinates): a dword of the image
    __device__ __forceinline__ uint32_t dw(uint32_t b) const {
        return win[slot_of<CS0>(p, b >> 4) * 4u + ((b >> 2) & 3u)];
    }
    __device__ __forceinline__ uint32_t be(uint32_t i, uint32_t n) const {
        const uint32_t x0 = i - L;
        if (x0 + n <= avail) {
            const uint32_t b = sh + x0;
            const uint32_t a = b & ~3u;
            const uint32_t d0 = dw(a);
            // the second dword only when the bytes straddle it (then it lies
            // in the staged pieces); clamped to them so that a speculated
            // read stays inside this packet's slots
            const uint32_t a1 = a + 4u < 16u * CS0 ? a + 4u : a;
            const uint32_t d1 = ((b & 3u) + n > 4u) ? dw(a1) : 0u;
            return __builtin_bswap32(__builtin_amdgcn_alignbyte(d1, d0, b & 3u)) >> (32u - 8u * n);
        }
        uint32_t v = 0;
        const auto* gg = gbl(g);
        for (uint32_t j = 0; j < n; ++j) v = (v << 8) | gg[i + j];
        return v;
    }
    __device__ __forceinline__ uint32_t get(uint32_t hdr, Field f) const {
        return (be(hdr + f.byte0(), f.nbytes()) >> f.rshift()) & f.mask();
    }
    __device__ __forceinline__ bool more() const {
        bounds();
        return k + 1 < nseg;
    }
    // Step into a chunk at arena offset o, length l; c = chunk 0's staged
    // pieces (k == 0), else 0: the chunk's bytes are staged only if it lies
    // in chunk 0's window.
    __device__ __forceinline__ void enter(uint64_t o, uint32_t l, uint32_t c) {
        g = arena + o - L;
        const uint32_t e = L + l;
        len = e > 65535u ? 65535u : e;  // record offsets are u16
        sh = (uint32_t)((uintptr_t)(arena + o) & 15u);
        avail = c ? (l < 16u * c - sh ? l : 16u * c - sh) : 0u;
        if (k != 0) {
            const int64_t d = (int64_t)o - b0;
            if (d >= 0 && d < (int64_t)span0) {
                sh = (uint32_t)d;
                avail = l < span0 - sh ? l : span0 - sh;
            }
        }
    }
    __device__ __forceinline__ void advance() {
        bounds();
        ++k;
        L = len;
        if (NPRE >= 1 && k + 1 < nseg && k == 1) enter(o1, l1, 0u);
        else if (NPRE >= 2 && k + 1 < nseg && k == 2) enter(o2, l2, 0u);
        else if (NPRE >= 3 && k + 1 < nseg && k == 3) enter(o3, l3, 0u);
        else if constexpr (DENSE) {
            const uint64_t v = gbl(seg_off)[s0 + k];  // (offset << 16) | length
            enter(v >> 16, (uint32_t)(v & 0xffffu), 0u);
        } else {
            enter(gbl(seg_off)[s0 + k], gbl(seg_len)[s0 + k], 0u);
        }
    }
};

struct Rec {
    uint32_t status, err_layer, l3_kind, l4_kind, n_vlan, n_v6ext, l4_proto, flags;
    uint32_t l3_off, l4_off, payload_off, ethertype;
    uint32_t o_udp, o_gen, i_eth;  // tunnel: outer_udp / outer_encap / inner_eth offsets
};

__device__ __forceinline__ uint2 pack8(const Rec& r) {
    // ingot_rec8 (include/ingot_gpu.h)
    const uint32_t layer = r.status ? (r.err_layer & 3u) : 0u;
    uint2 o;
    o.x = (r.status & 15u) | (layer << 4) | (r.l3_kind << 6) |
          ((r.l4_kind | (r.n_vlan << 3) | ((r.flags & 1u) << 5)) << 8) | (r.n_v6ext << 16) |
          (r.l4_proto << 24);
    o.y = (r.l4_off & 0xffffu) | (r.payload_off << 16);
    return o;
}

__device__ __forceinline__ uint4 pack(const Rec& r) {
    uint4 o;
    o.x = r.status | (r.err_layer << 8) | (r.l3_kind << 16) | (r.l4_kind << 24);
    o.y = r.n_vlan | (r.n_v6ext << 8) | (r.l4_proto << 16) | (r.flags << 24);
    o.z = (r.l3_off & 0xffffu) | (r.l4_off << 16);
    o.w = (r.payload_off & 0xffffu) | (r.ethertype << 16);
    return o;
}

__device__ __forceinline__ uint32_t eh_class(uint32_t h) {
    // IpProtocol::class (ip.rs:40-54)
    if (h == 44u) return EH_FRAGMENT;
    const bool r6564 = h == 0u || h == 43u || h == 60u || h == 135u || h == 139u || h == 140u ||
                       h == 253u || h == 254u;
    return r6564 ? EH_RFC6564 : EH_NONE;
}

__device__ __forceinline__ uint8_t ecn_from_network(uint32_t raw) {
    return (uint8_t)(raw == 3u ? 1u : raw);  // Ecn::from_network, ip.rs:111-119
}

template <class FR>
__device__ __forceinline__ void copy_bytes(const FR& f, uint32_t at, uint8_t* dst, uint32_t n) {
    for (uint32_t k = 0; k < n; k += 4) {
        const uint32_t m = n - k < 4u ? n - k : 4u;  // never read past the field
        const uint32_t v = f.be(at + k, m) << (8u * (4u - m));
        dst[k] = (uint8_t)(v >> 24);
        dst[k + 1] = (uint8_t)(v >> 16);
        if (k + 2 < n) dst[k + 2] = (uint8_t)(v >> 8);
        if (k + 3 < n) dst[k + 3] = (uint8_t)v;
    }
}

// IPv6 extension headers after the fixed header: `subparse(on_next_layer)`
// with hint = next_header (mod.rs:1933-1938), i.e. RepeatedView::parse_choice
// over the rest of the slice (util.rs:199-216): Unwanted (a non-EH class) ends
// the chain, TooSmall is the header's error.  On return q is past the last EH
// and h is its next_header.  false = TooSmall.
template <bool FIELDS, class FR>
__device__ __forceinline__ bool v6_ext_chain(const FR& f, uint32_t len, uint32_t& q, uint32_t& h,
                                             uint32_t& n_eh, ingot_v6eh* eh) {
    while (q < len) {
        const uint32_t c = eh_class(h);
        if (c == EH_NONE) break;  // Err(Unwanted) => break
        uint32_t used, nh, x = 0;
        if (c == EH_FRAGMENT) {
            if (len - q < v6frag::LEN) return false;
            nh = f.be(q, 1);
            used = v6frag::LEN;
        } else {
            if (len - q < v6ext6564::FIXED) return false;
            x = f.be(q, 2);
            nh = x >> 8;
            used = 8u + 8u * (x & 0xffu);  // 2 + (6 + ext_len*8), ip.rs:209
            if (len - q < used) return false;
        }
        if constexpr (FIELDS) {
            if (n_eh < INGOT_MAX_EH_FIELDS) {
                ingot_v6eh* e = &eh[n_eh];
                e->kind = (uint8_t)c;
                e->off = (uint16_t)q;
                e->next_header = (uint8_t)nh;
                if (c == EH_FRAGMENT) {
                    e->ext_len = (uint8_t)f.get(q, v6frag::reserved);
                    e->frag_offset = (uint16_t)f.get(q, v6frag::fragment_offset);
                    e->frag_res_more =
                        (uint8_t)((f.get(q, v6frag::res) << 1) | f.get(q, v6frag::more_frags));
                    e->ident = f.get(q, v6frag::ident);
                } else {
                    e->ext_len = (uint8_t)(x & 0xffu);
                    e->frag_offset = 0;
                    e->frag_res_more = 0;
                    e->ident = 0;
                }
            }
        }
        ++n_eh;
        q += used;
        h = nh;
    }
    return true;
}

// ---------------------------------------------------------------------------
// The chain walk: `<Chain>::parse_slice` for one frame.
// Layer indices are the chain's PacketParseError labels (parse.rs:36-50).
// F: the (inner) frame's getters; T: the tunnel's outer getters (FIELDS only).
// ---------------------------------------------------------------------------
// parse_read: a layer's TooSmall is StraddledHeader when another chunk exists
// (ParseError::convert_read_parse, error.rs:65-72).
template <class FR>
__device__ __forceinline__ uint32_t read_error(const FR& f, uint32_t code) {
    if constexpr (FR::kRead) {
        if (code == INGOT_ERR_TOO_SMALL && f.more()) return INGOT_ERR_STRADDLED_HEADER;
    }
    return code;
}

template <int CHAIN, bool FIELDS, class FR>
__device__ __forceinline__ void walk(FR& f, Rec& r, ingot_fields* F, ingot_tunnel_fields* T) {
    constexpr bool TUN = CHAIN == INGOT_CHAIN_GENEVE_OVER_V6;
    constexpr uint32_t L_L3 = CHAIN == INGOT_CHAIN_VLAN_ULP ? 2u : TUN ? 5u : 1u;
    constexpr uint32_t L_L4 = L_L3 + 1u;
    constexpr bool ULP = CHAIN != INGOT_CHAIN_UDP_PARSER;  // Ulp vs L4 choice
    uint32_t len = f.len;  // end of the current chunk (parse_read) / of the frame

    r = Rec{};
    r.err_layer = 0xffu;
#define FAIL(layer, code)                  \
    do {                                   \
        r.status = read_error(f, (code));  \
        r.err_layer = (layer);             \
        return;                            \
    } while (0)
    // parse_read's slice step after a non-final layer (parse.rs:205-218): an
    // exhausted chunk is replaced by the next; none left is TooSmall here.
#define NEXT_SLICE(layer)                              \
    do {                                               \
        if constexpr (FR::kRead) {                     \
            if (p == len) {                            \
                if (!f.more()) {                       \
                    r.status = INGOT_ERR_TOO_SMALL;    \
                    r.err_layer = (layer);             \
                    return;                            \
                }                                      \
                f.advance();                           \
                len = f.len;                           \
            }                                          \
        }                                              \
    } while (0)

    // -- layer 0: Ethernet (ethernet.rs:46-55); Accessor 14 B else TooSmall.
    if (len < eth::LEN) FAIL(0u, INGOT_ERR_TOO_SMALL);
    uint32_t et = f.get(0, eth::ethertype);
    uint32_t p = eth::LEN;
    r.payload_off = p;
    r.ethertype = et;
    if constexpr (FIELDS && TUN) {
        copy_bytes(f, 0, T->outer_eth_destination, 6);
        copy_bytes(f, 6, T->outer_eth_source, 6);
        T->outer_eth_ethertype = (uint16_t)et;
    } else if constexpr (FIELDS) {
        copy_bytes(f, 0, F->eth_destination, 6);
        copy_bytes(f, 6, F->eth_source, 6);
        F->eth_ethertype = (uint16_t)et;
    }
    if constexpr (CHAIN != INGOT_CHAIN_GENERIC_ULP) NEXT_SLICE(0u);

    // GeneveOverV6Tunnel's outer layers (ingot-examples/src/packets.rs:27-40).
    if constexpr (TUN) {
        // -- layer 1 outer_v6: #[ingot(from = "L3<Q>")] Ipv6 — the L3 choice
        // parses, then TryFrom keeps only the Ipv6 variant (choice.rs:153-187).
        // The generated order is parse_choice -> slice step -> conversion
        // (parse.rs:402-407), so under parse_read an IPv4 header that ends
        // the last chunk is TooSmall before it can be Unwanted.
        if (et == ET_IPV4) {
            r.l3_kind = INGOT_L3_IPV4;
            r.l3_off = p;
            if (len - p < ipv4::LEN) FAIL(1u, INGOT_ERR_TOO_SMALL);
            const uint32_t ihl = f.get(p, ipv4::ihl);
            const uint32_t opt = ihl * 4u > 20u ? ihl * 4u - 20u : 0u;
            if (len - p - ipv4::LEN < opt) FAIL(1u, INGOT_ERR_TOO_SMALL);
            r.l4_proto = f.get(p, ipv4::protocol);
            p += ipv4::LEN + opt;
            r.payload_off = p;
            NEXT_SLICE(1u);
            FAIL(1u, INGOT_ERR_UNWANTED);
        }
        if (et != ET_IPV6) FAIL(1u, INGOT_ERR_UNWANTED);
        r.l3_kind = INGOT_L3_IPV6;
        r.l3_off = p;
        if (len - p < ipv6::LEN) FAIL(1u, INGOT_ERR_TOO_SMALL);
        uint32_t h = f.get(p, ipv6::next_header);
        uint32_t q = p + ipv6::LEN;
        uint32_t n_eh = 0;
        const bool eh_ok = v6_ext_chain<false>(f, len, q, h, n_eh, nullptr);
        r.n_v6ext = n_eh > 255u ? 255u : n_eh;
        if (!eh_ok) FAIL(1u, INGOT_ERR_TOO_SMALL);
        if constexpr (FIELDS) {
            T->outer_v6_version = (uint8_t)f.get(p, ipv6::version);
            T->outer_v6_dscp = (uint8_t)f.get(p, ipv6::dscp);
            T->outer_v6_ecn_raw = (uint8_t)f.get(p, ipv6::ecn);
            T->outer_v6_ecn = ecn_from_network(T->outer_v6_ecn_raw);
            T->outer_v6_flow_label = f.get(p, ipv6::flow_label);
            T->outer_v6_payload_len = (uint16_t)f.get(p, ipv6::payload_len);
            T->outer_v6_next_header = (uint8_t)f.get(p, ipv6::next_header);
            T->outer_v6_hop_limit = (uint8_t)f.get(p, ipv6::hop_limit);
            copy_bytes(f, p + ipv6::SOURCE_BYTE, T->outer_v6_source, 16);
            copy_bytes(f, p + ipv6::DESTINATION_BYTE, T->outer_v6_destination, 16);
            T->outer_v6_ext_len = (uint16_t)(q - p - ipv6::LEN);
            T->outer_v6_n_ext = (uint8_t)r.n_v6ext;
            T->outer_l4_proto = (uint8_t)h;
        }
        p = q;
        r.payload_off = p;
        r.l4_proto = h;
        NEXT_SLICE(1u);

        // -- layer 2 outer_udp: #[ingot(from = "L4<Q>")] Udp (TCP parses, takes
        // the slice step, then is Unwanted; anything else is Unwanted at the
        // choice).
        if (h == IPP_TCP) {
            r.l4_kind = INGOT_L4_TCP;
            r.l4_off = p;
            if (len - p < tcp::LEN) FAIL(2u, INGOT_ERR_TOO_SMALL);
            const uint32_t doff = f.get(p, tcp::data_offset);
            const uint32_t opt = doff * 4u > 20u ? doff * 4u - 20u : 0u;
            if (len - p - tcp::LEN < opt) FAIL(2u, INGOT_ERR_TOO_SMALL);
            p += tcp::LEN + opt;
            r.payload_off = p;
            NEXT_SLICE(2u);
            FAIL(2u, INGOT_ERR_UNWANTED);
        }
        if (h != IPP_UDP) FAIL(2u, INGOT_ERR_UNWANTED);
        r.l4_kind = INGOT_L4_UDP;
        r.l4_off = p;
        r.o_udp = p;
        if (len - p < udp::LEN) FAIL(2u, INGOT_ERR_TOO_SMALL);
        if constexpr (FIELDS) {
            T->outer_udp_off = (uint16_t)p;
            T->outer_udp_source = (uint16_t)f.get(p, udp::source);
            T->outer_udp_destination = (uint16_t)f.get(p, udp::destination);
            T->outer_udp_length = (uint16_t)f.get(p, udp::length);
            T->outer_udp_checksum = (uint16_t)f.get(p, udp::checksum);
        }
        p += udp::LEN;
        r.payload_off = p;
        NEXT_SLICE(2u);

        // -- layer 3 outer_encap: Geneve (geneve.rs:16-44): 8 B, then options
        // split_at(opt_len*4) subparsed as Repeated<GeneveOpt>
        // (mod.rs:1940-1957, util.rs:199-216); an option overrunning the span
        // is TooSmall (GeneveOpt never returns Unwanted).
        r.o_gen = p;
        if (len - p < geneve::LEN) FAIL(3u, INGOT_ERR_TOO_SMALL);
        const uint32_t g0 = f.be(p, 4);  // version | opt_len | flags | protocol_type
        const uint32_t span = ((g0 >> 24) & 0x3fu) * 4u;
        if (len - p - geneve::LEN < span) FAIL(3u, INGOT_ERR_TOO_SMALL);
        uint32_t read = 0, n_opt = 0, crit = 0;
        bool opt_bad = false;
        while (read < span) {
            const uint32_t o = p + geneve::LEN + read, rem = span - read;
            if (rem < geneve_opt::LEN) { opt_bad = true; break; }
            const uint32_t ow = f.be(o, 4);
            const uint32_t data = (ow & 0x1fu) * 4u;
            if (rem - geneve_opt::LEN < data) { opt_bad = true; break; }
            if constexpr (FIELDS) {
                if (n_opt < INGOT_MAX_GENEVE_OPT_FIELDS) {
                    ingot_geneve_opt* g = &T->geneve_opt[n_opt];
                    g->opt_class = (uint16_t)(ow >> 16);
                    g->data_off = (uint16_t)(o + geneve_opt::LEN);
                    g->option_type = (uint8_t)(ow >> 8);
                    g->reserved = (uint8_t)((ow >> 5) & 7u);
                    g->length = (uint8_t)(ow & 0x1fu);
                }
            }
            crit |= (ow >> 15) & 1u;  // GeneveOptionType::is_critical (geneve.rs:72-76)
            ++n_opt;
            read += geneve_opt::LEN + data;
        }
        if (opt_bad) {
            if constexpr (FIELDS) {
                for (uint32_t k = 0; k < INGOT_MAX_GENEVE_OPT_FIELDS; ++k)
                    T->geneve_opt[k] = ingot_geneve_opt{};
            }
            FAIL(3u, INGOT_ERR_TOO_SMALL);
        }
        if constexpr (FIELDS) {
            const uint32_t g1 = f.be(p + 4u, 4);  // vni | reserved
            T->geneve_off = (uint16_t)p;
            T->geneve_version = (uint8_t)(g0 >> 30);
            T->geneve_opt_len = (uint8_t)((g0 >> 24) & 0x3fu);
            T->geneve_flags = (uint8_t)((g0 >> 16) & geneve::FLAGS_KNOWN);  // from_bits_truncate
            T->geneve_protocol_type = (uint16_t)g0;
            T->geneve_vni = g1 >> 8;
            T->geneve_reserved = (uint8_t)g1;
            T->geneve_n_opts = (uint8_t)(n_opt > 255u ? 255u : n_opt);
            T->geneve_critical = (uint8_t)crit;
        }
        p += geneve::LEN + span;
        r.payload_off = p;
        NEXT_SLICE(3u);

        // -- layer 4 inner_eth; from here the record describes the inner frame.
        r.i_eth = p;
        if (len - p < eth::LEN) FAIL(4u, INGOT_ERR_TOO_SMALL);
        et = f.get(p, eth::ethertype);
        if constexpr (FIELDS) {
            T->inner_eth_off = (uint16_t)p;
            copy_bytes(f, p, F->eth_destination, 6);
            copy_bytes(f, p + 6u, F->eth_source, 6);
            F->eth_ethertype = (uint16_t)et;
        }
        r.flags = INGOT_REC_INNER;
        r.l3_kind = r.l4_kind = INGOT_L3_NONE;
        r.l3_off = r.l4_off = 0;
        r.n_v6ext = 0;
        r.l4_proto = 0;
        r.ethertype = et;
        p += eth::LEN;
        r.payload_off = p;
        // control = exit_on_arp; the Option<> sled allows Accept here.
        if (et == ET_ARP) {
            r.flags |= INGOT_REC_ACCEPTED;
            NEXT_SLICE(4u);  // parse_read still steps past skipped layers
            NEXT_SLICE(5u);
            return;
        }
        NEXT_SLICE(4u);
    }

    // GenericUlp: control = exit_on_arp on inner_eth (packets.rs:45-51); the
    // Option<> sled allows Accept at layer 0 (parse.rs:144-156, 221-254).
    if constexpr (CHAIN == INGOT_CHAIN_GENERIC_ULP) {
        if (et == ET_ARP) {
            r.flags = INGOT_REC_ACCEPTED;
            NEXT_SLICE(0u);  // parse_read still steps past skipped layers
            NEXT_SLICE(1u);
            return;
        }
        NEXT_SLICE(0u);
    }

    // -- build-defined VLAN layer: up to two VlanBody tags (ethernet.rs:57-65).
    if constexpr (CHAIN == INGOT_CHAIN_VLAN_ULP) {
        for (uint32_t v = 0; v < 2u && (et == ET_VLAN || et == ET_QINQ); ++v) {
            if (len - p < vlan::LEN) FAIL(1u, INGOT_ERR_TOO_SMALL);
            if constexpr (FIELDS) {
                F->vlan_priority[v] = (uint8_t)f.get(p, vlan::priority);
                F->vlan_dei[v] = (uint8_t)f.get(p, vlan::dei);
                F->vlan_vid[v] = (uint16_t)f.get(p, vlan::vid);
            }
            et = f.get(p, vlan::ethertype);
            if constexpr (FIELDS) F->vlan_ethertype[v] = (uint16_t)et;
            p += vlan::LEN;
            r.n_vlan = v + 1u;
            r.payload_off = p;
            r.ethertype = et;
            NEXT_SLICE(1u);
        }
    }

    // -- L3 choice (choices.rs:17-21): IPV4 -> Ipv4, IPV6 -> Ipv6, else Unwanted.
    uint32_t proto;
    if (et == ET_IPV4) {
        r.l3_kind = INGOT_L3_IPV4;
        r.l3_off = p;
        if (len - p < ipv4::LEN) FAIL(L_L3, INGOT_ERR_TOO_SMALL);
        const uint32_t ihl = f.get(p, ipv4::ihl);
        const uint32_t opt = ihl * 4u > 20u ? ihl * 4u - 20u : 0u;  // ip.rs:91 saturating_sub
        if (len - p - ipv4::LEN < opt) FAIL(L_L3, INGOT_ERR_TOO_SMALL);
        proto = f.get(p, ipv4::protocol);
        if constexpr (FIELDS) {
            F->v4_version = (uint8_t)f.get(p, ipv4::version);
            F->v4_ihl = (uint8_t)ihl;
            F->v4_dscp = (uint8_t)f.get(p, ipv4::dscp);
            F->v4_ecn_raw = (uint8_t)f.get(p, ipv4::ecn);
            F->v4_ecn = ecn_from_network(F->v4_ecn_raw);
            F->v4_total_len = (uint16_t)f.get(p, ipv4::total_len);
            F->v4_identification = (uint16_t)f.get(p, ipv4::identification);
            F->v4_flags = (uint8_t)f.get(p, ipv4::flags);
            F->v4_fragment_offset = (uint16_t)f.get(p, ipv4::fragment_offset);
            F->v4_hop_limit = (uint8_t)f.get(p, ipv4::hop_limit);
            F->v4_protocol = (uint8_t)proto;
            F->v4_checksum = (uint16_t)f.get(p, ipv4::checksum);
            copy_bytes(f, p + 12u, F->v4_source, 4);
            copy_bytes(f, p + 16u, F->v4_destination, 4);
            F->v4_options_off = (uint16_t)(p + ipv4::LEN);
            F->v4_options_len = (uint16_t)opt;
        }
        p += ipv4::LEN + opt;
    } else if (et == ET_IPV6) {
        r.l3_kind = INGOT_L3_IPV6;
        r.l3_off = p;
        if (len - p < ipv6::LEN) FAIL(L_L3, INGOT_ERR_TOO_SMALL);
        uint32_t h = f.get(p, ipv6::next_header);
        uint32_t q = p + ipv6::LEN;
        uint32_t n_eh = 0;
        const bool eh_ok = v6_ext_chain<FIELDS>(f, len, q, h, n_eh, FIELDS ? F->v6_eh : nullptr);
        r.n_v6ext = n_eh > 255u ? 255u : n_eh;
        if (!eh_ok) {
            if constexpr (FIELDS) {
                for (uint32_t k = 0; k < INGOT_MAX_EH_FIELDS; ++k) F->v6_eh[k] = ingot_v6eh{};
            }
            FAIL(L_L3, INGOT_ERR_TOO_SMALL);
        }
        proto = h;
        if constexpr (FIELDS) {
            F->v6_version = (uint8_t)f.get(p, ipv6::version);
            F->v6_dscp = (uint8_t)f.get(p, ipv6::dscp);
            F->v6_ecn_raw = (uint8_t)f.get(p, ipv6::ecn);
            F->v6_ecn = ecn_from_network(F->v6_ecn_raw);
            F->v6_flow_label = f.get(p, ipv6::flow_label);
            F->v6_payload_len = (uint16_t)f.get(p, ipv6::payload_len);
            F->v6_next_header = (uint8_t)f.get(p, ipv6::next_header);
            F->v6_hop_limit = (uint8_t)f.get(p, ipv6::hop_limit);
            copy_bytes(f, p + ipv6::SOURCE_BYTE, F->v6_source, 16);
            copy_bytes(f, p + ipv6::DESTINATION_BYTE, F->v6_destination, 16);
            F->v6_ext_off = (uint16_t)(p + ipv6::LEN);
            F->v6_ext_len = (uint16_t)(q - p - ipv6::LEN);
        }
        p = q;
    } else {
        FAIL(L_L3, INGOT_ERR_UNWANTED);
    }
    r.payload_off = p;
    r.l4_proto = proto;
    NEXT_SLICE(L_L3);

    // -- L4 choice (choices.rs:25-29) / Ulp choice (choices.rs:32-38).
    uint32_t kind;
    if (proto == IPP_TCP) kind = INGOT_L4_TCP;
    else if (proto == IPP_UDP) kind = INGOT_L4_UDP;
    else if (ULP && proto == IPP_ICMP) kind = INGOT_L4_ICMPV4;
    else if (ULP && proto == IPP_ICMP_V6) kind = INGOT_L4_ICMPV6;
    else FAIL(L_L4, INGOT_ERR_UNWANTED);
    r.l4_kind = kind;
    r.l4_off = p;
    if (kind == INGOT_L4_TCP) {
        if (len - p < tcp::LEN) FAIL(L_L4, INGOT_ERR_TOO_SMALL);
        const uint32_t doff = f.get(p, tcp::data_offset);
        const uint32_t opt = doff * 4u > 20u ? doff * 4u - 20u : 0u;  // tcp.rs:28
        if (len - p - tcp::LEN < opt) FAIL(L_L4, INGOT_ERR_TOO_SMALL);
        if constexpr (FIELDS) {
            F->l4_source = (uint16_t)f.get(p, tcp::source);
            F->l4_destination = (uint16_t)f.get(p, tcp::destination);
            F->tcp_sequence = f.get(p, tcp::sequence);
            F->tcp_acknowledgement = f.get(p, tcp::acknowledgement);
            F->tcp_data_offset = (uint8_t)doff;
            F->tcp_reserved = (uint8_t)f.get(p, tcp::reserved);
            F->tcp_flags = (uint8_t)f.get(p, tcp::flags);  // from_bits_truncate: all 8 bits
            F->tcp_window_size = (uint16_t)f.get(p, tcp::window_size);
            F->tcp_checksum = (uint16_t)f.get(p, tcp::checksum);
            F->tcp_urgent_ptr = (uint16_t)f.get(p, tcp::urgent_ptr);
            F->tcp_options_off = (uint16_t)(p + tcp::LEN);
            F->tcp_options_len = (uint16_t)opt;
        }
        p += tcp::LEN + opt;
    } else if (kind == INGOT_L4_UDP) {
        if (len - p < udp::LEN) FAIL(L_L4, INGOT_ERR_TOO_SMALL);
        if constexpr (FIELDS) {
            F->l4_source = (uint16_t)f.get(p, udp::source);
            F->l4_destination = (uint16_t)f.get(p, udp::destination);
            F->udp_length = (uint16_t)f.get(p, udp::length);
            F->udp_checksum = (uint16_t)f.get(p, udp::checksum);
        }
        p += udp::LEN;
    } else {
        if (len - p < icmp::LEN) FAIL(L_L4, INGOT_ERR_TOO_SMALL);
        if constexpr (FIELDS) {
            F->icmp_ty = (uint8_t)f.get(p, icmp::ty);
            F->icmp_code = (uint8_t)f.get(p, icmp::code);
            F->icmp_checksum = (uint16_t)f.get(p, icmp::checksum);
            copy_bytes(f, p + 4u, F->icmp_rest_of_hdr, 4);
        }
        p += icmp::LEN;
    }
    r.payload_off = p;
    // UdpParser: `#[ingot(from = "L4<Q>")] l4: UdpPacket` converts after the
    // parse; a Tcp variant is Unwanted (choice.rs:153-187, parse.rs:196-200).
    if constexpr (CHAIN == INGOT_CHAIN_UDP_PARSER) {
        if (kind != INGOT_L4_UDP) FAIL(L_L4, INGOT_ERR_UNWANTED);
    }
#undef FAIL
#undef NEXT_SLICE
}

// ---------------------------------------------------------------------------
// Kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ const ParseArgs& base_args(const ParseArgs& a) { return a; }
__device__ __forceinline__ const ParseArgs& base_args(const FlowArgs& a) { return a.p; }
__device__ __forceinline__ const ParseArgs& base_args(const ModifyArgs& a) { return a.p; }

// The header at chain layer `layer` of a parsed-Ok record, if it is of `kind`.
template <int CHAIN>
__device__ __forceinline__ bool header_at(const Rec& r, uint32_t layer, uint32_t kind,
                                          uint32_t index, uint32_t& h) {
    const uint32_t k3 = r.l3_kind == INGOT_L3_IPV4 ? HK_V4 : r.l3_kind == INGOT_L3_IPV6 ? HK_V6
                                                                                      : 0xffu;
    const uint32_t k4 = r.l4_kind == INGOT_L4_TCP   ? HK_TCP
                        : r.l4_kind == INGOT_L4_UDP ? HK_UDP
                        : r.l4_kind != INGOT_L4_NONE ? HK_ICMP
                                                     : 0xffu;
    uint32_t have = 0xffu;
    h = 0;
    if constexpr (CHAIN == INGOT_CHAIN_GENEVE_OVER_V6) {
        switch (layer) {
        case 0: have = HK_ETH; break;
        case 1: have = HK_V6; h = eth::LEN; break;
        case 2: have = HK_UDP; h = r.o_udp; break;
        case 3: have = HK_GENEVE; h = r.o_gen; break;
        case 4: have = HK_ETH; h = r.i_eth; break;
        case 5: have = k3; h = r.l3_off; break;
        case 6: have = k4; h = r.l4_off; break;
        }
    } else if constexpr (CHAIN == INGOT_CHAIN_VLAN_ULP) {
        switch (layer) {
        case 0: have = HK_ETH; break;
        case 1:
            if (index < r.n_vlan) have = HK_VLAN;
            h = eth::LEN + vlan::LEN * index;
            break;
        case 2: have = k3; h = r.l3_off; break;
        case 3: have = k4; h = r.l4_off; break;
        }
    } else {
        switch (layer) {
        case 0: have = HK_ETH; break;
        case 1: have = k3; h = r.l3_off; break;
        case 2: have = k4; h = r.l4_off; break;
        }
    }
    return have == kind;
}

// Where a setter's bytes go.  An aligned WB_BYTES block that lies wholly
// inside the frame and inside the staged chunks is written back whole from the
// staged copy after all edits (`dirty` marks its first chunk): HBM then sees
// full blocks instead of byte-masked partial writes.  Other bytes are stored
// at once.  The staged copy always gets the byte.
// Measured on C2 parse-and-decr (1 M x 64 B): 32-B sectors 23.1 us/step vs
// byte stores 25.2 and whole 64-B lines 26.8 (non-temporal stores: no gain).
constexpr uint32_t WB_BYTES = 32;  // write-back unit (aligned), see below

struct EditSink {
    uint8_t* frame;     // frame start in HBM
    uint64_t off;       // frame start, arena offset
    int64_t base;       // staging base (16-B aligned address), arena offset
    uint32_t len;       // frame length
    uint32_t staged;    // staged chunks for this frame (0 = none)
    uint32_t dirty;     // sector first-chunk bits
    uint32_t mis;       // arena address mod 32 (sectors are aligned addresses)
};

template <class FR>
__device__ __forceinline__ void put_byte(const FR& f, EditSink& k, uint32_t i, uint8_t v) {
    f.put_staged(i, v);
    const int64_t a = (int64_t)(k.off + i);
    const int64_t s = ((a + k.mis) & ~(int64_t)(WB_BYTES - 1u)) - k.mis;  // aligned sector
    if (s >= (int64_t)k.off && s + WB_BYTES <= (int64_t)(k.off + k.len) &&
        s + WB_BYTES <= k.base + 16 * (int64_t)k.staged) {
        k.dirty |= 1u << (uint32_t)((s - k.base) >> 4);
    } else {
        gbl_mut(k.frame)[i] = v;
    }
}

// One generated setter: read-modify-write of the field's covering bytes,
// neighbouring bits preserved (bitfield.rs:188-315), big-endian.  The bytes
// are read through the frame view (staged window first).
template <class FR>
__device__ __forceinline__ void apply_edit(const FR& f, EditSink& sink, uint32_t h,
                                           const Edit& e) {
    uint64_t w = f.be(h + e.byte0, e.nbytes);  // fields span <= 4 bytes
    const uint32_t fm = e.bits >= 32 ? 0xffffffffu : ((1u << e.bits) - 1u);
    const uint32_t cur = (uint32_t)(w >> e.rshift) & fm;
    uint32_t v;
    switch (e.op) {
    case INGOT_OP_ADD: v = cur + e.value; break;
    case INGOT_OP_SUB: v = cur - e.value; break;
    case INGOT_OP_AND: v = cur & e.value; break;
    case INGOT_OP_OR: v = cur | e.value; break;
    case INGOT_OP_XOR: v = cur ^ e.value; break;
    default: v = e.value; break;
    }
    w = (w & ~((uint64_t)fm << e.rshift)) | ((uint64_t)(v & fm) << e.rshift);
    for (uint32_t k = 0; k < e.nbytes; ++k)
        put_byte(f, sink, h + e.byte0 + k, (uint8_t)(w >> (8u * (e.nbytes - 1u - k))));
}

// RSS Toeplitz over one 32-bit input word (MSB first) whose first bit is
// input bit B: XOR in the key window W[B + k] for every set bit k.  W is
// lane-uniform (kernel argument), so only the data bits are per lane.
// Nibble tables in LDS: entry (p, v) = XOR of the key windows of the set bits
// of nibble value v at input nibble position p (FLOW_INPUT_BITS/4 = 72
// positions), so a 32-bit input word = 8 LDS lookups.  Every instruction of
// the hash reads one position p (all lanes), i.e. 16 entries; ds_read_b32
// banks are (dword mod 32) per 32-lane group, so 16 entries stored once sit
// in 16 banks (2-way+ conflicts).  FLOW_COPIES = 2 stores the table 2x
// interleaved (entry (p, v) copy c at dword 32p + 2v + c, lane L reading copy
// L & 1): conflict-free, 9 KiB.  One copy (4.5 KiB, the default) measured
// faster on config 5 (390 vs 400 us/step): the smaller footprint fits 6
// blocks per CU instead of 5, worth more than the conflicts cost.  Built once
// per block (the flows grid is persistent).
constexpr uint32_t FLOW_POS = FLOW_INPUT_BITS / 4;
#ifndef INGOT_REC_SKIP
#define INGOT_REC_SKIP 12
#endif
#ifndef INGOT_FLOW_SKIP
#define INGOT_FLOW_SKIP 12
#endif
#ifndef INGOT_FLOW_COPIES
#define INGOT_FLOW_COPIES 1
#endif
constexpr uint32_t FLOW_COPIES = INGOT_FLOW_COPIES;
constexpr uint32_t FLOW_TAB = FLOW_POS * 16 * FLOW_COPIES;

__device__ __forceinline__ void build_flow_table(uint32_t* tab, const uint32_t* W) {
    for (uint32_t e = threadIdx.x; e < FLOW_TAB; e += BLOCK) {
        const uint32_t p = e / (16u * FLOW_COPIES), v = (e / FLOW_COPIES) & 15u;
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) acc ^= ((v >> (3u - k)) & 1u) ? W[4u * p + k] : 0u;
        tab[e] = acc;
    }
}

// The 16-bit table (OUT_FLOWS16): entry (p, v) = the low 16 bits of the
// 32-bit entry, two per dword (entry e at half-word e).  The low 16 bits of a
// Toeplitz hash are the XOR of the low 16 bits of its key windows, so the
// flow bin (hash & bin_mask, bins <= 65,536) is unchanged; 2,304 B instead
// of 4,608 per block.
constexpr uint32_t FLOW_TAB16 = FLOW_POS * 16 / 2;  // dwords
static_assert(FLOW_TAB16 == FLOW_TAB16_DW, "kernels.h's table size");

// Computed by the host (api.cpp: FlowArgs::tab16, from the same key windows)
// and loaded per block: 144 16-B loads from the kernel arguments instead of
// 1,152 entries built from W.
__device__ __forceinline__ void load_flow_table16(uint32_t* tab, const uint32_t* src) {
    for (uint32_t d = threadIdx.x; d < FLOW_TAB16 / 4u; d += BLOCK)
        reinterpret_cast<uint4*>(tab)[d] = reinterpret_cast<const uint4*>(src)[d];
}

// Flow classification (ingot_gpu_flow_hist): hash of src|dst|ports.
// Appending zero ports leaves a Toeplitz hash unchanged, so ICMP/other L4 use
// the same word positions with a zero port word — and an IPv4 input
// (src|dst|ports, 3 words) is the IPv6 word sequence with zero words after
// its ports.  Every lane therefore hashes 9 words at the same table positions:
// no v4/v6 divergence in the LDS lookups (72 per packet, not 24 + 72 per
// mixed wave).
struct FlowWords {
    uint32_t w[9];
};

// The hash input words of a parsed-Ok packet with an L3 layer (false: not
// counted).  The address block (2 words for IPv4, 8 for IPv6, contiguous)
// is read in one burst and one v_perm (align + byte swap) per word: 9 LDS
// dwords when the staged window holds it, else the (at most 3) 16-B chunks
// holding it from L2 — instead of a bounds check, two reads and a wait (or 4
// byte loads) per word.  The port word: LDS, or aligned dwords past the
// window (IPv6 EH chains).
// lanes (k_flows_bits): the path is chosen per lane — a lane
// whose block lies past its window reads it from L2 while the others read
// LDS (a split wave runs both paths, each under its lanes' mask) — so that a
// window ending before some lanes' IPv6 addresses does not send every lane
// of the wave to L2.
template <class FR>
__device__ __forceinline__ bool flow_words(const FR& f, const Rec& r, FlowWords& x,
                                           bool lanes = false) {
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) x.w[k] = 0;
    if (r.status != INGOT_OK || r.l3_kind == INGOT_L3_NONE) return false;
    const bool ports = r.l4_kind == INGOT_L4_TCP || r.l4_kind == INGOT_L4_UDP;
    const uint32_t pw = ports ? f.be32(r.l4_off) : 0u;
    const bool v6 = r.l3_kind == INGOT_L3_IPV6;
    const uint32_t a = r.l3_off + (v6 ? ipv6::SOURCE_BYTE : 12u);  // source address
    const uint32_t naddr = v6 ? 8u : 2u;                            // address words
    uint32_t w[8];
    // one path per wave: a wave split between the two runs both
    const bool in = a + 4u * naddr <= f.avail;
    if (lanes ? in : __all(in)) f.template be_words<8>(a, w);
    else f.be_words_global8(a, naddr, w);
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) {
        const uint32_t ak = k < 8 ? w[k] : 0u;
        x.w[k] = k < naddr ? ak : (k == naddr ? pw : 0u);
    }
    return true;
}

// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96; the
// compiler does not form it from two XORs).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Toeplitz of the 9 words from the LDS nibble tables (LDS only).  Lookup
// (position q, nibble v, copy cp) is at byte 64C q + 4C v + 4cp of the table
// (C = FLOW_COPIES); the table is 64C-B aligned, so the per-lane part
// (4C v | 4cp | base) is one shift + one v_and_or and the position rides in
// the ds_read offset.
__device__ __forceinline__ uint32_t toeplitz9(const FlowWords& x, const uint32_t* tab) {
    uint32_t base = (uint32_t)(size_t)(const lds_u32*)tab +
                    (FLOW_COPIES == 2 ? (threadIdx.x & 1u) << 2 : 0u);  // + table copy
    // opaque to the optimiser: otherwise it folds the position into the OR
    // (one extra v_or per lookup) instead of the ds_read offset
    asm volatile("" : "+v"(base));
    uint32_t h = 0;
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) {
        uint32_t t[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            // nibble j (MSB first) -> byte offset nibble * 4 * FLOW_COPIES
            constexpr uint32_t L = FLOW_COPIES == 2 ? 3u : 2u;
            const uint32_t s = 28u - 4u * j;
            const uint32_t v8 = s >= L ? (x.w[k] >> (s - L)) : (x.w[k] << (L - s));
            const lds_u32* e = (const lds_u32*)(size_t)((v8 & (15u << L)) | base);
            t[j] = e[(8u * k + j) * 16u * FLOW_COPIES];
        }
        h = xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), xor3(t[6], t[7], h));
    }
    return h;
}

// The low 16 bits of the Toeplitz hash of the 9 words from the 16-bit table:
// lookup (position q, nibble v) is the half-word at byte 32 q + 2 v (the
// table is 32-B aligned: one shift + one v_and_or per lookup, the position
// in the ds_read_u16 offset).
__device__ __forceinline__ uint32_t toeplitz9_16(const FlowWords& x, const uint32_t* tab) {
    typedef __attribute__((address_space(3))) const uint16_t lds_u16;
    uint32_t base = (uint32_t)(size_t)(const lds_u32*)tab;
    asm volatile("" : "+v"(base));
    uint32_t h = 0;
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) {
        uint32_t t[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t s = 28u - 4u * j;
            const uint32_t v8 = s >= 1u ? (x.w[k] >> (s - 1u)) : (x.w[k] << 1u);
            lds_u16* e = (lds_u16*)(size_t)((v8 & (15u << 1)) | base);
            t[j] = e[(8u * k + j) * 16u];
        }
        h = xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), xor3(t[6], t[7], h));
    }
    return h;
}

// (a & b) ^ c in one VALU op (v_bitop3_b32, truth table 0x6a).
__device__ __forceinline__ uint32_t andxor(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6a" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// The same low 16 bits of the Toeplitz hash as toeplitz9_16, without a
// table: bit q of the hash is the parity of the input bits ANDed with the key
// bits that reach bit q, i.e. of XOR_k (x.w[k] & W[32 k + 31 - q]) (bit
// 31 - r of W[32 k + 31 - q] is key bit 32 k + r + 31 - q: bit q of the
// window of input bit 32 k + r).  Input word k needs W[32 k + 16 .. 32 k + 31],
// 16 consecutive key windows: one 64-B scalar load from the kernel arguments
// per word, 16 running parities in VGPRs — 9 x 16 v_bitop3 + 16 popcounts per
// packet, no LDS and no per-tile table copy.  W points into the kernel
// argument segment (constant address space) so the loads are scalar.
typedef __attribute__((address_space(4))) const uint32_t kar_u32;
__device__ __forceinline__ uint32_t toeplitz9_bits16(const FlowWords& x, kar_u32* W) {
    uint32_t t[16];
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) t[q] = x.w[0] & W[31u - q];
#pragma unroll
    for (uint32_t k = 1; k < 9; ++k) {
#pragma unroll
        for (uint32_t q = 0; q < 16; ++q) t[q] = andxor(x.w[k], W[32u * k + 31u - q], t[q]);
    }
    uint32_t h = 0;
#pragma unroll
    for (uint32_t q = 0; q < 16; ++q) h |= ((uint32_t)__builtin_popcount(t[q]) & 1u) << q;
    return h;
}

template <bool H16, class FR>
__device__ __forceinline__ bool flow_hash(const FR& f, const Rec& r, const uint32_t* tab,
                                          uint32_t& h, bool lanes = false) {
    FlowWords x;
    const bool ok = flow_words(f, r, x, lanes);
    if constexpr (H16) h = ok ? toeplitz9_16(x, tab) : 0u;
    else h = ok ? toeplitz9(x, tab) : 0u;
    return ok;
}

// Blocks of `kernel` one CU holds at once (its LDS / VGPR footprint), queried
// once per (kernel instance, device).  Keyed by the kernel's address: every
// k_parse<..., ARGS> instance has the same function type, and their LDS
// footprints differ with the window (about 9 blocks per CU at 3 chunks, 4 at 8).
template <class K>
uint32_t resident_per_cu(K kernel) {
    struct Entry {
        const void* k;
        int dev, blocks;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const void* key = reinterpret_cast<const void*>(kernel);
    std::lock_guard<std::mutex> g(mu);
    for (const Entry& e : cache)
        if (e.k == key && e.dev == dev) return (uint32_t)e.blocks;
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, kernel, BLOCK, 0) != hipSuccess || v < 1)
        v = 1;
    cache.push_back(Entry{key, dev, v});
    return (uint32_t)v;
}

// Grid: one 64-packet tile per wave (4 waves per block) up to `cap` blocks;
// larger batches grid-stride.  Measured on MI355X at config-2 size: one tile
// per wave beats 2 tiles per wave by ~2.5% (tools/microbench.py).
uint32_t grid_for(uint64_t n, uint32_t max_blocks) {
    const uint64_t tiles = (n + WAVE - 1) / WAVE;
    const uint64_t want = (tiles + WAVES - 1) / WAVES;
    const uint64_t cap = max_blocks ? max_blocks : 65536ull;
    const uint64_t g = want < cap ? want : cap;
    return (uint32_t)(g ? g : 1);
}

}  // namespace
}  // namespace ingot_gpu
