// parse.hip — CDNA4 (gfx950) batched L2/L3/L4 header extraction.
//
// Replaces ingot's per-packet parse path for a whole batch:
//   * the chain driver `parse_slice` (ingot-macros/src/parse.rs:496-509,
//     layer fragments 292-416) -> `walk()`;
//   * the generated per-header bodies `HeaderParse::parse_choice`
//     (ingot-macros/src/packet/mod.rs:1831-2005) over Accessor chunks
//     (ingot-types/src/accessor.rs:30-67) -> the per-layer blocks of `walk()`;
//   * the `#[choice]` dispatch (choice.rs:231-246) -> ethertype / protocol
//     switches; the IPv6 extension-header loop RepeatedView::parse_choice
//     (ingot-types/src/util.rs:189-228) -> the EH loop;
//   * the XRef getters (bitfield.rs:40-315) -> `Frame::get(Field)` over the
//     constexpr layouts in layouts.h.
//
// Execution model (one lane per packet, 64 packets per wave-tile):
//   1. descriptors: lane i loads its own (offset, len) — coalesced;
//   2. staging: the wave copies the first bytes of its 64 frames (a window of
//      NCH 16-B chunks per frame) HBM -> LDS with `global_load_lds_dwordx4`
//      (LDS-DMA, 1 KiB per wave instruction, no VGPR round trip).  The LDS
//      image is lane-linear per instruction, so the per-packet chunk order is
//      XOR-swizzled on the *source* address (power-of-two NCH) to keep both
//      per-lane dword reads (4-way floor) and b128 reads conflict-free;
//   3. parse: each lane walks Ethernet -> (VLAN) -> IPv4/IPv6(+EHs) -> L4 on
//      its own window, reading big-endian fields with aligned LDS dword pairs
//      + v_alignbyte; bytes past the window (long option / EH chains) are read
//      straight from HBM by the lanes that need them;
//   4. output: one 16-B record per lane (dwordx4, fully coalesced), or the
//      256-B field block in parity mode.
// No MFMA: this is integer field extraction bounded by HBM bandwidth.
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include <type_traits>

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
    *dst = v;
}
__device__ __forceinline__ void store_rec(uint2* dst, const uint2& v, uint32_t pol) {
    const u32x2 x{v.x, v.y};
    INGOT_ST_SWITCH("global_store_dwordx2")
    *dst = v;
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
// PROBE (the compacted slow path, INGOT_TUNE_SLOW_PATH = 1): a read past the
// window loads nothing — it sets `miss` and yields 0, and the walk's loops
// stop; the lane is walked again over a larger, re-staged window.
template <uint32_t NCH, bool PROBE = false>
struct Frame {
    static constexpr bool kRead = false;
    static constexpr bool kProbe = PROBE;
    const lds_u32* win;  // this wave's LDS image
    uint32_t p;          // packet index within the wave (== lane)
    uint32_t sh;         // frame start inside its first staged chunk (0..15)
    uint32_t avail;      // frame bytes [0, avail) are staged in LDS
    uint32_t len;        // frame length
    const uint8_t* g;    // frame start in HBM
    mutable uint32_t miss = 0;  // PROBE: a read fell past the window

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
        } else if constexpr (PROBE) {
            miss = 1u;
            v = 0u;
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
        const uint4* q = reinterpret_cast<const uint4*>(at & ~(uintptr_t)15);
        const uint32_t r = (uint32_t)(at & 15u);
        const uint32_t end = r + 4u * nw;
        const uint4 z = make_uint4(0, 0, 0, 0);
        const uint4 c0 = q[0];
        const uint4 c1 = end > 16u ? q[1] : z;
        const uint4 c2 = end > 32u ? q[2] : z;
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
        const uint32_t* d = reinterpret_cast<const uint32_t*>(at & ~(uintptr_t)3);
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
        for (uint32_t k = 0; k < n; ++k) v = (v << 8) | g[i + k];
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

// parse_read's view of a multi-chunk packet (parse.rs:511-537): offsets are
// logical (the chunks concatenated); `len` is the end of the current chunk, so
// every bounds check in the walk is a chunk bound.  Chunk 0 is staged in LDS
// like a single frame; later chunks are read from L2/HBM.
template <uint32_t NCH>
struct SegFrame : Frame<NCH> {
    static constexpr bool kRead = true;
    const uint8_t* arena;
    const uint64_t* seg_off;
    const uint16_t* seg_len;
    uint32_t s0, k, nseg;  // first chunk's index, current chunk, chunk count

    // Frame::be serves reads: bytes below `avail` (chunk 0's window) from LDS,
    // the rest through g, which advance() rebases so that g[i] is logical
    // byte i of the current chunk.
    __device__ __forceinline__ bool more() const { return k + 1 < nseg; }
    // next_chunk(): the next chunk starts at logical offset `len`.
    __device__ __forceinline__ void advance() {
        ++k;
        const uint32_t l = seg_len[s0 + k];
        this->g = arena + seg_off[s0 + k] - this->len;
        const uint32_t e = this->len + l;
        this->len = e > 65535u ? 65535u : e;  // record offsets are u16
    }
};

// parse_read with the header chunks staged (k_parse_read): the descriptors
// of the first four chunks, except a packet's last, are loaded up front; chunk 0 gets CS0 16-B slots per
// packet (packet-major, like a frame's window: a packet's pieces sit side by
// side, so the wave's requests for one frame coalesce) and each later chunk
// e < 4 that is not the packet's last one gets CS_e pieces in planes (plane
// π holds that piece of all 64 packets: one LDS-DMA instruction per piece
// for the whole wave).  A packet's last chunk is taken to hold the payload
// (an mblk chain's tail) and is read on demand like chunks past the fourth.
// A chunk without planes of its own that lies inside chunk 0's window (chunks
// cut from one buffer, like the reference bench's one chunk per header) is
// staged with chunk 0's pieces and read from there.
// Offsets are logical as in SegFrame; `len` is the current chunk's end.
template <int CS0, int CS1, int CS2, int CS3, bool DENSE = false>
struct SegFrameP {
    static constexpr bool kRead = true;
    static constexpr bool kProbe = false;
    const lds_u32* win;  // this wave's image: 64 x CS0 slots, then the planes
    uint32_t p;          // lane
    uint32_t L, len;     // current chunk: logical [L, len)
    uint32_t plane, sh, avail;  // its first plane (chunks >= 1), start in it, staged bytes
    const uint8_t* g;    // g[i] = logical byte i of the current chunk
    const uint8_t* arena;
    const uint64_t* seg_off;
    const uint16_t* seg_len;
    uint32_t s0, k, nseg;
    uint64_t o0, o1, o2, o3;  // the first four chunks' offsets and lengths
    uint32_t l0, l1, l2, l3;
    int64_t b0;      // chunk 0's window: arena bytes [b0, b0 + span0) staged
    uint32_t span0;
    static constexpr uint32_t kW0 = 0xffffffffu;  // `plane` of a chunk read from that window

    static constexpr uint32_t cs(uint32_t e) {
        return e == 0 ? CS0 : e == 1 ? CS1 : e == 2 ? CS2 : e == 3 ? CS3 : 0;
    }
    static constexpr uint32_t pb(uint32_t e) {  // first plane of chunk e >= 1
        return e == 1 ? 0 : e == 2 ? CS1 : CS1 + CS2;
    }
    // staged chunk-relative byte b of the current chunk: a dword of the image
    __device__ __forceinline__ uint32_t dw(uint32_t b) const {
        const uint32_t c = b >> 4;
        const uint32_t slot =
            k == 0 || plane == kW0 ? slot_of<CS0>(p, c) : WAVE * (CS0 + plane + c) + p;
        return win[slot * 4u + ((b >> 2) & 3u)];
    }
    __device__ __forceinline__ uint32_t be(uint32_t i, uint32_t n) const {
        const uint32_t x0 = i - L;
        if (x0 + n <= avail) {
            const uint32_t b = sh + x0;
            const uint32_t a = b & ~3u;
            const uint32_t d0 = dw(a);
            const uint32_t d1 = ((b & 3u) + n > 4u) ? dw(a + 4u) : 0u;
            return __builtin_bswap32(__builtin_amdgcn_alignbyte(d1, d0, b & 3u)) >> (32u - 8u * n);
        }
        uint32_t v = 0;
        for (uint32_t j = 0; j < n; ++j) v = (v << 8) | g[i + j];
        return v;
    }
    __device__ __forceinline__ uint32_t get(uint32_t hdr, Field f) const {
        return (be(hdr + f.byte0(), f.nbytes()) >> f.rshift()) & f.mask();
    }
    __device__ __forceinline__ bool more() const { return k + 1 < nseg; }
    // chunk e's staged pieces: chunk 0 always; later ones unless last
    __device__ __forceinline__ static uint32_t staged(uint32_t e, uint32_t nseg) {
        return e == 0 ? CS0 : (e + 1 < nseg ? cs(e) : 0u);
    }
    __device__ __forceinline__ void enter(uint64_t o, uint32_t l, uint32_t pl, uint32_t c) {
        g = arena + o - L;
        const uint32_t e = L + l;
        len = e > 65535u ? 65535u : e;  // record offsets are u16
        plane = pl;
        sh = (uint32_t)((uintptr_t)(arena + o) & 15u);
        avail = c ? (l < 16u * c - sh ? l : 16u * c - sh) : 0u;
        if (k != 0 && c == 0) {
            const int64_t d = (int64_t)o - b0;
            if (d >= 0 && d < (int64_t)span0) {
                plane = kW0;
                sh = (uint32_t)d;
                avail = l < span0 - sh ? l : span0 - sh;
            }
        }
    }
    __device__ __forceinline__ void advance() {
        ++k;
        L = len;
        // chunks 1..3 that are not the packet's last had their descriptors
        // loaded with chunk 0's; the last chunk (the payload) and chunks past
        // the fourth are looked up when the walk reaches them
        if (k + 1 < nseg && k == 1) enter(o1, l1, pb(1), staged(1, nseg));
        else if (k + 1 < nseg && k == 2) enter(o2, l2, pb(2), staged(2, nseg));
        else if (k + 1 < nseg && k == 3) enter(o3, l3, pb(3), staged(3, nseg));
        else if constexpr (DENSE) {
            const uint64_t v = seg_off[s0 + k];  // (offset << 16) | length
            enter(v >> 16, (uint32_t)(v & 0xffffu), 0u, 0u);
        } else {
            enter(seg_off[s0 + k], seg_len[s0 + k], 0u, 0u);
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
        if constexpr (FR::kProbe) {
            if (f.miss) break;  // walked again over a larger window
        }
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
        if (et == ET_IPV4) {
            r.l3_kind = INGOT_L3_IPV4;
            r.l3_off = p;
            if (len - p < ipv4::LEN) FAIL(1u, INGOT_ERR_TOO_SMALL);
            const uint32_t ihl = f.get(p, ipv4::ihl);
            const uint32_t opt = ihl * 4u > 20u ? ihl * 4u - 20u : 0u;
            if (len - p - ipv4::LEN < opt) FAIL(1u, INGOT_ERR_TOO_SMALL);
            r.payload_off = p + ipv4::LEN + opt;
            r.l4_proto = f.get(p, ipv4::protocol);
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

        // -- layer 2 outer_udp: #[ingot(from = "L4<Q>")] Udp (TCP parses, then
        // is Unwanted; anything else is Unwanted at the choice).
        if (h == IPP_TCP) {
            r.l4_kind = INGOT_L4_TCP;
            r.l4_off = p;
            if (len - p < tcp::LEN) FAIL(2u, INGOT_ERR_TOO_SMALL);
            const uint32_t doff = f.get(p, tcp::data_offset);
            const uint32_t opt = doff * 4u > 20u ? doff * 4u - 20u : 0u;
            if (len - p - tcp::LEN < opt) FAIL(2u, INGOT_ERR_TOO_SMALL);
            r.payload_off = p + tcp::LEN + opt;
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
            if constexpr (FR::kProbe) {
                if (f.miss) break;
            }
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
        k.frame[i] = v;
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
template <class FR>
__device__ __forceinline__ bool flow_words(const FR& f, const Rec& r, FlowWords& x) {
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
    if (__all(a + 4u * naddr <= f.avail)) f.template be_words<8>(a, w);
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

template <bool H16, class FR>
__device__ __forceinline__ bool flow_hash(const FR& f, const Rec& r, const uint32_t* tab,
                                          uint32_t& h) {
    FlowWords x;
    const bool ok = flow_words(f, r, x);
    if constexpr (H16) h = ok ? toeplitz9_16(x, tab) : 0u;
    else h = ok ? toeplitz9(x, tab) : 0u;
    return ok;
}

// Index of the j-th set bit of m (j < popcount(m)): binary search on
// popcounts, 6 steps.
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t j) {
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t w = 32; w; w >>= 1) {
        const uint64_t lo = (1ull << w) - 1ull;
        const uint32_t c = (uint32_t)__popcll(m & lo);
        if (j >= c) {
            j -= c;
            m >>= w;
            pos += w;
        } else {
            m &= lo;
        }
    }
    return pos;
}

// The compacted slow path (INGOT_TUNE_SLOW_PATH = 1; A/B against per-lane
// byte loads).  After a PROBE walk over the NCH-chunk window,
// the lanes whose chain ran past it are balloted and ranked (prefix count of
// the ballot); in batches of B = 64 NCH / NCH2 lanes the wave re-stages the
// first NCH2 = 2 NCH chunks of just those frames into its LDS image,
// compacted (rank-major, lane-linear per LDS-DMA instruction: every
// instruction fills 64 slots of the batch), and walks those lanes again over
// the larger window; bytes past it are read per lane from L2/HBM.  This is
// the GPU form of the reference's unbounded EH loop (util.rs:206-216) and
// long IPv4/TCP options (ip.rs:91, tcp.rs:28).
template <uint32_t NCH, int CHAIN>
__device__ __forceinline__ void slow_rewalk(const Frame<NCH, true>& fr, Rec& r, bool valid,
                                            uint32_t* wimg, uint32_t lane, const uint8_t* arena,
                                            int64_t base, uint32_t sh, uint32_t len) {
    constexpr uint32_t NCH2 = 2u * NCH;
    constexpr uint32_t B = WAVE * NCH / NCH2;
    const bool miss = valid && fr.miss;
    const uint64_t m = __ballot(miss);
    if (!m) return;
    const uint32_t K = (uint32_t)__popcll(m);
    const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    const uint32_t take2 = len < 16u * NCH2 - sh ? len : 16u * NCH2 - sh;
    const uint32_t nch2 = (sh + take2 + 15u) >> 4;
    for (uint32_t b0 = 0; b0 < K; b0 += B) {
        // every lane's reads of the image have returned (their values were
        // consumed by the walk) before LDS-DMA overwrites it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t cp = q / NCH2, c = q - cp * NCH2;
            const uint32_t j = b0 + cp;
            const uint32_t src = nth_set_bit(m, j < K ? j : K - 1u);
            const uint32_t np = (uint32_t)__shfl((int)nch2, (int)src);
            const int64_t bp = (int64_t)__shfl((long long)base, (int)src);
            if (j < K && c < np) stage16(arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (miss && rank >= b0 && rank < b0 + B) {
            Frame<NCH2> f2{(const lds_u32*)wimg, rank - b0, sh, take2, len, fr.g};
            walk<CHAIN, false>(f2, r, nullptr, nullptr);
        }
    }
}

template <uint32_t NCH, int LAYOUT, int CHAIN, int MODE, class ARGS, int SLOW = 0>
__global__ __launch_bounds__(BLOCK) void k_parse(ARGS args) {
    const ParseArgs& a = base_args(args);
    constexpr bool TUN = CHAIN == INGOT_CHAIN_GENEVE_OVER_V6;
    constexpr uint32_t WIN = NCH * 16u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;  // dwords per wave image
    // No slack past the last image: every LDS read stays inside its packet's
    // slots (Frame::be clamps the second dword of a pair, be_words the chunk),
    // so 5-chunk images take exactly 20 KiB per block and 8 blocks fit a CU.
    // NCH = 0: no staging, every read goes to L2/HBM.
    __shared__ __attribute__((aligned(16))) uint32_t s_win[NCH ? WAVES * WAVE_DW : 16];
    constexpr bool FLOWS = MODE == OUT_FLOWS || MODE == OUT_FLOWS16;
    constexpr bool H16 = MODE == OUT_FLOWS16;
    __shared__ __attribute__((aligned(64 * FLOW_COPIES)))
    uint32_t s_tab[FLOWS ? (H16 ? FLOW_TAB16 : FLOW_TAB) : 1];
    if constexpr (FLOWS) {
        if constexpr (H16) load_flow_table16(s_tab, args.tab16);
        else build_flow_table(s_tab, args.w);
        __syncthreads();
    }

    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint32_t mis = (uint32_t)((uintptr_t)a.arena & 31u);  // arena address mod 32
    // Record modes never read the MAC addresses either (walk<CHAIN, false>
    // reads Ethernet's ethertype only), so frames addressed by offset start
    // their window at the chunk holding byte 12 too.
    // (NCH = 0, nothing staged: no skip — the window's end SKIP + WIN - sh
    // would underflow.)
    constexpr bool RECM = MODE == OUT_REC16 || MODE == OUT_REC8;
    constexpr uint32_t SKIP =
        NCH == 0 ? 0u
        : FLOWS && LAYOUT == LAYOUT_INDEXED && !TUN ? INGOT_FLOW_SKIP
        : RECM && !SLOW && (LAYOUT == LAYOUT_INDEXED || LAYOUT == LAYOUT_PACKED) ? INGOT_REC_SKIP
                                                                                  : 0u;
    static_assert(SKIP <= 12u, "the walk reads the ethertype at frame byte 12");

    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles;
         t += (uint64_t)gridDim.x * WAVES) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        uint64_t off;
        uint32_t len;
        uint32_t s0 = 0, nseg = 0;
        if constexpr (LAYOUT == LAYOUT_SEGMENTED) {
            // chunk 0 is staged like a frame; the rest is read on demand
            s0 = valid ? a.pkt_seg[i] : 0u;
            nseg = valid ? a.pkt_seg[i + 1] - s0 : 0u;
            off = nseg ? a.off[s0] : 0u;
            len = nseg ? (uint32_t)a.len[s0] : 0u;
        } else if constexpr (LAYOUT == LAYOUT_STRIDED) {
            off = i * a.stride;
            len = valid ? (a.len ? (uint32_t)a.len[i] : a.stride) : 0u;
            if (len > a.stride) len = a.stride;  // a slot holds at most one frame
        } else if constexpr (LAYOUT == LAYOUT_PACKED) {
            // frames back to back: offset = the tile's base + the exclusive
            // prefix of the tile's lengths (wavefront scan, 6 shuffle steps)
            len = valid ? (uint32_t)a.len[i] : 0u;
            uint32_t x = len;
#pragma unroll
            for (uint32_t d = 1; d < WAVE; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, d);
                if (lane >= d) x += y;
            }
            off = a.off[t / PACKED_GROUP] + a.tile_local[t] + (x - len);
            if (valid && a.off_out) a.off_out[i] = off;
        } else {
            off = valid ? a.off[i] : 0u;
            len = valid ? (uint32_t)a.len[i] : 0u;
        }
        // 16-B alignment of the absolute address (the arena itself may be at
        // any alignment): the staged chunks are aligned loads, `base` may sit
        // up to 15 B before the arena (same 16-B block: same page).
        // Flows (indexed frames): the window starts at the 16-B chunk holding
        // frame byte SKIP (12, the ethertype), not at the frame start — the
        // MAC addresses are never read there, and NCH chunks then reach past
        // the IPv6 addresses and ports.  Frame bytes [SKIP - sh, SKIP - sh +
        // WIN) are staged; the walk reads nothing below SKIP, so `avail` (the
        // window's end) is the only bound Frame checks, and fr.sh = sh - SKIP
        // (mod 2^32) maps frame byte i >= SKIP to image byte i + sh - SKIP.
        const uint32_t sh = (uint32_t)((off + SKIP + mis) & 15u);
        const int64_t base = (int64_t)off + (int64_t)SKIP - (int64_t)sh;
        uint32_t take, nch;
        if constexpr (SKIP == 0) {
            take = NCH == 0 ? 0u : (len < WIN - sh ? len : WIN - sh);
            nch = (sh + take + 15u) >> 4;
        } else {
            uint32_t wend = SKIP + WIN - sh;  // frame byte after the window
            if (a.linewin) {
                // Line-completing window: stage up to the end of the 128-B
                // line chunk linewin - 1 lies in (at least linewin chunks, at
                // most NCH).  HBM moves those lines whole anyway; staging the
                // rest of them spares the walk re-reading their bytes past
                // a fixed window from L2 after the line has been evicted.
                const uint32_t lp = (uint32_t)((uintptr_t)(a.arena + base) >> 4) & 7u;
                uint32_t want = ((lp + a.linewin + 7u) & ~7u) - lp;
                if (want > NCH) want = NCH;
                wend = SKIP + 16u * want - sh;
            }
            take = len < wend ? len : wend;
            const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
            nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
        }

        // Stage: instruction k, lane L fills LDS slot q = 64k + L, i.e.
        // packet p = q / NCH, swizzled chunk c.  (LDS-DMA: lane-linear image.)
#pragma unroll
        for (uint32_t k = 0; k < (NCH ? NCH : 1u) && NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            constexpr uint32_t NCH1 = NCH ? NCH : 1u;
            const uint32_t pp = q / NCH1;
            const uint32_t c = (q - pp * NCH1) ^ swz<NCH>(pp);
            const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
            int64_t bp;
            if constexpr (LAYOUT == LAYOUT_STRIDED) {
                bp = (int64_t)((t * WAVE + pp) * a.stride);
            } else {
                bp = (int64_t)__shfl((long long)base, (int)pp);
            }
            if (c < np) stage16p(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, a.policy);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        static_assert(!SLOW || (LAYOUT == LAYOUT_INDEXED && MODE == OUT_REC16),
                      "the compacted slow path is built for indexed 16-B records");
        using FR = typename std::conditional<LAYOUT == LAYOUT_SEGMENTED, SegFrame<NCH>,
                                             Frame<NCH, SLOW != 0>>::type;
        FR fr;
        fr.win = (const lds_u32*)wimg;
        fr.p = lane;
        fr.sh = sh - SKIP;
        fr.avail = take;
        fr.len = len;
        fr.g = a.arena + off;
        if constexpr (LAYOUT == LAYOUT_SEGMENTED) {
            fr.arena = a.arena;
            fr.seg_off = a.off;
            fr.seg_len = a.len;
            fr.s0 = s0;
            fr.k = 0;
            fr.nseg = nseg;
        }
        Rec r;
        if constexpr (MODE == OUT_FIELDS) {
            // ingot_fields, or ingot_geneve_fields (inner + outer) for the tunnel.
            using OutT = typename std::conditional<TUN, ingot_geneve_fields, ingot_fields>::type;
            OutT* G = static_cast<OutT*>(a.out) + (valid ? i : 0);
            if (valid) {
                uint4* z = reinterpret_cast<uint4*>(G);
#pragma unroll
                for (int k = 0; k < (int)(sizeof(OutT) / 16); ++k) z[k] = make_uint4(0, 0, 0, 0);
                ingot_fields* F;
                ingot_tunnel_fields* T = nullptr;
                if constexpr (TUN) {
                    F = &G->inner;
                    T = &G->outer;
                } else {
                    F = G;
                }
                walk<CHAIN, true>(fr, r, F, T);
                reinterpret_cast<uint4*>(F)[0] = pack(r);
            }
        } else if constexpr (MODE == OUT_REC8) {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            if (valid) store_rec(static_cast<uint2*>(a.out) + i, pack8(r), a.policy);
        } else if constexpr (MODE == OUT_MODIFY) {
            // parse, then the setters in order (each sees the previous
            // edits' bytes: put8 updates HBM and the staged window)
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            if (valid && r.status == INGOT_OK) {
                EditSink sink{const_cast<uint8_t*>(a.arena) + off, off, base, len, NCH ? nch : 0u,
                              0u, mis};
                for (uint32_t k = 0; k < args.n_edits; ++k) {
                    const Edit e = args.e[k];
                    uint32_t h;
                    if (header_at<CHAIN>(r, e.layer, e.kind, e.index, h))
                        apply_edit(fr, sink, h, e);
                }
                // whole-sector write-back of the staged copy
                uint4* dst = reinterpret_cast<uint4*>(const_cast<uint8_t*>(a.arena) + base);
                for (uint32_t d = sink.dirty; d; d &= d - 1u) {
                    const uint32_t c = __builtin_ctz(d);
#pragma unroll
                    for (uint32_t q = 0; q < WB_BYTES / 16u; ++q) dst[c + q] = fr.chunk(c + q);
                }
            }
            if (valid && a.out) static_cast<uint4*>(a.out)[i] = pack(r);
            // the window writes must land before the next tile's LDS-DMA
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if constexpr (FLOWS) {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            uint32_t h;
            const bool counted = valid && flow_hash<H16>(fr, r, s_tab, h);
            if (valid) {
                args.flow[i] = counted ? (h & args.bin_mask) : INGOT_FLOW_NONE;
                if (args.hash) args.hash[i] = h;
            }
        } else {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            if constexpr (SLOW)
                slow_rewalk<NCH, CHAIN>(fr, r, valid, wimg, lane, a.arena, base, sh, len);
            if (valid) store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        }
        if constexpr (LAYOUT == LAYOUT_SEGMENTED) {
            if (valid && a.chunk) a.chunk[i] = (uint16_t)fr.k;
        }
        // The next tile's LDS-DMA overwrites this image: every lane's reads
        // above have returned (their values were consumed by the store).
    }
}

// parse_read over chunk lists with the header chunks staged (SegFrameP): per
// tile, the packets' chunk bounds and the first four chunks' descriptors are
// loaded together (independent loads), chunk 0 is staged packet-major like a
// frame window, the later non-final chunks plane by plane, then the walk —
// no dependent descriptor or byte load for headers inside staged pieces.
// One 64-packet tile per wave.
template <int CS0, int CS1, int CS2, int CS3, int CHAIN, int MODE, bool DENSE = false>
__global__ __launch_bounds__(BLOCK) void k_parse_read(ParseArgs a) {
    using FR = SegFrameP<CS0, CS1, CS2, CS3, DENSE>;
    constexpr uint32_t P = CS0 + CS1 + CS2 + CS3;
    constexpr uint32_t WAVE_DW = WAVE * P * 4u;
    constexpr bool TUN = CHAIN == INGOT_CHAIN_GENEVE_OVER_V6;
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW + 16];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles;
         t += (uint64_t)gridDim.x * WAVES) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        const uint32_t s0 = valid ? a.pkt_seg[i] : 0u;
        const uint32_t nseg = valid ? a.pkt_seg[i + 1] - s0 : 0u;
        FR fr;
        if constexpr (DENSE) {
            // one 8-B entry per chunk: (offset << 16) | length; chunks 1..3
            // only when not the packet's last (SegFrameP::advance)
            const uint64_t v0 = nseg > 0 ? a.off[s0] : 0u;
            const uint64_t v1 = nseg > 2 ? a.off[s0 + 1] : 0u;
            const uint64_t v2 = nseg > 3 ? a.off[s0 + 2] : 0u;
            const uint64_t v3 = nseg > 4 ? a.off[s0 + 3] : 0u;
            fr.o0 = v0 >> 16;
            fr.o1 = v1 >> 16;
            fr.o2 = v2 >> 16;
            fr.o3 = v3 >> 16;
            fr.l0 = (uint32_t)(v0 & 0xffffu);
            fr.l1 = (uint32_t)(v1 & 0xffffu);
            fr.l2 = (uint32_t)(v2 & 0xffffu);
            fr.l3 = (uint32_t)(v3 & 0xffffu);
        } else {
            fr.o0 = nseg > 0 ? a.off[s0] : 0u;
            fr.o1 = nseg > 2 ? a.off[s0 + 1] : 0u;
            fr.o2 = nseg > 3 ? a.off[s0 + 2] : 0u;
            fr.o3 = nseg > 4 ? a.off[s0 + 3] : 0u;
            fr.l0 = nseg > 0 ? a.len[s0] : 0u;
            fr.l1 = nseg > 2 ? a.len[s0 + 1] : 0u;
            fr.l2 = nseg > 3 ? a.len[s0 + 2] : 0u;
            fr.l3 = nseg > 4 ? a.len[s0 + 3] : 0u;
        }
        // chunk 0, packet-major: instruction k, lane L fills slot 64k + L =
        // packet q / CS0, piece (q mod CS0) ^ swz (16-B aligned absolute
        // addresses; pieces only below the chunk's end)
        const uint32_t sh0 = (uint32_t)((uintptr_t)(a.arena + fr.o0) & 15u);
        const int64_t base0 = (int64_t)fr.o0 - (int64_t)sh0;
        // chunk 0's window: CS0 pieces, or (a.linewin = m) a line-completing
        // window — at least m pieces, then to the end of that 128-B line
        // (k_parse's windows), at most CS0
        uint32_t want = CS0;
        if (a.linewin) {
            const uint32_t lp = (uint32_t)((uintptr_t)(a.arena + base0) >> 4) & 7u;
            want = ((lp + a.linewin + 7u) & ~7u) - lp;
            if (want > (uint32_t)CS0) want = CS0;
        }
        const uint32_t wlim = 16u * want;
        uint32_t ext = nseg ? sh0 + (fr.l0 < wlim - sh0 ? fr.l0 : wlim - sh0) : 0u;
        // a later non-last chunk without planes that starts inside chunk 0's
        // window: stage the window's pieces up to its end (or the window's)
        auto widen = [&](uint32_t e, uint64_t o, uint32_t l) {
            const int64_t d = (int64_t)o - base0;
            if (FR::cs(e) == 0 && e + 1 < nseg && d >= 0 && d < (int64_t)wlim) {
                const uint32_t end = (uint32_t)d + l < wlim ? (uint32_t)d + l : wlim;
                ext = end > ext ? end : ext;
            }
        };
        widen(1, fr.o1, fr.l1);
        widen(2, fr.o2, fr.l2);
        widen(3, fr.o3, fr.l3);
        const uint32_t n0 = (ext + 15u) >> 4;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)CS0; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / CS0;
            const uint32_t c = (q - pp * CS0) ^ swz<CS0>(pp);
            const uint32_t np = (uint32_t)__shfl((int)n0, (int)pp);
            const int64_t bp = (int64_t)__shfl((long long)base0, (int)pp);
            if (c < np) stage16(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
        // chunks 1..3 unless last: piece j of chunk e into plane CS0 + pb(e) + j
        auto stage_chunk = [&](uint32_t e, uint64_t o, uint32_t l) {
            const uint32_t sh = (uint32_t)((uintptr_t)(a.arena + o) & 15u);
            const uint32_t c = FR::staged(e, nseg);
            for (uint32_t j = 0; j < FR::cs(e); ++j)
                if (j < c && 16u * j < sh + l)
                    stage16(a.arena + o - sh + 16u * j,
                            wimg + (CS0 + FR::pb(e) + j) * WAVE * 4u, false);
        };
        if constexpr (CS1 > 0) stage_chunk(1, fr.o1, fr.l1);
        if constexpr (CS2 > 0) stage_chunk(2, fr.o2, fr.l2);
        if constexpr (CS3 > 0) stage_chunk(3, fr.o3, fr.l3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        fr.win = (const lds_u32*)wimg;
        fr.p = lane;
        fr.arena = a.arena;
        fr.seg_off = a.off;
        fr.seg_len = a.len;
        fr.s0 = s0;
        fr.k = 0;
        fr.nseg = nseg;
        fr.L = 0;
        fr.b0 = base0;
        fr.span0 = 16u * n0;
        fr.enter(fr.o0, fr.l0, 0u, nseg ? want : 0u);
        Rec r;
        if constexpr (MODE == OUT_FIELDS) {
            using OutT = typename std::conditional<TUN, ingot_geneve_fields, ingot_fields>::type;
            OutT* G = static_cast<OutT*>(a.out) + (valid ? i : 0);
            if (valid) {
                uint4* z = reinterpret_cast<uint4*>(G);
#pragma unroll
                for (int k = 0; k < (int)(sizeof(OutT) / 16); ++k) z[k] = make_uint4(0, 0, 0, 0);
                ingot_fields* F;
                ingot_tunnel_fields* T = nullptr;
                if constexpr (TUN) {
                    F = &G->inner;
                    T = &G->outer;
                } else {
                    F = G;
                }
                walk<CHAIN, true>(fr, r, F, T);
                reinterpret_cast<uint4*>(F)[0] = pack(r);
            }
        } else {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            if (valid) store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        }
        if (valid && a.chunk) a.chunk[i] = (uint16_t)fr.k;
        // the next tile's LDS-DMA overwrites this image: every lane's reads
        // above have returned (their values were consumed by the stores)
    }
}

template <int CS0, int CS1, int CS2, int CS3, int MODE, bool DENSE = false>
hipError_t launch_read(const ParseArgs& a, int chain, uint32_t grid, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL(
            (k_parse_read<CS0, CS1, CS2, CS3, INGOT_CHAIN_UDP_PARSER, MODE, DENSE>),
            dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL(
            (k_parse_read<CS0, CS1, CS2, CS3, INGOT_CHAIN_GENERIC_ULP, MODE, DENSE>),
            dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL(
            (k_parse_read<CS0, CS1, CS2, CS3, INGOT_CHAIN_VLAN_ULP, MODE, DENSE>),
            dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(
            (k_parse_read<CS0, CS1, CS2, CS3, INGOT_CHAIN_GENEVE_OVER_V6, MODE, DENSE>),
            dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    }
    return hipGetLastError();
}

// Flow classification with the hash overlapped (INGOT_TUNE_FLOW_KERNEL = 1):
// the persistent k_parse<…, OUT_FLOWS*> loop stages a tile, waits, walks,
// hashes and stores, so the ~72 LDS table lookups per packet run while no
// HBM request of that wave is in flight.  Here a wave reads its tile's hash
// input words out of the LDS image into registers right after the walk,
// issues the next tile's LDS-DMA into the same image (its descriptors were
// loaded during the walk), and only then computes the Toeplitz hash from
// the table — the next tile's HBM latency covers the hash.  One LDS image
// per wave, as in k_parse.
template <uint32_t NCH, int LAYOUT, int CHAIN, bool H16>
__global__ __launch_bounds__(BLOCK) void k_flows(FlowArgs args) {
    static_assert(LAYOUT == LAYOUT_INDEXED || LAYOUT == LAYOUT_STRIDED, "indexed or slots");
    const ParseArgs& a = args.p;
    constexpr bool TUN = CHAIN == INGOT_CHAIN_GENEVE_OVER_V6;
    constexpr uint32_t WIN = NCH * 16u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    constexpr uint32_t SKIP = LAYOUT == LAYOUT_INDEXED && !TUN ? INGOT_FLOW_SKIP : 0u;
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW + 16];
    __shared__ __attribute__((aligned(64))) uint32_t s_tab[H16 ? FLOW_TAB16 : FLOW_TAB];
    if constexpr (H16) load_flow_table16(s_tab, args.tab16);
    else build_flow_table(s_tab, args.w);
    __syncthreads();

    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint64_t step = (uint64_t)gridDim.x * WAVES;
    const uint32_t mis = (uint32_t)((uintptr_t)a.arena & 31u);

    // this lane's frame of tile tt: offset and length
    auto desc = [&](uint64_t tt, uint64_t& off, uint32_t& len) {
        const uint64_t i = tt * WAVE + lane;
        const bool valid = i < a.n;
        if constexpr (LAYOUT == LAYOUT_STRIDED) {
            off = i * a.stride;
            len = valid ? (a.len ? (uint32_t)a.len[i] : a.stride) : 0u;
            if (len > a.stride) len = a.stride;
        } else {
            off = valid ? a.off[i] : 0u;
            len = valid ? (uint32_t)a.len[i] : 0u;
        }
    };
    // the window of a frame (as k_parse): staged bytes and chunk count
    auto window = [&](uint64_t off, uint32_t len, uint32_t& sh, int64_t& base, uint32_t& take,
                      uint32_t& nch) {
        sh = (uint32_t)((off + SKIP + mis) & 15u);
        base = (int64_t)off + (int64_t)SKIP - (int64_t)sh;
        if constexpr (SKIP == 0) {
            take = len < WIN - sh ? len : WIN - sh;
            nch = (sh + take + 15u) >> 4;
        } else {
            const uint32_t wend = SKIP + WIN - sh;
            take = len < wend ? len : wend;
            const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
            nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
        }
    };
    auto stage = [&](uint64_t tt, int64_t base, uint32_t nch) {
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
            int64_t bp;
            if constexpr (LAYOUT == LAYOUT_STRIDED) bp = (int64_t)((tt * WAVE + pp) * a.stride);
            else bp = (int64_t)__shfl((long long)base, (int)pp);
            if (c < np) stage16(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
    };

    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;
    uint64_t off;
    uint32_t len, sh, take, nch;
    int64_t base;
    desc(t, off, len);
    window(off, len, sh, base, take, nch);
    stage(t, base, nch);
    for (;;) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t staged
        const uint64_t tn = t + step;
        const bool more = tn < ntiles;
        uint64_t offn = 0;
        uint32_t lenn = 0;
        if (more) desc(tn, offn, lenn);  // in flight during the walk
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        Frame<NCH> fr{(const lds_u32*)wimg, lane, sh - SKIP, take, len, a.arena + off};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        FlowWords x;
        const bool counted = valid && flow_words(fr, r, x);
        // every lane's reads of the image have returned before the next
        // tile's LDS-DMA overwrites it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (more) {
            window(offn, lenn, sh, base, take, nch);
            stage(tn, base, nch);
        }
        uint32_t h = 0;
        if (counted) {
            if constexpr (H16) h = toeplitz9_16(x, s_tab);
            else h = toeplitz9(x, s_tab);
        }
        if (valid) {
            args.flow[i] = counted ? (h & args.bin_mask) : INGOT_FLOW_NONE;
            if (args.hash) args.hash[i] = h;
        }
        if (!more) break;
        t = tn;
        off = offn;
        len = lenn;
    }
}

// Pipelined variant for fixed slots with no length array (C2-style rings):
// each wave walks several tiles and keeps the next DEPTH-1 tiles' LDS-DMA in
// flight while it parses the current one (DEPTH LDS images per wave, used
// round robin).  Requires stride >= 16*NCH.
template <uint32_t NCH, uint32_t DEPTH, int CHAIN, int MODE>
__global__ __launch_bounds__(BLOCK) void k_parse_pipe(ParseArgs a) {
    constexpr uint32_t WIN = NCH * 16u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    constexpr uint32_t IMG_DW = WAVES * WAVE_DW + 16u;
    __shared__ __attribute__((aligned(16))) uint32_t s_img[DEPTH * IMG_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* img0 = s_img + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint64_t step = (uint64_t)gridDim.x * WAVES;
    const uint32_t take = a.stride < WIN ? a.stride : WIN;

    auto stage = [&](uint64_t tt, uint32_t* img) {
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            uint64_t slot = tt * WAVE + pp;
            if (slot >= a.n) slot = a.n - 1u;  // a valid address for the tail tile
            stage16p(a.arena + slot * a.stride + 16u * c, img + k * WAVE * 4u, a.policy);
        }
    };
    auto parse = [&](uint64_t tt, const uint32_t* img) {
        const uint64_t i = tt * WAVE + lane;
        Frame<NCH> fr{(const lds_u32*)img, lane, 0u, take, a.stride, a.arena + i * a.stride};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        if (i < a.n) {
            if constexpr (MODE == OUT_REC8) store_rec(static_cast<uint2*>(a.out) + i, pack8(r), a.policy);
            else store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        }
    };

    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;
    // prologue: the first DEPTH-1 tiles
#pragma unroll
    for (uint32_t d = 0; d + 1u < DEPTH; ++d)
        if (t + d * step < ntiles) stage(t + d * step, img0 + d * IMG_DW);
    for (uint32_t j = 0;; ++j) {
        const uint64_t tn = t + (DEPTH - 1u) * step;
        if (tn < ntiles) {
            stage(tn, img0 + ((j + DEPTH - 1u) % DEPTH) * IMG_DW);
            // everything but the youngest DEPTH-1 tiles' loads has landed
            // (record stores count too, so this is conservative)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * NCH) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        parse(t, img0 + (j % DEPTH) * IMG_DW);
        t += step;
        if (t >= ntiles) break;
    }
}

// One 32-bit word read past every cache (system scope: a doorbell in pinned
// host memory, written by the host while the kernel runs), made uniform.
// A vector load in asm: the compiler would turn a uniform plain load into a
// scalar one served from the scalar cache, and never see the new value.
__device__ __forceinline__ uint32_t load_system_u32(const uint32_t* p) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                 : "=v"(v)
                 : "v"(p)
                 : "memory");
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Persistent ring consumer (ingot_gpu_parse_ring): k_parse_pipe's staging and
// walk over the tiles of up to INGOT_RING_MAX_BATCHES batches in one launch.
// The batches' tiles are laid end to end and wave w of the W in the grid
// takes tiles w, w + W, w + 2W, ..., so every wave crosses the batch
// boundaries with its next tile's LDS-DMA already in flight: one grid ramp-up
// and one drain per launch instead of one per batch (the per-launch cost the
// two-stream schedule only half hides).  Tiles of batch b are
// staged only once b is published: b < a.published (known at launch), else
// the doorbell word >= db_first + b, polled by the wave that needs it.
template <uint32_t NCH, uint32_t DEPTH, int CHAIN, int MODE>
__global__ __launch_bounds__(BLOCK) void k_parse_ring(RingArgs a) {
    constexpr uint32_t WIN = NCH * 16u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    constexpr uint32_t IMG_DW = WAVES * WAVE_DW + 16u;
    __shared__ __attribute__((aligned(16))) uint32_t s_img[DEPTH * IMG_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* img0 = s_img + wave * WAVE_DW;
    const uint32_t tpb = a.tiles_per_batch;
    const uint32_t W = gridDim.x * WAVES;
    const uint32_t total = tpb * a.nbatches;  // < 2^32 (api.cpp)
    const uint32_t g0 = blockIdx.x * WAVES + wave;
    if (g0 >= total) return;
    const uint32_t J = (total - g0 + W - 1u) / W;  // this wave's tiles
    const uint32_t take = a.stride < WIN ? a.stride : WIN;
    uint32_t avail = a.published;  // batches [0, avail) are known published
    bool live = true;              // false once this wave gave up waiting

    // Batch b published?  Polls only past `avail`: one lane's system-scope
    // load of the doorbell, sleeping between polls, until the word reaches
    // db_first + b or the wave's wait exceeds timeout_ticks.  On success the
    // wave's caches are invalidated (system-scope acquire) before it stages
    // the new batch, so frames written after the launch started are seen.
    auto ready = [&](uint32_t b) -> bool {
        if (b < avail) return true;
        if (!a.doorbell) return false;
        const uint64_t t0 = wall_clock64();
        for (;;) {
            const uint32_t v = load_system_u32(a.doorbell);
            if (v >= a.db_first + b) {
                const uint32_t pub = v - a.db_first + 1u;
                avail = pub < a.nbatches ? pub : a.nbatches;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                return true;
            }
            if (wall_clock64() - t0 > a.timeout_ticks) {
                if (a.status && lane == 0) atomicOr(a.status, 1u);
                return false;
            }
            __builtin_amdgcn_s_sleep(32);
        }
    };
    // (batch, tile) cursors of the next tile to stage and to parse
    uint32_t sb = g0 / tpb, st = g0 - sb * tpb;
    uint32_t pb = sb, pt = st;
    auto adv = [&](uint32_t& b, uint32_t& t) {
        t += W;
        while (t >= tpb) {
            t -= tpb;
            ++b;
        }
    };
    auto stage = [&](uint32_t b, uint32_t t, uint32_t* img) {
        const uint8_t* arena = a.b[b].arena;
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            uint64_t slot = (uint64_t)t * WAVE + pp;
            if (slot >= a.n) slot = a.n - 1u;  // a valid address for the tail tile
            stage16p(arena + slot * a.stride + 16u * c, img + k * WAVE * 4u, a.policy);
        }
    };
    auto parse = [&](uint32_t b, uint32_t t, const uint32_t* img) {
        const uint64_t i = (uint64_t)t * WAVE + lane;
        Frame<NCH> fr{(const lds_u32*)img, lane, 0u, take, a.stride, a.b[b].arena + i * a.stride};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        if (i < a.n) {
            if constexpr (MODE == OUT_REC8)
                store_rec(static_cast<uint2*>(a.b[b].out) + i, pack8(r), a.policy);
            else
                store_rec(static_cast<uint4*>(a.b[b].out) + i, pack(r), a.policy);
        }
    };
    // stage the next tile when there is one and its batch is published
    auto issue = [&](uint32_t& js) -> bool {
        if (!live || js >= J) return false;
        if (!ready(sb)) {
            live = false;
            return false;
        }
        stage(sb, st, img0 + (js % DEPTH) * IMG_DW);
        ++js;
        adv(sb, st);
        return true;
    };

    uint32_t js = 0;  // tiles staged so far
#pragma unroll
    for (uint32_t d = 0; d + 1u < DEPTH; ++d) issue(js);
    for (uint32_t j = 0; j < js; ++j) {
        // tile j's loads have landed: only the DEPTH-1 younger tiles' loads
        // may still be in flight (record stores count too: conservative)
        if (issue(js) && js - j == DEPTH)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * NCH) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        parse(pb, pt, img0 + (j % DEPTH) * IMG_DW);
        adv(pb, pt);
        // every lane's reads of this image have returned before it is restaged
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
}

// In-place rewrite on a slot ring (C2m: the reference's parse-and-decr-v4):
// k_parse_pipe's multi-tile staging, then the setters edit the staged copy
// (put_staged) and mark the write-back units they touch; the wave writes the
// dirty 16-B chunks back lane-linearly from its LDS image — the inverse of the
// staging map, so one store instruction covers 16 consecutive slots instead
// of 64 scattered ones.  Write-back unit `a.wb` bytes (16, 32 or 64, aligned
// within the slot); slots >= 64 B, the whole window inside every frame.
template <uint32_t NCH, uint32_t DEPTH, int CHAIN>
__global__ __launch_bounds__(BLOCK) void k_modify_pipe(ModifyArgs m) {
    const ParseArgs& a = m.p;
    constexpr uint32_t WIN = NCH * 16u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    constexpr uint32_t IMG_DW = WAVES * WAVE_DW + 16u;
    __shared__ __attribute__((aligned(16))) uint32_t s_img[DEPTH * IMG_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* img0 = s_img + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint64_t step = (uint64_t)gridDim.x * WAVES;
    const bool nt_ld = a.policy & 1u;
    uint8_t* arena = const_cast<uint8_t*>(a.arena);
    const uint32_t unit_ch = m.wb / 16u;  // chunks per write-back unit

    auto stage = [&](uint64_t tt, uint32_t* img) {
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            uint64_t slot = tt * WAVE + pp;
            if (slot >= a.n) slot = a.n - 1u;
            stage16(a.arena + slot * a.stride + 16u * c, img + k * WAVE * 4u, nt_ld);
        }
    };
    auto modify = [&](uint64_t tt, uint32_t* img) {
        const uint64_t i = tt * WAVE + lane;
        const bool valid = i < a.n;
        uint8_t* frame = arena + (valid ? i : 0) * a.stride;
        Frame<NCH> fr{(const lds_u32*)img, lane, 0u, WIN, a.stride, frame};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        uint32_t dirty = 0;
        if (valid && r.status == INGOT_OK) {
            for (uint32_t k = 0; k < m.n_edits; ++k) {
                const Edit& e = m.e[k];
                uint32_t h;
                if (!header_at<CHAIN>(r, e.layer, e.kind, e.index, h)) continue;
                // the setter (bitfield.rs:188-315): read-modify-write of the
                // covering bytes through the staged copy
                uint64_t w = fr.be(h + e.byte0, e.nbytes);
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
                for (uint32_t b = 0; b < e.nbytes; ++b) {
                    const uint32_t at = h + e.byte0 + b;
                    const uint8_t x = (uint8_t)(w >> (8u * (e.nbytes - 1u - b)));
                    if (at < WIN) {
                        fr.put_staged(at, x);
                        const uint32_t c0 = (at >> 4) & ~(unit_ch - 1u);
                        dirty |= ((1u << unit_ch) - 1u) << c0;
                    } else {
                        frame[at] = x;  // past the window (slots > 64 B)
                    }
                }
            }
        }
        if (valid && a.out) store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        // every lane's staged edits are in LDS before any lane reads them back
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            const uint32_t d = (uint32_t)__shfl((int)dirty, (int)pp);
            if ((d >> c) & 1u) {
                const uint32_t* src = img + q * 4u;
                const uint4 v = make_uint4(src[0], src[1], src[2], src[3]);
                store_rec(reinterpret_cast<uint4*>(arena + (tt * WAVE + pp) * a.stride + 16u * c),
                          v, a.policy);
            }
        }
    };

    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;
#pragma unroll
    for (uint32_t d = 0; d + 1u < DEPTH; ++d)
        if (t + d * step < ntiles) stage(t + d * step, img0 + d * IMG_DW);
    for (uint32_t j = 0;; ++j) {
        const uint64_t tn = t + (DEPTH - 1u) * step;
        if (tn < ntiles) {
            stage(tn, img0 + ((j + DEPTH - 1u) % DEPTH) * IMG_DW);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * NCH) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        modify(t, img0 + (j % DEPTH) * IMG_DW);
        // the write-back's LDS reads are done before this image is restaged
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t += step;
        if (t >= ntiles) break;
    }
}

template <uint32_t DEPTH>
hipError_t launch_modify_pipe(const ModifyArgs& a, int chain, uint32_t grid, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_modify_pipe<4, DEPTH, INGOT_CHAIN_UDP_PARSER>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_modify_pipe<4, DEPTH, INGOT_CHAIN_GENERIC_ULP>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL((k_modify_pipe<4, DEPTH, INGOT_CHAIN_VLAN_ULP>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <uint32_t NCH, uint32_t DEPTH, int MODE>
hipError_t launch_pipe(const ParseArgs& a, int chain, uint32_t grid, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_UDP_PARSER, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_GENERIC_ULP, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_VLAN_ULP, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
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

// persist_cus != 0: a persistent grid, capped at the blocks the device holds
// at once (cus x resident_per_cu), so no CU runs a second partial round.
template <uint32_t NCH, int LAYOUT, int MODE, class ARGS, int SLOW = 0>
hipError_t launch_chain(const ARGS& a, int chain, uint32_t grid, hipStream_t s,
                        uint32_t persist_cus = 0) {
    auto go = [&](auto kernel) {
        uint32_t g = grid;
        if (persist_cus) {
            const uint32_t cap = persist_cus * resident_per_cu(kernel);
            if (g > cap) g = cap;
        }
        hipLaunchKernelGGL(kernel, dim3(g), dim3(BLOCK), 0, s, a);
    };
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_UDP_PARSER, MODE, ARGS, SLOW>);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_GENERIC_ULP, MODE, ARGS, SLOW>);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_VLAN_ULP, MODE, ARGS, SLOW>);
        break;
    default:
        if constexpr (MODE == OUT_REC8) {
            return hipErrorInvalidValue;  // not offered for the tunnel (api.cpp)
        } else {
            go(k_parse<NCH, LAYOUT, INGOT_CHAIN_GENEVE_OVER_V6, MODE, ARGS, SLOW>);
        }
        break;
    }
    return hipGetLastError();
}

template <uint32_t NCH, int LAYOUT>
hipError_t launch_mode(const ParseArgs& a, int chain, int mode, uint32_t grid, hipStream_t s) {
    switch (mode) {
    case OUT_REC8: return launch_chain<NCH, LAYOUT, OUT_REC8>(a, chain, grid, s);
    case OUT_FIELDS: return launch_chain<NCH, LAYOUT, OUT_FIELDS>(a, chain, grid, s);
    default: return launch_chain<NCH, LAYOUT, OUT_REC16>(a, chain, grid, s);
    }
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

hipError_t launch_parse(const ParseArgs& args, int layout_kind, int chain, int mode,
                        const Tuning& t, hipStream_t s) {
    if (args.n == 0) return hipSuccess;
    ParseArgs a = args;
    // Cache policy (INGOT_TUNE_CACHE_POLICY; measured on MI355X, interleaved
    // A/B): records are written once and never re-read by the
    // kernel, so they are stored non-temporal by default (C3 609 -> 600,
    // C3s 130 -> 127, C4 321 -> 316, C6 399 -> 395 us/step).  Frame bytes are
    // staged non-temporal only by the ring kernel, whose window is the whole
    // 64-B slot (C2 single stream 16.8 -> 15.1 us, two streams 13.5 -> 12.2);
    // elsewhere bytes past the window are re-read from L2, and nt staging
    // costs 19% (C3) / 15% (C3s).  The ring kernel's 16-B records are stored
    // at device scope (`sc1`, written through the XCD's L2) instead of nt:
    // 2 streams 12.32 -> 11.90 us/step, 1 stream 15.33 -> 15.19 (interleaved
    // A/B, profiles/r02_store_scope_ab.json); 8-B records, the rewrite ring
    // and the packed / slotted kernels gain nothing from it (or lose: C3 sc1
    // without nt 588 -> 608 us).  4 = plain loads and stores.
    const bool ring = t.pipeline != 1 && !t.window_strided && layout_kind == LAYOUT_STRIDED &&
                      !a.len && chain != INGOT_CHAIN_GENEVE_OVER_V6 && a.stride >= 64u &&
                      (a.stride == 64u || !t.host_arena) &&
                      (mode == OUT_REC16 || mode == OUT_REC8);
    if (t.cache_policy == 0) a.policy = mode == OUT_FIELDS ? 0u : ring ? (mode == OUT_REC16 ? 11u : 3u) : 2u;
    else a.policy = (uint32_t)t.cache_policy & 0x1fbu;
    const uint32_t g = grid_for(a.n, t.max_blocks);
    // parse_read over chunk lists: chunk 0 staged in a 4-chunk (64-B) window
    // (first mblk-style chunks are short header blocks), the rest from L2/HBM.
    if (layout_kind == LAYOUT_SEGMENTED) {
        if (mode != OUT_FIELDS && mode != OUT_REC16) return hipErrorInvalidValue;
        // dense chunk table (ingot_gpu_parse_read_dense): no length array,
        // one (offset << 16) | length entry per chunk
        if (!a.len) {
            return mode == OUT_FIELDS ? launch_read<4, 0, 0, 0, OUT_FIELDS, true>(a, chain, g, s)
                                      : launch_read<4, 0, 0, 0, OUT_REC16, true>(a, chain, g, s);
        }
        // INGOT_TUNE_READ_PLAN: 16-B pieces staged per chunk of the first four.
        // Measured (tools/abtune.py, us per launch): the
        // reference's one-header-per-chunk shape (c2r, 1 M) 33.3 on demand
        // (9) / 25.1 {4,0,0,0} / 24.2 {2,2,2,0} / 27.0 {4,2,2,0}; header +
        // payload chunks (c3r, 16.7 M) 651 / 667 / 681 / 769 — extra planes
        // cost occupancy on the gather-bound shape.  Default (round 2): chunk
        // 0 in a line-completing window of 3 to 5 pieces (to the end of the
        // 128-B line its third piece lies in; k_parse's windows, DESIGN.md
        // §4): c3r 676 -> 651 us, c2r 23.05 -> 23.24; 3 to 8 pieces reads 15%
        // fewer bytes but loses occupancy (724 us).  1 = the round-1 {4,0,0,0}.
        if (t.read_plan == 9) {
            return mode == OUT_FIELDS ? launch_chain<4, LAYOUT_SEGMENTED, OUT_FIELDS>(a, chain, g, s)
                                      : launch_chain<4, LAYOUT_SEGMENTED, OUT_REC16>(a, chain, g, s);
        }
        if (mode == OUT_FIELDS) return launch_read<4, 0, 0, 0, OUT_FIELDS>(a, chain, g, s);
        // chunk pools in mapped host memory keep the round-1 window (every
        // staged piece is a PCIe read there)
        switch (t.read_plan ? t.read_plan : t.host_arena ? 1 : 11) {
        case 2: return launch_read<2, 2, 2, 0, OUT_REC16>(a, chain, g, s);
        case 3: return launch_read<4, 2, 2, 0, OUT_REC16>(a, chain, g, s);
        case 4: return launch_read<4, 1, 1, 0, OUT_REC16>(a, chain, g, s);
        case 5: return launch_read<3, 0, 0, 0, OUT_REC16>(a, chain, g, s);
        case 6: return launch_read<2, 0, 0, 0, OUT_REC16>(a, chain, g, s);
        case 7:  // line-completing chunk-0 windows of 2 / 4 to 8 pieces
        case 8: {
            ParseArgs b = a;
            b.linewin = t.read_plan == 7 ? 2u : 4u;
            return launch_read<8, 0, 0, 0, OUT_REC16>(b, chain, g, s);
        }
        case 10: {  // ... of 2 to 5 pieces (11, the default: 3 to 5)
            ParseArgs b = a;
            b.linewin = 2u;
            return launch_read<5, 0, 0, 0, OUT_REC16>(b, chain, g, s);
        }
        case 1: return launch_read<4, 0, 0, 0, OUT_REC16>(a, chain, g, s);
        default: {  // 11
            ParseArgs b = a;
            b.linewin = 3u;
            return launch_read<5, 0, 0, 0, OUT_REC16>(b, chain, g, s);
        }
        }
    }
    // Staged window (16-B chunks per frame); defaults measured on MI355X with
    // interleaved A/B in one process (tools/abtune.py):
    //  * packed frames: 3 chunks (C3 595-598 us/step at 2-3 chunks, 614 at 4,
    //    637 at 5, 838 at 9, 648 with no staging);
    //  * slots > 64 B: 3 chunks (C3s 127 us vs 169 at 8); slots <= 64 B: the
    //    whole 64-B slot (4 chunks; C2 is flat from 2 to 4 chunks).
    // Small windows win: they fetch only the header lines and keep LDS per
    // wave low; the rest of a long chain is read from L2/HBM on demand.
    // The tunnel's inner headers start ~88 B in: stage 8 chunks (128 B).
    const bool tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    // C2-style rings (slots >= 64 B, no length array, record output): the
    // double-buffered multi-tile kernel.  Its grid is a whole number of blocks
    // per CU (default 2), so the tiles spread evenly; measured on MI355X (1 M x
    // 64 B, interleaved A/B): 16.6-16.7 vs 18.6-18.8 us per launch on one
    // stream, 13.5-13.6 vs 14.2-14.4 us per step on two; 6 or 12 tiles per
    // wave (uneven over the CUs) lose most of it.
    if (ring) {
        const uint64_t tiles = (a.n + WAVE - 1) / WAVE;
        uint64_t blocks;
        if (t.pipeline > 1) {
            const uint64_t waves = (tiles + (uint64_t)t.pipeline - 1) / (uint64_t)t.pipeline;
            blocks = (waves + WAVES - 1) / WAVES;
        } else {
            const uint64_t cap = 2ull * t.cus;
            blocks = (tiles + WAVES - 1) / WAVES;
            if (blocks > cap) blocks = cap;
        }
        const uint32_t pg = (uint32_t)(blocks ? blocks : 1);
        if (t.pipe_depth == 3)
            return mode == OUT_REC8 ? launch_pipe<4, 3, OUT_REC8>(a, chain, pg, s)
                                    : launch_pipe<4, 3, OUT_REC16>(a, chain, pg, s);
        if (t.pipe_depth == 4)
            return mode == OUT_REC8 ? launch_pipe<4, 4, OUT_REC8>(a, chain, pg, s)
                                    : launch_pipe<4, 4, OUT_REC16>(a, chain, pg, s);
        return mode == OUT_REC8 ? launch_pipe<4, 2, OUT_REC8>(a, chain, pg, s)
                                : launch_pipe<4, 2, OUT_REC16>(a, chain, pg, s);
    }
    // Frames in mapped host memory (ingot_gpu_host_map, zero-copy over
    // PCIe): a read past the window is a PCIe round trip per byte, so larger
    // windows win there (measured, tools/hostpath.py --zero-copy, Mpkt/s:
    // packed C3 202 / 221 / 230 / 211 at 3 / 4 / 5 / 8 chunks; 2048-B slots
    // C3s 256 / 270 / 311 / 317 at 3 / 4 / 5 / 8).
    const bool host = t.host_arena;
    if (layout_kind == LAYOUT_STRIDED) {
        const int w = t.window_strided ? t.window_strided
                      : tun ? 8 : (a.stride <= 64u ? 4 : host ? 8 : 3);
        if (w == 100) return launch_mode<0, LAYOUT_STRIDED>(a, chain, mode, g, s);
        if (w == 2) return launch_mode<2, LAYOUT_STRIDED>(a, chain, mode, g, s);
        if (w == 3) return launch_mode<3, LAYOUT_STRIDED>(a, chain, mode, g, s);
        if (w == 4) return launch_mode<4, LAYOUT_STRIDED>(a, chain, mode, g, s);
        if (w == 5) return launch_mode<5, LAYOUT_STRIDED>(a, chain, mode, g, s);
        return launch_mode<8, LAYOUT_STRIDED>(a, chain, mode, g, s);
    }
    // Records on frames addressed by offset (device arenas, not the tunnel):
    // a line-completing window (ParseArgs::linewin) from the chunk holding
    // byte 12 to the end of the 128-B line its second chunk lies in, at most
    // 5 chunks.  The walk reads the ethertype, IPv4 ihl / protocol and the
    // IPv6 next header in its first two chunks; the rest of that line comes
    // along in the same HBM fetch, so TCP's data offset and EH bytes there
    // are read from LDS instead of from an L2 line that has often been
    // evicted by then.  PMC read bytes per C3 frame: fixed 2 chunks 217,
    // 3 chunks 206, line-completing 172 — the line floor of the walk's bytes
    // is 169 (tools/line_floor.py); us per launch C3 562 -> 544, C3p 583 ->
    // 553, C4 302 -> 288 (round 2, interleaved; profiles/r02_window_ab.json).
    // The tunnel chain's records (outer headers ~80 B, the inner chain past
    // them) take at least 6 chunks, then to the line end, at most 9: C6 400 ->
    // 394 us (fixed 8; a minimum of 2 loses: 468).  Field and rewrite modes
    // keep fixed windows.
    int wi = t.window_indexed;
    if (!wi && (mode == OUT_REC16 || mode == OUT_REC8) && !host)
        wi = !tun ? 25 : layout_kind == LAYOUT_INDEXED ? 1069 : 0;
    if (wi > 1000) {  // 1000 + 10 m + k: line-completing, m to k chunks
        a.linewin = (uint32_t)(wi - 1000) / 10u;
        wi = (wi - 1000) % 10;
    } else if (wi > 20 && wi < 100) {  // 20 + k: line-completing, 2 to k chunks
        a.linewin = 2;
        wi -= 20;
    }
    if (layout_kind == LAYOUT_PACKED) {
        switch (wi ? wi : tun ? 8 : host ? 5 : 3) {
        case 2: return launch_mode<2, LAYOUT_PACKED>(a, chain, mode, g, s);
        case 3: return launch_mode<3, LAYOUT_PACKED>(a, chain, mode, g, s);
        case 8: return launch_mode<8, LAYOUT_PACKED>(a, chain, mode, g, s);
        default: return launch_mode<5, LAYOUT_PACKED>(a, chain, mode, g, s);
        }
    }
    // The compacted slow path (INGOT_TUNE_SLOW_PATH = 1, 16-B records,
    // device arenas): default windows only.
    if (t.slow_path == 1 && mode == OUT_REC16 && !host && !t.window_indexed)
        return tun ? launch_chain<8, LAYOUT_INDEXED, OUT_REC16, ParseArgs, 1>(a, chain, g, s)
                   : launch_chain<3, LAYOUT_INDEXED, OUT_REC16, ParseArgs, 1>(a, chain, g, s);
    switch (wi ? wi : tun ? 8 : host ? 5 : 3) {
    case 100: return launch_mode<0, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 2: return launch_mode<2, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 3: return launch_mode<3, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 4: return launch_mode<4, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 6: return launch_mode<6, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 8: return launch_mode<8, LAYOUT_INDEXED>(a, chain, mode, g, s);
    case 9: return launch_mode<9, LAYOUT_INDEXED>(a, chain, mode, g, s);
    default: return launch_mode<5, LAYOUT_INDEXED>(a, chain, mode, g, s);
    }
}

// Ring rewrite kernel defaults (k_modify_pipe; measured).
constexpr uint32_t kModifyRingWb = 64;
constexpr uint32_t kModifyRingPolicy = 3;  // nt staging loads + nt write-back

// Parse + rewrite: the default windows of the record path.
hipError_t launch_modify(const ModifyArgs& args, int layout_kind, int chain, const Tuning& t,
                         hipStream_t s) {
    if (args.p.n == 0) return hipSuccess;
    ModifyArgs a = args;
    const uint32_t g = grid_for(a.p.n, t.max_blocks);
    const bool tun = chain == INGOT_CHAIN_GENEVE_OVER_V6;
    // Slot rings (slots >= 64 B, no length array): the multi-tile kernel with
    // lane-linear write-back (k_modify_pipe).  Defaults measured on MI355X
    // (DESIGN.md §1c): write-back unit WB, plain staging loads.
    if (t.pipeline != 1 && !t.window_strided && layout_kind == LAYOUT_STRIDED && !a.p.len &&
        !tun && a.p.stride >= 64u) {
        a.wb = t.writeback ? (uint32_t)t.writeback : kModifyRingWb;
        a.p.policy = t.cache_policy ? (uint32_t)t.cache_policy & 0x3bu : kModifyRingPolicy;
        const uint64_t tiles = (a.p.n + WAVE - 1) / WAVE;
        uint64_t blocks;
        if (t.pipeline > 1) {
            const uint64_t waves = (tiles + (uint64_t)t.pipeline - 1) / (uint64_t)t.pipeline;
            blocks = (waves + WAVES - 1) / WAVES;
        } else {
            const uint64_t cap = 2ull * t.cus;
            blocks = (tiles + WAVES - 1) / WAVES;
            if (blocks > cap) blocks = cap;
        }
        const uint32_t pg = (uint32_t)(blocks ? blocks : 1);
        return t.pipe_depth == 3 ? launch_modify_pipe<3>(a, chain, pg, s)
                                 : launch_modify_pipe<2>(a, chain, pg, s);
    }
    if (layout_kind == LAYOUT_STRIDED) {
        if (tun) return launch_chain<8, LAYOUT_STRIDED, OUT_MODIFY>(a, chain, g, s);
        return a.p.stride <= 64u ? launch_chain<4, LAYOUT_STRIDED, OUT_MODIFY>(a, chain, g, s)
                                 : launch_chain<3, LAYOUT_STRIDED, OUT_MODIFY>(a, chain, g, s);
    }
    return tun ? launch_chain<8, LAYOUT_INDEXED, OUT_MODIFY>(a, chain, g, s)
               : launch_chain<3, LAYOUT_INDEXED, OUT_MODIFY>(a, chain, g, s);
}

// Flow mode needs the addresses (IPv6: 32 bytes past byte 22) and ports, so
// its default window is 5 chunks from the chunk holding byte 12 (SKIP in
// k_parse: 392 -> 384 us per C5 flow_hist vs 5 chunks from the frame start;
// 4 chunks from byte 12: 387); the same tuning knobs override the size.
template <uint32_t NCH, int LAYOUT, bool H16>
hipError_t launch_flows_pipe(const FlowArgs& a, int chain, uint32_t grid, hipStream_t s,
                             uint32_t cus) {
    auto go = [&](auto kernel) {
        uint32_t g = grid;
        if (cus) {
            const uint32_t cap = cus * resident_per_cu(kernel);
            if (g > cap) g = cap;
        }
        hipLaunchKernelGGL(kernel, dim3(g), dim3(BLOCK), 0, s, a);
    };
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER: go(k_flows<NCH, LAYOUT, INGOT_CHAIN_UDP_PARSER, H16>); break;
    case INGOT_CHAIN_GENERIC_ULP: go(k_flows<NCH, LAYOUT, INGOT_CHAIN_GENERIC_ULP, H16>); break;
    case INGOT_CHAIN_VLAN_ULP: go(k_flows<NCH, LAYOUT, INGOT_CHAIN_VLAN_ULP, H16>); break;
    default: go(k_flows<NCH, LAYOUT, INGOT_CHAIN_GENEVE_OVER_V6, H16>); break;
    }
    return hipGetLastError();
}

template <int MODE>
hipError_t launch_flows_mode(const FlowArgs& a, int layout_kind, int chain, const Tuning& t,
                             hipStream_t s) {
    const uint32_t g = grid_for(a.p.n, t.max_blocks);
    constexpr bool H16 = MODE == OUT_FLOWS16;
    // The 16-bit table comes with the kernel arguments (a block loads it in
    // one 16-B load per thread), so the default grid is one tile per wave like
    // the plain parse, the hardware dispatcher refilling CUs as blocks finish:
    // C5 flows kernel 314.8 us vs 329.5 persistent (plain parse of the same
    // frames 312.8; profiles/r02_flows_grid_ab.json).  The 32-bit table is
    // built per block (1,152 entries from the key windows), so its grid is
    // persistent; INGOT_TUNE_FLOW_KERNEL = 2 makes the 16-bit one persistent
    // too.  Fixed max_blocks: grid-stride over that many blocks.
    const uint32_t pc = t.max_blocks || (H16 && t.flow_kernel == 0) ? 0u : t.cus;
    // INGOT_TUNE_FLOW_KERNEL = 1: the hash-overlapped kernel (k_flows) at the
    // default windows.  Measured on C5 (tools/abtune.py, us per step incl.
    // the histogram): 360.7 vs 363.6 on one stream, 350.2 vs
    // 337.3 on the bench's two — not the default.
    if (t.flow_kernel == 1 && !t.window_indexed && !t.window_strided) {
        if (layout_kind == LAYOUT_STRIDED)
            return a.p.stride <= 64u ? launch_flows_pipe<4, LAYOUT_STRIDED, H16>(a, chain, g, s, pc)
                                     : launch_flows_pipe<5, LAYOUT_STRIDED, H16>(a, chain, g, s, pc);
        return launch_flows_pipe<5, LAYOUT_INDEXED, H16>(a, chain, g, s, pc);
    }
    if (layout_kind == LAYOUT_STRIDED) {
        switch (t.window_strided ? t.window_strided : (a.p.stride <= 64u ? 4 : 5)) {
        case 3: return launch_chain<3, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        case 4: return launch_chain<4, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        case 8: return launch_chain<8, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        default: return launch_chain<5, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        }
    }
    // Device arenas: a line-completing window of 4 to 5 chunks (the 5-tuple
    // of an untagged v4 frame ends 26 B past byte 12's chunk, a v6 one 46 B):
    // C5 flows kernel 330 -> 326 us (fixed 5; 4 to 6 chunks 367, 3 to 5 392;
    // round 2, interleaved, profiles/r02_window_ab.json).
    int wi = t.window_indexed;
    if (!wi && !t.host_arena && layout_kind == LAYOUT_INDEXED) wi = 1045;
    if (wi > 20 && wi != 100) {  // line-completing windows (ParseArgs::linewin)
        FlowArgs b = a;
        b.p.linewin = wi > 1000 ? (uint32_t)(wi - 1000) / 10u : 2u;
        switch (wi > 1000 ? (wi - 1000) % 10 : wi - 20) {
        case 3: return launch_chain<3, LAYOUT_INDEXED, MODE>(b, chain, g, s, pc);
        case 4: return launch_chain<4, LAYOUT_INDEXED, MODE>(b, chain, g, s, pc);
        case 6: return launch_chain<6, LAYOUT_INDEXED, MODE>(b, chain, g, s, pc);
        case 8: return launch_chain<8, LAYOUT_INDEXED, MODE>(b, chain, g, s, pc);
        default: return launch_chain<5, LAYOUT_INDEXED, MODE>(b, chain, g, s, pc);
        }
    }
    switch (wi ? wi : 5) {
    case 3: return launch_chain<3, LAYOUT_INDEXED, MODE>(a, chain, g, s, pc);
    case 4: return launch_chain<4, LAYOUT_INDEXED, MODE>(a, chain, g, s, pc);
    case 6: return launch_chain<6, LAYOUT_INDEXED, MODE>(a, chain, g, s, pc);
    default: return launch_chain<5, LAYOUT_INDEXED, MODE>(a, chain, g, s, pc);
    }
}

hipError_t launch_flows(const FlowArgs& a, int layout_kind, int chain, const Tuning& t,
                        hipStream_t s) {
    if (a.p.n == 0) return hipSuccess;
    // With a table built per block, the grid is persistent: exactly the
    // blocks the device holds at once (resident_per_cu, per kernel instance),
    // each wave walking tiles.  Measured on C5 (round 1, 32-bit table built
    // per block; parse+hash+histogram, us per step): one tile per wave 546,
    // 4 blocks per CU 434, 5 per CU 402, 6 / 8 per CU (a second partial
    // round) 511 / 443.  A double-buffered variant
    // (next tile staged while hashing, 3 blocks per CU for its two images)
    // measured 526 vs 454 at the time.
    // Bins <= 65,536 and no full hash requested: the 16-bit table
    // (OUT_FLOWS16) suffices — the flow bins are identical.
    const bool h16 = t.flow_table != 32 && a.bin_mask <= 0xffffu && !a.hash;
    return h16 ? launch_flows_mode<OUT_FLOWS16>(a, layout_kind, chain, t, s)
               : launch_flows_mode<OUT_FLOWS>(a, layout_kind, chain, t, s);
}

template <uint32_t DEPTH, int MODE>
hipError_t launch_ring_chain(const RingArgs& a, int chain, uint32_t grid, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_parse_ring<4, DEPTH, INGOT_CHAIN_UDP_PARSER, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_parse_ring<4, DEPTH, INGOT_CHAIN_GENERIC_ULP, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL((k_parse_ring<4, DEPTH, INGOT_CHAIN_VLAN_ULP, MODE>), dim3(grid),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// The ring consumer's grid is persistent: blocks per CU x CUs (default 2,
// like the single-batch ring kernel), capped at one tile per wave.  Cache
// policy as k_parse_pipe's (nt staging loads; 16-B records stored sc1).
hipError_t launch_ring(const RingArgs& args, int chain, int mode, const Tuning& t,
                       hipStream_t s) {
    RingArgs a = args;
    if (a.nbatches == 0 || a.n == 0) return hipSuccess;
    if (t.cache_policy == 0) a.policy = mode == OUT_REC16 ? 11u : 3u;
    else a.policy = (uint32_t)t.cache_policy & 0x1fbu;
    const uint64_t total = (uint64_t)a.tiles_per_batch * a.nbatches;
    const uint64_t bpc = t.ring_grid ? (uint64_t)t.ring_grid : 2ull;
    uint64_t blocks = (total + WAVES - 1) / WAVES;
    if (blocks > bpc * t.cus) blocks = bpc * t.cus;
    const uint32_t g = (uint32_t)(blocks ? blocks : 1);
    const bool r8 = mode == OUT_REC8;
    switch (t.pipe_depth) {
    case 3: return r8 ? launch_ring_chain<3, OUT_REC8>(a, chain, g, s)
                      : launch_ring_chain<3, OUT_REC16>(a, chain, g, s);
    case 4: return r8 ? launch_ring_chain<4, OUT_REC8>(a, chain, g, s)
                      : launch_ring_chain<4, OUT_REC16>(a, chain, g, s);
    default: return r8 ? launch_ring_chain<2, OUT_REC8>(a, chain, g, s)
                       : launch_ring_chain<2, OUT_REC16>(a, chain, g, s);
    }
}

bool tuning_valid(int key, int value) {
    switch (key) {
    case INGOT_TUNE_RING_GRID:
        return value >= 0 && value <= 8;
    case INGOT_TUNE_WINDOW_INDEXED:  // 20 + k: line-completing, up to k chunks
        return value == 0 || (value >= 2 && value <= 6) || value == 8 || value == 9 ||
               value == 100 || (value >= 22 && value <= 26) || value == 28 || value == 29 ||
               (value > 1000 && value < 1100 && (value - 1000) / 10 >= 1 &&
                (value - 1000) / 10 <= (value - 1000) % 10 &&
                ((value - 1000) % 10 >= 2 && (value - 1000) % 10 != 7));
    case INGOT_TUNE_WINDOW_STRIDED:
        return value == 0 || (value >= 2 && value <= 5) || value == 8 || value == 100;
    case INGOT_TUNE_MAX_BLOCKS:
        return value >= 0;
    case INGOT_TUNE_PIPELINE:
        return value >= 0 && value <= 64;
    case INGOT_TUNE_CACHE_POLICY:  // 0-4, or bits 0-1 with store (3-5) / load (6-8) variants
        return (value >= 0 && value <= 4) ||
               (value >= 8 && value < 512 && ((value >> 3) & 7) <= 5 && ((value >> 6) & 7) <= 6);
    case INGOT_TUNE_PIPE_DEPTH:
        return value == 0 || (value >= 2 && value <= 4);
    case INGOT_TUNE_WRITEBACK:
        return value == 0 || value == 16 || value == 32 || value == 64;
    case INGOT_TUNE_FLOW_TABLE:
        return value == 0 || value == 16 || value == 32;
    case INGOT_TUNE_SLOW_PATH:
        return value == 0 || value == 1;
    case INGOT_TUNE_READ_PLAN:
        return (value >= 0 && value <= 11);
    case INGOT_TUNE_FLOW_KERNEL:
        return value >= 0 && value <= 2;
    default:
        return false;
    }
}

}  // namespace ingot_gpu
