// read.hip — parse_read over chunk lists (ingot_gpu_parse_read*,
// ingot-macros/src/parse.rs:511-537): the k_parse_read kernel with the header
// chunks staged in LDS (SegFrameP) and its launcher; DESIGN.md §1b.
#include "walk.h"

namespace ingot_gpu {
namespace {

// parse_read over chunk lists with chunk 0 staged (SegFrameP): per tile, the
// packets' chunk bounds and the first four chunks' descriptors are loaded
// together (independent loads), chunk 0 is staged packet-major like a frame
// window (with any later non-final chunk that lies inside that window), then
// the walk — no dependent descriptor or byte load for headers inside staged
// pieces.  One 64-packet tile per wave.  (Staging later chunks in planes, a
// persistent grid with a descriptor lookahead and fewer prefetched
// descriptors all measured slower — DESIGN.md §1b; git history, round 4.)
//
// NPRE (0 or 3): descriptors of chunks 1..NPRE loaded with chunk 0's (when
// not the packet's last); later chunks are looked up when the walk reaches
// them.
//
// FIRST (ingot_gpu_parse_read_first): chunk 0's descriptor comes from the
// per-packet array a.first, indexed by the packet like pkt_seg, so it is
// loaded together with the chunk bounds — one HBM round trip before the
// staging instead of two (pkt_seg, then the chunk table at pkt_seg[i]).
//
// LAZY (with FIRST; INGOT_TUNE_READ_PLAN 17): the chunk bounds are not
// loaded per tile at all — chunk 0 comes from a.first — but by the walk, per
// lane, only when it needs them (SegFrameP::bounds): one descriptor stream
// (8 B per packet) instead of two for packets whose headers lie in chunk 0.
template <int CS0, int CHAIN, int MODE, bool DENSE = false, int NPRE = 3, bool FIRST = false,
          bool LAZY = false>
__global__ __launch_bounds__(BLOCK) void k_parse_read(ParseArgs a) {
    static_assert(!LAZY || (FIRST && NPRE == 0), "lazy bounds: chunk 0 per packet, no prefetch");
    using FR = SegFrameP<CS0, DENSE, NPRE, LAZY>;
    constexpr uint32_t WAVE_DW = WAVE * CS0 * 4u;
    constexpr bool TUN = CHAIN == INGOT_CHAIN_GENEVE_OVER_V6;
    // no slack past the last image: SegFrameP::be clamps the second dword of
    // a pair to the current chunk's staged pieces (a 5-piece image is then
    // exactly 20 KiB per block)
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint64_t W = (uint64_t)gridDim.x * WAVES;
    uint64_t t = (uint64_t)blockIdx.x * WAVES + wave;
    if (t >= ntiles) return;

    // packet i's chunk bounds (clamped index: always one load pair); LAZY:
    // none yet (FR::kUnknown for a packet of the batch, 0 past its end)
    auto load_pkt = [&](uint64_t tt, uint32_t& s0, uint32_t& ns) {
        uint64_t i = tt * WAVE + lane;
        const bool v = i < a.n;
        if constexpr (LAZY) {
            s0 = 0;
            ns = v ? FR::kUnknown : 0u;
            return;
        }
        if (!v) i = a.n - 1u;
        const uint32_t b0 = a.pkt_seg[i], b1 = a.pkt_seg[i + 1];
        s0 = v ? b0 : 0u;
        ns = v ? b1 - b0 : 0u;
    };
    // chunk 0's descriptor (none for a packet without chunks)
    auto load_d0 = [&](uint32_t s0, uint32_t ns, uint64_t& o0, uint32_t& l0) {
        if constexpr (DENSE) {
            const uint64_t v = ns ? a.off[s0] : 0u;
            o0 = v >> 16;
            l0 = (uint32_t)(v & 0xffffu);
        } else {
            o0 = ns ? a.off[s0] : 0u;
            l0 = ns ? a.len[s0] : 0u;
        }
    };
    // FIRST: chunk 0's (offset << 16) | length of packet tt's lane, loaded
    // beside its bounds (clamped index: always one load)
    auto load_first = [&](uint64_t tt, uint32_t ns, uint64_t& o, uint32_t& l) {
        uint64_t i = tt * WAVE + lane;
        if (i >= a.n) i = a.n - 1u;
        const uint64_t v = a.first[i];
        o = ns ? v >> 16 : 0u;  // (LAZY: ns is kUnknown for every packet of the batch)
        l = ns ? (uint32_t)(v & 0xffffu) : 0u;
    };
    uint32_t s0, nseg;
    uint64_t o0;
    uint32_t l0;
    load_pkt(t, s0, nseg);
    if constexpr (FIRST) load_first(t, nseg, o0, l0);
    else load_d0(s0, nseg, o0, l0);

    for (;;) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        FR fr;
        fr.o0 = o0;
        fr.l0 = l0;
        if constexpr (DENSE) {
            // one 8-B entry per chunk: (offset << 16) | length; chunks 1..3
            // only when not the packet's last (SegFrameP::advance)
            const uint64_t v1 = nseg > 2 ? a.off[s0 + 1] : 0u;
            const uint64_t v2 = nseg > 3 ? a.off[s0 + 2] : 0u;
            const uint64_t v3 = nseg > 4 ? a.off[s0 + 3] : 0u;
            fr.o1 = v1 >> 16;
            fr.o2 = v2 >> 16;
            fr.o3 = v3 >> 16;
            fr.l1 = (uint32_t)(v1 & 0xffffu);
            fr.l2 = (uint32_t)(v2 & 0xffffu);
            fr.l3 = (uint32_t)(v3 & 0xffffu);
        } else {
            fr.o1 = NPRE >= 1 && nseg > 2 ? a.off[s0 + 1] : 0u;
            fr.o2 = NPRE >= 2 && nseg > 3 ? a.off[s0 + 2] : 0u;
            fr.o3 = NPRE >= 3 && nseg > 4 ? a.off[s0 + 3] : 0u;
            fr.l1 = NPRE >= 1 && nseg > 2 ? a.len[s0 + 1] : 0u;
            fr.l2 = NPRE >= 2 && nseg > 3 ? a.len[s0 + 2] : 0u;
            fr.l3 = NPRE >= 3 && nseg > 4 ? a.len[s0 + 3] : 0u;
        }
        // chunk 0, packet-major: instruction k, lane L fills slot 64k + L =
        // packet q / CS0, piece (q mod CS0) ^ swz (16-B aligned absolute
        // addresses; pieces only below the chunk's end).  Records never read
        // the MAC addresses (the walk reads Ethernet's ethertype only), so, as
        // in k_parse, the window starts at the piece holding chunk 0's byte
        // SKIP = 12: a frame starting in the last 12 bytes of a 128-B line
        // does not fetch that line.  Staged byte sh0 + j is chunk-0 byte
        // SKIP + j.
        constexpr uint32_t SKIP = MODE == OUT_REC16 ? INGOT_REC_SKIP : 0u;
        const uint32_t sh0 = (uint32_t)((uintptr_t)(a.arena + fr.o0 + SKIP) & 15u);
        const int64_t base0 = (int64_t)fr.o0 + (int64_t)SKIP - (int64_t)sh0;
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
        // the window's end in staged bytes: chunk 0's end, or the window's
        // (nothing when chunk 0 ends before byte SKIP)
        const int64_t e0 = (int64_t)sh0 + (int64_t)fr.l0 - (int64_t)SKIP;
        uint32_t ext = nseg && e0 > 0 ? (e0 < (int64_t)wlim ? (uint32_t)e0 : wlim) : 0u;
        // a later non-last chunk that starts inside chunk 0's window: stage
        // the window's pieces up to its end (or the window's)
        auto widen = [&](uint32_t e, uint64_t o, uint32_t l) {
            const int64_t d = (int64_t)o - base0;
            if (e + 1 < nseg && d >= 0 && d < (int64_t)wlim) {
                const uint32_t end = (uint32_t)d + l < wlim ? (uint32_t)d + l : wlim;
                ext = end > ext ? end : ext;
            }
        };
        if constexpr (NPRE >= 1) widen(1, fr.o1, fr.l1);
        if constexpr (NPRE >= 2) widen(2, fr.o2, fr.l2);
        if constexpr (NPRE >= 3) widen(3, fr.o3, fr.l3);
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
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        fr.win = (const lds_u32*)wimg;
        fr.p = lane;
        fr.arena = a.arena;
        fr.seg_off = a.off;
        fr.seg_len = a.len;
        fr.s0 = s0;
        fr.k = 0;
        fr.nseg = nseg;
        fr.pkt_seg = a.pkt_seg;
        fr.pi = i;
        fr.L = 0;
        fr.b0 = base0;
        fr.span0 = 16u * n0;
        fr.enter(fr.o0, fr.l0, nseg ? want : 0u);
        if constexpr (SKIP != 0) {
            // chunk-0 byte i >= SKIP is staged byte i + sh0 - SKIP (mod 2^32);
            // bytes [0, avail) count as staged (those below SKIP are never read)
            fr.sh = sh0 - SKIP;
            const uint32_t w0 = 16u * want + SKIP - sh0;
            fr.avail = nseg ? (fr.l0 < w0 ? fr.l0 : w0) : 0u;
        }
        Rec r;
        if constexpr (MODE == OUT_FIELDS) {
            using OutT = typename std::conditional<TUN, ingot_geneve_fields, ingot_fields>::type;
            OutT* G = static_cast<OutT*>(a.out) + (valid ? i : 0);
            if (valid) {
                uint4* z = reinterpret_cast<uint4*>(G);
#pragma unroll
                for (int k = 0; k < (int)(sizeof(OutT) / 16); ++k) st_global(z + k, make_uint4(0, 0, 0, 0));
                ingot_fields* F;
                ingot_tunnel_fields* T = nullptr;
                if constexpr (TUN) {
                    F = &G->inner;
                    T = &G->outer;
                } else {
                    F = G;
                }
                walk<CHAIN, true>(fr, r, F, T);
                st_global(reinterpret_cast<uint4*>(F), pack(r));
            }
        } else {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            if (valid) store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        }
        if (valid && a.chunk) a.chunk[i] = (uint16_t)fr.k;
        // the next tile's LDS-DMA overwrites this image: every lane's reads
        // above have returned (their values were consumed by the stores)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t += W;
        if (t >= ntiles) break;
        load_pkt(t, s0, nseg);
        if constexpr (FIRST) load_first(t, nseg, o0, l0);
        else load_d0(s0, nseg, o0, l0);
    }
}

template <int CS0, int MODE, bool DENSE = false, int NPRE = 3, bool FIRST = false,
          bool LAZY = false>
hipError_t launch_read(const ParseArgs& a, int chain, uint32_t g, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_parse_read<CS0, INGOT_CHAIN_UDP_PARSER, MODE, DENSE, NPRE, FIRST, LAZY>),
                           dim3(g), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_parse_read<CS0, INGOT_CHAIN_GENERIC_ULP, MODE, DENSE, NPRE, FIRST, LAZY>),
                           dim3(g), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL((k_parse_read<CS0, INGOT_CHAIN_VLAN_ULP, MODE, DENSE, NPRE, FIRST, LAZY>),
                           dim3(g), dim3(BLOCK), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL(
            (k_parse_read<CS0, INGOT_CHAIN_GENEVE_OVER_V6, MODE, DENSE, NPRE, FIRST, LAZY>), dim3(g),
            dim3(BLOCK), 0, s, a);
        break;
    }
    return hipGetLastError();
}

}  // namespace

// parse_read over chunk lists.  Measured (tools/abtune.py, us per launch,
// DESIGN.md §1b): the reference's one-header-per-chunk shape (c2r, 1 M) 33.3
// with descriptors and bytes on demand / 25.1 with chunk 0 in 4 pieces /
// 24.2 with later chunks in planes {2,2,2,0}; header + payload chunks (c3r,
// 16.7 M) 651 / 667 / 681 — extra planes cost occupancy on the
// gather-bound shape.  Default (round 2): chunk 0 in a line-completing window
// of 3 to 5 pieces (to the end of the 128-B line its third piece lies in;
// k_parse's windows): c3r 676 -> 651 us, c2r 23.05 -> 23.24.
// INGOT_TUNE_READ_PLAN 1 = the round-1 4-piece window (the default for chunk
// pools in mapped host memory, where every staged piece is a PCIe read).
hipError_t launch_segmented(const ParseArgs& a, int chain, int mode, const Tuning& t,
                            uint32_t g, hipStream_t s) {
    if (mode != OUT_FIELDS && mode != OUT_REC16) return hipErrorInvalidValue;
    // dense chunk table (ingot_gpu_parse_read_dense): no length array, one
    // (offset << 16) | length entry per chunk; 4 pieces of chunk 0 (the
    // knob does not apply)
    if (!a.len)
        return mode == OUT_FIELDS ? launch_read<4, OUT_FIELDS, true>(a, chain, g, s)
                                  : launch_read<4, OUT_REC16, true>(a, chain, g, s);
    // chunk 0's descriptor per packet (ingot_gpu_parse_read_first): loaded
    // beside the bounds; 17 = the bounds loaded lazily by the walk
    if (a.first) {
        if (mode == OUT_FIELDS)
            return launch_read<4, OUT_FIELDS, false, 3, true>(a, chain, g, s);
        if (t.host_arena || t.read_plan == 1)
            return launch_read<4, OUT_REC16, false, 3, true>(a, chain, g, s);
        ParseArgs b = a;
        b.linewin = 3u;
        if (t.read_plan == 17)
            return launch_read<5, OUT_REC16, false, 0, true, true>(b, chain, g, s);
        return launch_read<5, OUT_REC16, false, 3, true>(b, chain, g, s);
    }
    if (mode == OUT_FIELDS) return launch_read<4, OUT_FIELDS>(a, chain, g, s);
    if (t.read_plan == 1 || (t.read_plan == 0 && t.host_arena))
        return launch_read<4, OUT_REC16>(a, chain, g, s);
    ParseArgs b = a;  // 0 / 11 / 17 (17 applies to parse_read_first only)
    b.linewin = 3u;
    return launch_read<5, OUT_REC16>(b, chain, g, s);
}

}  // namespace ingot_gpu
