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
#include "walk.h"

namespace ingot_gpu {
namespace {

template <uint32_t NCH, int LAYOUT, int CHAIN, int MODE, class ARGS>
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
        : RECM && (LAYOUT == LAYOUT_INDEXED || LAYOUT == LAYOUT_PACKED) ? INGOT_REC_SKIP
                                                                                  : 0u;
    static_assert(SKIP <= 12u, "the walk reads the ethertype at frame byte 12");

    const uint64_t tstep = (uint64_t)gridDim.x * WAVES;
    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles; t += tstep) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        uint64_t off;
        uint32_t len;
        if constexpr (LAYOUT == LAYOUT_STRIDED) {
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

        Frame<NCH> fr{(const lds_u32*)wimg, lane, sh - SKIP, take, len, a.arena + off};
        Rec r;
        if constexpr (MODE == OUT_FIELDS) {
            // ingot_fields, or ingot_geneve_fields (inner + outer) for the tunnel.
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
                    for (uint32_t q = 0; q < WB_BYTES / 16u; ++q) st_global(dst + c + q, fr.chunk(c + q));
                }
            }
            if (valid && a.out) st_global(static_cast<uint4*>(a.out) + i, pack(r));
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
            if (valid) store_rec(static_cast<uint4*>(a.out) + i, pack(r), a.policy);
        }
        // The next tile's LDS-DMA overwrites this image: every lane's reads
        // above have returned (their values were consumed by the store).
    }
}

// persist_cus != 0: a persistent grid, capped at the blocks the device holds
// at once (cus x resident_per_cu), so no CU runs a second partial round.
template <uint32_t NCH, int LAYOUT, int MODE, class ARGS>
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
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_UDP_PARSER, MODE, ARGS>);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_GENERIC_ULP, MODE, ARGS>);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        go(k_parse<NCH, LAYOUT, INGOT_CHAIN_VLAN_ULP, MODE, ARGS>);
        break;
    default:
        if constexpr (MODE == OUT_REC8) {
            return hipErrorInvalidValue;  // not offered for the tunnel (api.cpp)
        } else {
            go(k_parse<NCH, LAYOUT, INGOT_CHAIN_GENEVE_OVER_V6, MODE, ARGS>);
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
    // A/B, history/profiles/r02_store_scope_ab.json); 8-B records, the rewrite ring
    // and the packed / slotted kernels gain nothing from it (or lose: C3 sc1
    // without nt 588 -> 608 us).  4 = plain loads and stores.
    const bool ring = t.pipeline != 1 && !t.window_strided && layout_kind == LAYOUT_STRIDED &&
                      !a.len && chain != INGOT_CHAIN_GENEVE_OVER_V6 && a.stride >= 64u &&
                      (a.stride == 64u || !t.host_arena) &&
                      (mode == OUT_REC16 || mode == OUT_REC8);
    if (t.cache_policy == 0) a.policy = mode == OUT_FIELDS ? 0u : ring ? (mode == OUT_REC16 ? 11u : 3u) : 2u;
    else a.policy = (uint32_t)t.cache_policy & 0x1fbu;
    const uint32_t g = grid_for(a.n, t.max_blocks);
    if (layout_kind == LAYOUT_SEGMENTED) return launch_segmented(a, chain, mode, t, g, s);
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
    if (ring) return launch_slot_ring(a, chain, mode, t, s);
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
    // 553, C4 302 -> 288 (round 2, interleaved; history/profiles/r02_window_ab.json).
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
        !tun && a.p.stride >= 64u)
        return launch_modify_ring(a, chain, t, s);
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
template <int MODE>
hipError_t launch_flows_mode(const FlowArgs& a, int layout_kind, int chain, const Tuning& t,
                             hipStream_t s) {
    const uint32_t g = grid_for(a.p.n, t.max_blocks);
    constexpr bool H16 = MODE == OUT_FLOWS16;
    // The 16-bit table comes with the kernel arguments (a block loads it in
    // one 16-B load per thread), so the default grid is one tile per wave like
    // the plain parse, the hardware dispatcher refilling CUs as blocks finish:
    // C5 flows kernel 314.8 us vs 329.5 persistent (plain parse of the same
    // frames 312.8; history/profiles/r02_flows_grid_ab.json).  The 32-bit table is
    // built per block (1,152 entries from the key windows), so its grid is
    // persistent; INGOT_TUNE_FLOW_KERNEL = 2 makes the 16-bit one persistent
    // too.  Fixed max_blocks: grid-stride over that many blocks.
    // Offset-addressed device frames, 16-bit table (the C5 case):
    // k_flows_bits (tuple.hip): the plain parse's staging and walk, the
    // address block's source chosen per lane, and the Toeplitz hash bit by
    // bit from the key windows in SGPRs — no table, so the 5-chunk images fit
    // 8 blocks per CU like the plain parse.  Measured on C5 in six
    // interleaved runs: 1.3-2.2% faster than a table-in-image kernel, itself
    // 6-7% faster than this file's k_parse flows mode; 1.07-1.09x the plain
    // parse (profiles/r04_c5_table_free_hash_ab.json; the losing variants
    // are in git history).
    const bool tuple_ok = H16 && layout_kind == LAYOUT_INDEXED && !t.host_arena &&
                          !t.window_indexed && chain != INGOT_CHAIN_GENEVE_OVER_V6;
    if (tuple_ok) return launch_flows_tuple(a, chain, t, s);
    // Otherwise k_parse's flows mode (the full 32-bit hash, the tunnel chain,
    // slots, host arenas, explicit windows): one tile per wave with the
    // 16-bit table, a persistent grid with the 32-bit one (built per block).
    const uint32_t pc = t.max_blocks || H16 ? 0u : t.cus;
    if (layout_kind == LAYOUT_STRIDED) {
        switch (t.window_strided ? t.window_strided : (a.p.stride <= 64u ? 4 : 5)) {
        case 3: return launch_chain<3, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        case 4: return launch_chain<4, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        case 8: return launch_chain<8, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        default: return launch_chain<5, LAYOUT_STRIDED, MODE>(a, chain, g, s, pc);
        }
    }
    // Device arenas: a line-completing window of 5 to 6 chunks (the 5-tuple
    // of an untagged v4 frame ends 26 B past byte 12's chunk, a v6 one 46 B,
    // and an IPv6 EH chain's ports later): the C5 flows kernel, interleaved
    // beside the 4-to-5 window of rounds 2-3 on three boxes, 358.0 -> 350.8,
    // 356.9 -> 349.3, 362.6 -> 350.9 us (-2..-3%; profiles/r03_c5_*_ab.json,
    // r04_c5_window_ab.json) at equal PMC bytes (210.5 B/frame): fewer lanes
    // read EH / port bytes past the window one by one, although 6-chunk
    // images fit 6 blocks per CU instead of 7.  4-to-6 windows: 367 (round 2).
    int wi = t.window_indexed;
    if (!wi && !t.host_arena && layout_kind == LAYOUT_INDEXED) wi = 1056;
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

hipError_t launch_flows(const FlowArgs& args, int layout_kind, int chain, const Tuning& t,
                        hipStream_t s) {
    if (args.p.n == 0) return hipSuccess;
    FlowArgs a = args;
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

bool tuning_valid(int key, int value) {
    switch (key) {
    case INGOT_TUNE_RING_GRID:
        return value >= 0 && value <= 8;
    case INGOT_TUNE_RING_GROUPS:
        return value == 0 || value == 1 || value == 2 || value == 4;
    case INGOT_TUNE_XCD_REMAP:
        return value >= 0 && value <= 5;
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
    case INGOT_TUNE_SLOW_PATH:  // per-lane loads past the window only (the others: git history)
        return value == 0;
    case INGOT_TUNE_READ_PLAN:
        return value == 0 || value == 1 || value == 11 || value == 17;
    case INGOT_TUNE_FLOW_KERNEL:  // 15 = the default, k_flows_bits
        return value == 0 || value == 15;
    default:
        return false;
    }
}

}  // namespace ingot_gpu
