// tuple.hip — config 5's flow classification kernels:
//   * k_flows_bits (INGOT_TUNE_FLOW_KERNEL 15, the default for
//     offset-addressed device frames): the plain parse's 5-chunk window and
//     walk, and the Toeplitz hash computed bit by bit from the key windows in
//     SGPRs — no table, so the block's LDS is its window images (8 blocks per
//     CU) and no tile copies a table;
//   * k_flows_imgtab (10-13; 13 the round-4 default before it): the table
//     copied into each wave's image per tile instead of a block-wide LDS copy;
//   * k_flows_tuple (4-9, A/B): the 5-tuple's chunks past the window
//     fetched by a wavefront ballot + prefix scan, described here.
//
// The flows kernel needs bytes the plain parse never reads: the IPv6
// addresses (frame bytes 22..54 behind 0-2 VLAN tags) and the L4 ports.
// k_parse<…, OUT_FLOWS16> stages a wider window for every lane (4..5 chunks,
// line-completing) so that most lanes find them in LDS; every lane of every
// wave pays for the lines only some of them need.  Here each wave stages
// exactly the plain parse's window (2..NCH chunks, line-completing from the
// chunk holding byte 12), then:
//   1. every lane computes the 16-B chunks of its 5-tuple span past its
//      window (EARLY: speculatively from the window's first bytes — Ethernet,
//      VLAN tags, IPv4 ihl / protocol, IPv6 next header — before the walk;
//      LATE: exactly, from the walk's record);
//   2. a wavefront prefix scan of the per-lane chunk counts gives each lane
//      its slots in a per-wave overflow image, compacted (no holes);
//   3. one LDS-DMA instruction per 64 slots fetches them: slot q's owner lane
//      is found by a 6-step binary search over the inclusive scan (shuffles),
//      so every instruction fills up to 64 slots whatever the lanes' counts;
//   4. the walk runs (EARLY: while the overflow DMA is in flight), then the
//      hash reads each dword of the tuple from the window, the overflow image,
//      or (a chunk past both: an IPv6 EH chain's ports, or an overflow image
//      already full) L2/HBM.
// Records are not written (flow ids only), exactly as k_parse's flows mode.
#include "walk.h"

namespace ingot_gpu {
namespace {

// EARLY: the 5-tuple's frame-byte span [start, end) as far as the window's
// first bytes tell — the addresses, and the ports when the L4 header follows
// the L3 header directly (IPv4 after its options, IPv6 without extension
// headers).  Only a fetch hint: the hash reads whatever it needs wherever it
// lies, so a span that turns out wrong costs bytes, never results.
template <int CHAIN, class FR>
__device__ __forceinline__ void tuple_span_early(const FR& f, uint32_t& start, uint32_t& end) {
    start = end = 0;
    const uint32_t len = f.len;
    if (len < eth::LEN) return;
    uint32_t et = f.get(0, eth::ethertype);
    uint32_t p = eth::LEN;
    if constexpr (CHAIN == INGOT_CHAIN_VLAN_ULP) {
        for (uint32_t v = 0; v < 2u && (et == ET_VLAN || et == ET_QINQ); ++v) {
            if (len - p < vlan::LEN) return;
            et = f.get(p, vlan::ethertype);
            p += vlan::LEN;
        }
    }
    if (et == ET_IPV4) {
        if (len - p < ipv4::LEN) return;
        const uint32_t ihl = f.get(p, ipv4::ihl);
        const uint32_t hl = ihl * 4u > ipv4::LEN ? ihl * 4u : ipv4::LEN;
        const uint32_t proto = f.get(p, ipv4::protocol);
        start = p + 12u;
        end = proto == IPP_TCP || proto == IPP_UDP ? p + hl + 4u : p + ipv4::LEN;
    } else if (et == ET_IPV6) {
        if (len - p < ipv6::LEN) return;
        const uint32_t nh = f.get(p, ipv6::next_header);
        start = p + ipv6::SOURCE_BYTE;
        end = nh == IPP_TCP || nh == IPP_UDP ? p + ipv6::LEN + 4u : p + ipv6::LEN;
    }
    if (end > len) end = len;
}

// LATE: the exact span from a parsed-Ok record — the address block, and the
// ports when they lie within 64 B of its start (else only the addresses; the
// port word is then read on its own).
__device__ __forceinline__ void tuple_span_late(const Rec& r, uint32_t& start, uint32_t& end) {
    start = end = 0;
    if (r.status != INGOT_OK || r.l3_kind == INGOT_L3_NONE) return;
    const bool v6 = r.l3_kind == INGOT_L3_IPV6;
    start = r.l3_off + (v6 ? ipv6::SOURCE_BYTE : 12u);
    end = start + (v6 ? 32u : 8u);
    const bool ports = r.l4_kind == INGOT_L4_TCP || r.l4_kind == INGOT_L4_UDP;
    if (ports && r.l4_off + 4u - start <= 64u && r.l4_off + 4u > end) end = r.l4_off + 4u;
}

template <uint32_t NCH, uint32_t OVF, bool EARLY, int CHAIN>
__global__ __launch_bounds__(BLOCK) void k_flows_tuple(FlowArgs args) {
    // OVF = 0: no overflow image — a lane's missing chunks go to the slots
    // of its own window image its window left free (LATE only: the walk is
    // done with the image by then)
    static_assert(OVF % WAVE == 0 && (OVF >= WAVE || !EARLY), "whole LDS-DMA instructions");
    const ParseArgs& a = args.p;
    constexpr uint32_t SKIP = 12u;  // windows from the chunk holding the ethertype
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW];
    __shared__ __attribute__((aligned(16))) uint32_t s_ovf[OVF ? WAVES * OVF * 4u : 4u];
    __shared__ __attribute__((aligned(32))) uint32_t s_tab[FLOW_TAB16];
    load_flow_table16(s_tab, args.tab16);
    __syncthreads();

    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* wimg = s_win + wave * WAVE_DW;
    uint32_t* ovf = s_ovf + wave * OVF * 4u;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint32_t mis = (uint32_t)((uintptr_t)a.arena & 31u);
    const uint64_t tstep = (uint64_t)gridDim.x * WAVES;

    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles; t += tstep) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        const uint64_t off = valid ? a.off[i] : 0u;
        const uint32_t len = valid ? (uint32_t)a.len[i] : 0u;
        // the plain parse's window (k_parse, line-completing from byte 12)
        const uint32_t sh = (uint32_t)((off + SKIP + mis) & 15u);
        const int64_t base = (int64_t)off + (int64_t)SKIP - (int64_t)sh;
        uint32_t wend = SKIP + 16u * NCH - sh;
        if (a.linewin) {
            const uint32_t lp = (uint32_t)((uintptr_t)(a.arena + base) >> 4) & 7u;
            uint32_t want = ((lp + a.linewin + 7u) & ~7u) - lp;
            if (want > NCH) want = NCH;
            wend = SKIP + 16u * want - sh;
        }
        const uint32_t take = len < wend ? len : wend;
        const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
        const uint32_t nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
        // every lane's reads of both images (previous tile) have returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
            const int64_t bp = (int64_t)__shfl((long long)base, (int)pp);
            if (c < np) stage16(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        Frame<NCH> fr{(const lds_u32*)wimg, lane, sh - SKIP, take, len, a.arena + off};
        // the 5-tuple's chunks past the window: c0 .. c0+m-1 (staged chunk
        // coordinates: chunk c lies at arena + base + 16 c; the window is
        // chunks 0 .. nch-1 and ends on a chunk boundary unless it ends the
        // frame, in which case nothing lies past it)
        uint32_t c0 = 0, m = 0, S = 0;
        bool ok = false;
        Rec r;
        auto fetch = [&](uint32_t start, uint32_t end) {
            if (end > take) {
                const uint32_t from = start > take ? start : take;
                c0 = (fr.sh + from) >> 4;
                m = ((fr.sh + end - 1u) >> 4) - c0 + 1u;
            }
            if constexpr (OVF == 0) {
                // into the lane's own free slots (logical chunks nch ..
                // NCH - 1 of its image): row k, lane L fills slot 64k + L =
                // packet pp's logical chunk c, as the staging did
                ok = nch + m <= NCH;
#pragma unroll
                for (uint32_t k = 0; k < NCH; ++k) {
                    const uint32_t q = k * WAVE + lane;
                    const uint32_t pp = q / NCH;
                    const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
                    const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
                    const uint32_t mp = (uint32_t)__shfl((int)m, (int)pp);
                    const uint32_t cp = (uint32_t)__shfl((int)c0, (int)pp);
                    const int64_t bp = (int64_t)__shfl((long long)base, (int)pp);
                    if (c >= np && c - np < mp && np + mp <= NCH)
                        stage16(a.arena + bp + 16u * (cp + c - np), wimg + k * WAVE * 4u, false);
                }
                return;
            }
            // wavefront prefix scan of the counts: this lane's first slot
            uint32_t x = m;
#pragma unroll
            for (uint32_t d = 1; d < WAVE; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, d);
                if (lane >= d) x += y;
            }
            S = x - m;
            ok = x <= OVF;
            const uint32_t T = (uint32_t)__shfl((int)x, (int)(WAVE - 1u));
#pragma unroll
            for (uint32_t k = 0; k < OVF / WAVE; ++k) {
                if (k * WAVE >= T) break;  // wave-uniform
                const uint32_t q = k * WAVE + lane;
                // owner of slot q: the first lane whose inclusive count exceeds q
                uint32_t j = 0;
#pragma unroll
                for (uint32_t s = WAVE / 2; s; s >>= 1) {
                    const uint32_t v = (uint32_t)__shfl((int)x, (int)(j + s - 1u));
                    if (v <= q) j += s;
                }
                const uint32_t sj = (uint32_t)__shfl((int)S, (int)j);
                const uint32_t cj = (uint32_t)__shfl((int)c0, (int)j);
                const int64_t bj = (int64_t)__shfl((long long)base, (int)j);
                if (q < T) stage16(a.arena + bj + 16u * (cj + q - sj), ovf + k * WAVE * 4u, false);
            }
        };
        if constexpr (EARLY) {
            uint32_t s0, e0;
            tuple_span_early<CHAIN>(fr, s0, e0);
            fetch(s0, e0);  // in flight during the walk
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
        } else {
            walk<CHAIN, false>(fr, r, nullptr, nullptr);
            uint32_t s0, e0;
            tuple_span_late(r, s0, e0);
            fetch(s0, e0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        // dword q (staged coordinates) of this lane's frame: window, overflow
        // image, else L2/HBM (an aligned dword of the frame's own chunks)
        auto dwv = [&](uint32_t q) -> uint32_t {
            const uint32_t c = q >> 2;
            if (c < nch) return wimg[slot_of<NCH>(lane, c) * 4u + (q & 3u)];
            if (ok && c - c0 < m) {
                if constexpr (OVF == 0) return wimg[slot_of<NCH>(lane, nch + c - c0) * 4u + (q & 3u)];
                else return ovf[(S + c - c0) * 4u + (q & 3u)];
            }
            return *reinterpret_cast<const uint32_t*>(a.arena + base + 4u * q);
        };
        FlowWords x;
#pragma unroll
        for (uint32_t k = 0; k < 9; ++k) x.w[k] = 0;
        const bool counted = valid && r.status == INGOT_OK && r.l3_kind != INGOT_L3_NONE;
        if (counted) {
            const bool v6 = r.l3_kind == INGOT_L3_IPV6;
            const uint32_t naddr = v6 ? 8u : 2u;
            const uint32_t b = fr.sh + r.l3_off + (v6 ? ipv6::SOURCE_BYTE : 12u);
            const uint32_t sel = (b & 3u) * 0x01010101u + 0x00010203u;
            // the block's dwords: naddr, plus the one its last bytes spill
            // into when it is not dword-aligned (never a dword past them)
            const uint32_t nd = naddr + ((b & 3u) ? 1u : 0u);
            uint32_t d[9];
#pragma unroll
            for (uint32_t k = 0; k < 9; ++k) d[k] = k < nd ? dwv((b >> 2) + k) : 0u;
            uint32_t pw = 0;
            if (r.l4_kind == INGOT_L4_TCP || r.l4_kind == INGOT_L4_UDP) {
                const uint32_t pb = fr.sh + r.l4_off;
                const uint32_t p0 = dwv(pb >> 2);
                const uint32_t p1 = (pb & 3u) ? dwv((pb >> 2) + 1u) : 0u;
                pw = __builtin_amdgcn_perm(p1, p0, (pb & 3u) * 0x01010101u + 0x00010203u);
            }
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) {
                const uint32_t w = __builtin_amdgcn_perm(d[k + 1], d[k], sel);
                x.w[k] = k < naddr ? w : (k == naddr ? pw : 0u);
            }
            x.w[8] = naddr == 8u ? pw : 0u;
        }
        const uint32_t h = counted ? toeplitz9_16(x, s_tab) : 0u;
        if (valid) {
            args.flow[i] = counted ? (h & args.bin_mask) : INGOT_FLOW_NONE;
            if (args.hash) args.hash[i] = h;
        }
    }
}

// The table-in-image flows kernel (INGOT_TUNE_FLOW_KERNEL 10 / 11): k_parse's
// flows mode without the block's LDS copy of the Toeplitz table.  That
// 2,304-B table is what keeps the flows kernel at 7 blocks per CU where the
// plain parse's 5-chunk images fit 8 (160 KiB / 20 KiB).  Here each wave
// copies the table into its own window image after the walk, once the hash
// input words are parked in the image's tail (three 16-B loads per lane from
// the kernel arguments, cache hits after the first tiles), hashes from there,
// and the next tile's staging overwrites it.  One extra L2 round trip per tile for
// an eighth more resident waves.
template <uint32_t NCH, int CHAIN, bool LANES>
__global__ __launch_bounds__(BLOCK, 8) void k_flows_imgtab(FlowArgs args) {
    const ParseArgs& a = args.p;
    constexpr uint32_t SKIP = 12u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    static_assert(WAVE_DW >= FLOW_TAB16 + 9u * WAVE, "the table and the parked words fit");
    __shared__ __attribute__((aligned(32))) uint32_t s_win[WAVES * WAVE_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint32_t mis = (uint32_t)((uintptr_t)a.arena & 31u);
    const uint64_t tstep = (uint64_t)gridDim.x * WAVES;

    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles; t += tstep) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        const uint64_t off = valid ? a.off[i] : 0u;
        const uint32_t len = valid ? (uint32_t)a.len[i] : 0u;
        const uint32_t sh = (uint32_t)((off + SKIP + mis) & 15u);
        const int64_t base = (int64_t)off + (int64_t)SKIP - (int64_t)sh;
        uint32_t wend = SKIP + 16u * NCH - sh;
        if (a.linewin) {
            const uint32_t lp = (uint32_t)((uintptr_t)(a.arena + base) >> 4) & 7u;
            uint32_t want = ((lp + a.linewin + 7u) & ~7u) - lp;
            if (want > NCH) want = NCH;
            wend = SKIP + 16u * want - sh;
        }
        const uint32_t take = len < wend ? len : wend;
        const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
        const uint32_t nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
        // every lane's reads of the image (the previous tile's table) are done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
            const int64_t bp = (int64_t)__shfl((long long)base, (int)pp);
            if (c < np) stage16(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Frame<NCH> fr{(const lds_u32*)wimg, lane, sh - SKIP, take, len, a.arena + off};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        bool counted;
        {
            FlowWords x;
            counted = valid && flow_words(fr, r, x, LANES);
            // the image is free once every lane's reads of it have returned:
            // park the hash input words behind where the table will go
            // (word k of lane L at dword FLOW_TAB16 + 64 k + L), so that no
            // register holds them across the table's fetch
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t k = 0; k < 9; ++k) wimg[FLOW_TAB16 + k * WAVE + lane] = x.w[k];
        }
        // copy the table in (FLOW_TAB16 dwords = 144 16-B pieces) from the
        // kernel arguments: plain 16-B loads + LDS stores (the arguments are
        // not a global-address-space source for LDS-DMA)
#pragma unroll
        for (uint32_t k = 0; k < (FLOW_TAB16 / 4u + WAVE - 1u) / WAVE; ++k) {
            const uint32_t q = k * WAVE + lane;
            if (q < FLOW_TAB16 / 4u)
                reinterpret_cast<uint4*>(wimg)[q] = reinterpret_cast<const uint4*>(args.tab16)[q];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        FlowWords x;
#pragma unroll
        for (uint32_t k = 0; k < 9; ++k) x.w[k] = wimg[FLOW_TAB16 + k * WAVE + lane];
        const uint32_t h = counted ? toeplitz9_16(x, wimg) : 0u;
        if (valid) {
            args.flow[i] = counted ? (h & args.bin_mask) : INGOT_FLOW_NONE;
            if (args.hash) args.hash[i] = h;
        }
    }
}

// The table-free flows kernel (INGOT_TUNE_FLOW_KERNEL 15): k_flows_imgtab's
// staging, walk and per-lane address source, and the hash computed bit by bit
// from the key windows in SGPRs (toeplitz9_bits16): no table copy per tile
// (one L2 round trip and 2,304 B of LDS writes), no parked words, no LDS reads
// for the hash; the images are the block's only LDS (20 KiB, 8 blocks per CU).
static_assert(std::is_standard_layout<FlowArgs>::value,
              "k_flows_bits reads FlowArgs::w at offsetof() in the kernarg segment");
template <uint32_t NCH, int CHAIN>
__global__ __launch_bounds__(BLOCK, 8) void k_flows_bits(FlowArgs args) {
    const ParseArgs& a = args.p;
    constexpr uint32_t SKIP = 12u;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    uint32_t* wimg = s_win + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint32_t mis = (uint32_t)((uintptr_t)a.arena & 31u);
    const uint64_t tstep = (uint64_t)gridDim.x * WAVES;

    for (uint64_t t = (uint64_t)blockIdx.x * WAVES + wave; t < ntiles; t += tstep) {
        const uint64_t i = t * WAVE + lane;
        const bool valid = i < a.n;
        const uint64_t off = valid ? a.off[i] : 0u;
        const uint32_t len = valid ? (uint32_t)a.len[i] : 0u;
        const uint32_t sh = (uint32_t)((off + SKIP + mis) & 15u);
        const int64_t base = (int64_t)off + (int64_t)SKIP - (int64_t)sh;
        uint32_t wend = SKIP + 16u * NCH - sh;
        if (a.linewin) {
            const uint32_t lp = (uint32_t)((uintptr_t)(a.arena + base) >> 4) & 7u;
            uint32_t want = ((lp + a.linewin + 7u) & ~7u) - lp;
            if (want > NCH) want = NCH;
            wend = SKIP + 16u * want - sh;
        }
        const uint32_t take = len < wend ? len : wend;
        const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
        const uint32_t nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
        // every lane's reads of the image (previous tile) have returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
            const int64_t bp = (int64_t)__shfl((long long)base, (int)pp);
            if (c < np) stage16(a.arena + bp + 16u * c, wimg + k * WAVE * 4u, false);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        Frame<NCH> fr{(const lds_u32*)wimg, lane, sh - SKIP, take, len, a.arena + off};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        FlowWords x;
        const bool counted = valid && flow_words(fr, r, x, true);
        // the key windows in the kernel arguments (FlowArgs is the only
        // explicit argument: offset 0 of the kernarg segment, the hidden
        // arguments follow it); the pointer is made opaque per tile so that
        // the 144 windows are loaded where the hash uses them instead of held
        // in SGPRs (spilled) across the loop
        kar_u32* W = (kar_u32*)((__attribute__((address_space(4))) const uint8_t*)
                                    __builtin_amdgcn_kernarg_segment_ptr() +
                                offsetof(FlowArgs, w));
        asm volatile("" : "+s"(W));
        const uint32_t h = counted ? toeplitz9_bits16(x, W) : 0u;
        if (valid) {
            args.flow[i] = counted ? (h & args.bin_mask) : INGOT_FLOW_NONE;
            if (args.hash) args.hash[i] = h;
        }
    }
}

template <uint32_t NCH>
hipError_t go_bits(const FlowArgs& a, int chain, uint32_t g, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_UDP_PARSER>), dim3(g), dim3(BLOCK), 0,
                           s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_GENERIC_ULP>), dim3(g), dim3(BLOCK), 0,
                           s, a);
        break;
    default:
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_VLAN_ULP>), dim3(g), dim3(BLOCK), 0, s,
                           a);
        break;
    }
    return hipGetLastError();
}

template <uint32_t NCH, bool LANES = false>
hipError_t go_imgtab(const FlowArgs& a, int chain, uint32_t g, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_flows_imgtab<NCH, INGOT_CHAIN_UDP_PARSER, LANES>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_flows_imgtab<NCH, INGOT_CHAIN_GENERIC_ULP, LANES>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((k_flows_imgtab<NCH, INGOT_CHAIN_VLAN_ULP, LANES>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    }
    return hipGetLastError();
}

template <uint32_t NCH, uint32_t OVF, bool EARLY>
hipError_t go_tuple(const FlowArgs& a, int chain, uint32_t g, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_flows_tuple<NCH, OVF, EARLY, INGOT_CHAIN_UDP_PARSER>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_flows_tuple<NCH, OVF, EARLY, INGOT_CHAIN_GENERIC_ULP>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((k_flows_tuple<NCH, OVF, EARLY, INGOT_CHAIN_VLAN_ULP>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    }
    return hipGetLastError();
}

}  // namespace

// Offset-addressed frames in device memory, 16-bit table, not the tunnel
// (launch_flows checks).  variant (INGOT_TUNE_FLOW_KERNEL): 4 = EARLY, 5
// chunks (the plain parse's window), 64 overflow slots; 5 = EARLY, 4 chunks;
// 6 = LATE, 5 chunks; 7 = EARLY, 5 chunks, 128 overflow slots; 8 = LATE,
// 5 chunks, each lane's missing chunks in its own window image's free slots;
// 9 = 8 with 4-chunk windows (the table then fits 8 blocks per CU);
// 10 / 11 / 12 = k_flows_imgtab (the table copied into each wave's image per
// tile) with 4..5 / 2..5 / 3..5-chunk windows; 13 = 10 with the address
// block's source chosen per lane (flow_words `lanes`); 15 = k_flows_bits
// (13 without a table: the hash bit by bit from the key windows; the default).
hipError_t launch_flows_tuple(const FlowArgs& args, int chain, int variant, const Tuning& t,
                              hipStream_t s) {
    FlowArgs a = args;
    a.p.linewin = 2;  // the plain parse's line-completing window (2..NCH)
    const uint32_t g = grid_for(a.p.n, t.max_blocks);
    if (variant == 15) {  // no table: the hash from the key windows (SGPRs)
        a.p.linewin = 4u;
        return go_bits<5>(a, chain, g, s);
    }
    if (variant >= 10 && variant <= 13) {  // table in the image: 4..5 / 2..5 / 3..5 windows
        a.p.linewin = variant == 11 ? 2u : variant == 12 ? 3u : 4u;
        return variant == 13 ? go_imgtab<5, true>(a, chain, g, s) : go_imgtab<5>(a, chain, g, s);
    }
    switch (variant) {
    case 5: return go_tuple<4, 64, true>(a, chain, g, s);
    case 6: return go_tuple<5, 64, false>(a, chain, g, s);
    case 7: return go_tuple<5, 128, true>(a, chain, g, s);
    case 8: return go_tuple<5, 0, false>(a, chain, g, s);
    case 9: return go_tuple<4, 0, false>(a, chain, g, s);
    default: return go_tuple<5, 64, true>(a, chain, g, s);
    }
}

}  // namespace ingot_gpu
