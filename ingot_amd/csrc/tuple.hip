// tuple.hip — config 5's flow classification kernel,
// k_flows_bits: the plain parse's 4-5 chunk window (line-completing from the
// chunk holding byte 12) and walk, the hash input words read per lane from
// the window or, for a lane whose address block lies past it, from L2, and
// the Toeplitz hash computed bit by bit from the key windows in SGPRs — no
// table, so the block's LDS is its window images (8 blocks per CU) and no
// tile copies a table.  The variants it beat (ballot / prefix-scan compacted
// 5-tuple fetch, table copied into each wave's image) are in git history
// (round 4); DESIGN.md §4.4 has their numbers.
// Records are not written (flow ids only), exactly as k_parse's flows mode.
#include "walk.h"

namespace ingot_gpu {
namespace {

// The table-free flows kernel: the plain parse's staging and walk, the
// address block's source chosen per lane (flow_words `lanes`), and the hash
// computed bit by bit from the key windows in SGPRs (toeplitz9_bits16): no
// LDS table, no LDS reads for the hash; the images are the block's only LDS
// (20 KiB, 8 blocks per CU).
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
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_UDP_PARSER>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_GENERIC_ULP>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    default:
        hipLaunchKernelGGL((k_flows_bits<NCH, INGOT_CHAIN_VLAN_ULP>), dim3(g),
                           dim3(BLOCK), 0, s, a);
        break;
    }
    return hipGetLastError();
}

}  // namespace

// Offset-addressed frames in device memory, 16-bit bins, not the tunnel
// (launch_flows checks): k_flows_bits over 4-5 chunk windows.
hipError_t launch_flows_tuple(const FlowArgs& args, int chain, const Tuning& t, hipStream_t s) {
    FlowArgs a = args;
    a.p.linewin = 4u;  // at least 4 chunks from byte 12's, then to the 128-B line end (<= 5)
    return go_bits<5>(a, chain, grid_for(a.p.n, t.max_blocks), s);
}

}  // namespace ingot_gpu
