// ring.hip — the slot-ring kernels: k_parse_pipe (one batch per launch,
// the next tile's LDS-DMA in flight while a wave parses one), k_parse_ring
// (the persistent ring consumer, ingot_gpu_parse_ring: many batches per
// launch behind an in-kernel doorbell) and k_modify_pipe (parse + setters in
// place); DESIGN.md §4, §1c.
#include "walk.h"

namespace ingot_gpu {
namespace {

// Pipelined variant for fixed slots with no length array (C2-style rings):
// each wave walks several tiles and keeps the next DEPTH-1 tiles' LDS-DMA in
// flight while it parses the current one (DEPTH LDS images per wave, used
// round robin).  Requires stride >= 16*NCH.
// POL != 0: the cache-policy word fixed at compile time (the launcher's
// defaults), so the staging loads and record stores carry their cache bits
// directly instead of the runtime policy switch around every instruction
// (a tree of scalar branches per chunk); 0 = a.policy at run time.
template <uint32_t NCH, uint32_t DEPTH, int CHAIN, int MODE, uint32_t POL = 0>
__global__ __launch_bounds__(BLOCK) void k_parse_pipe(ParseArgs a) {
    constexpr uint32_t WIN = NCH * 16u;
    const uint32_t pol = POL ? POL : a.policy;
    constexpr uint32_t WAVE_DW = WAVE * NCH * 4u;
    constexpr uint32_t IMG_DW = WAVES * WAVE_DW + 16u;
    __shared__ __attribute__((aligned(16))) uint32_t s_img[DEPTH * IMG_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u);
    const uint32_t wave = threadIdx.x / WAVE;
    uint32_t* img0 = s_img + wave * WAVE_DW;
    const uint64_t ntiles = (a.n + WAVE - 1u) / WAVE;
    const uint32_t take = a.stride < WIN ? a.stride : WIN;

    auto stage = [&](uint64_t tt, uint32_t* img) {
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t c = (q - pp * NCH) ^ swz<NCH>(pp);
            uint64_t slot = tt * WAVE + pp;
            if (slot >= a.n) slot = a.n - 1u;  // a valid address for the tail tile
            stage16p(a.arena + slot * a.stride + 16u * c, img + k * WAVE * 4u, pol);
        }
    };
    auto parse = [&](uint64_t tt, const uint32_t* img) {
        const uint64_t i = tt * WAVE + lane;
        Frame<NCH> fr{(const lds_u32*)img, lane, 0u, take, a.stride, a.arena + i * a.stride};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        if (i < a.n) {
            if constexpr (MODE == OUT_REC8) store_rec(static_cast<uint2*>(a.out) + i, pack8(r), pol);
            else store_rec(static_cast<uint4*>(a.out) + i, pack(r), pol);
        }
    };

    // Tile order (INGOT_TUNE_XCD_REMAP).  Bit 0: block b runs on XCD b % 8;
    // renumbered (b % 8) * G/8 + b / 8 ("XCD-major"), each XCD's blocks take
    // a contiguous eighth of every round of G x WAVES tiles instead of every
    // eighth block's tiles.  Bit 1: each wave walks a contiguous run of
    // tiles (wave w: tiles w*J .. w*J + J-1) instead of striding by the grid.
    uint32_t bid = blockIdx.x;
    if ((a.xcd_remap & 1u) && gridDim.x % 8u == 0u)
        bid = (bid % 8u) * (gridDim.x / 8u) + bid / 8u;
    const uint64_t gw = (uint64_t)bid * WAVES + wave;  // this wave's index in the grid
    const uint64_t nw = (uint64_t)gridDim.x * WAVES;
    uint64_t t, step, tend;
    if ((a.xcd_remap & 4u) && gridDim.x % 8u == 0u) {
        // bit 2: the batch in 8 contiguous regions, one per XCD, the XCD's
        // waves striding through its region
        const uint64_t x = blockIdx.x % 8u;
        const uint64_t nwx = (uint64_t)(gridDim.x / 8u) * WAVES;
        const uint64_t region = (ntiles + 7u) / 8u;
        t = x * region + (uint64_t)(blockIdx.x / 8u) * WAVES + wave;
        tend = (x + 1u) * region < ntiles ? (x + 1u) * region : ntiles;
        step = nwx;
    } else if (a.xcd_remap & 2u) {
        const uint64_t J = (ntiles + nw - 1u) / nw;
        t = gw * J;
        tend = t + J < ntiles ? t + J : ntiles;
        step = 1u;
    } else {
        t = gw;
        tend = ntiles;
        step = nw;
    }
    if (t >= tend) return;
    // prologue: the first DEPTH-1 tiles
#pragma unroll
    for (uint32_t d = 0; d + 1u < DEPTH; ++d)
        if (t + d * step < tend) stage(t + d * step, img0 + d * IMG_DW);
    for (uint32_t j = 0;; ++j) {
        const uint64_t tn = t + (DEPTH - 1u) * step;
        if (tn < tend) {
            stage(tn, img0 + ((j + DEPTH - 1u) % DEPTH) * IMG_DW);
            // tile j's loads have landed (vector-memory ops retire in issue
            // order, stores and LDS-DMA alike): younger than them are the
            // DEPTH-1 later tiles' loads and, once the pipeline is full, the
            // DEPTH-1 record stores of the tiles before j — which need not
            // have completed (counting them out left every tile waiting for
            // the previous record's write-through)
            if (j + 1u >= DEPTH)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * (NCH + 1u)) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * NCH) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        parse(t, img0 + (j % DEPTH) * IMG_DW);
        t += step;
        if (t >= tend) break;
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
    // wave-uniform (readfirstlane): the tile cursors, the batch index and
    // the batch table lookups stay scalar (SGPRs, s_load from the kernel
    // arguments) instead of a per-lane load of the batch pointers per tile
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
    uint32_t* img0 = s_img + wave * WAVE_DW;
    const uint32_t tpb = a.tiles_per_batch;
    // Batch groups (RingArgs::groups = G): the grid is cut into G groups of
    // blocks (8 consecutive blocks, one per XCD, per group in turn), group q
    // consuming batches q, q+G, q+2G, ... — G batches in flight at once, as G
    // streams of per-batch launches would have (launch_ring: G divides the
    // grid into whole 8-block rows).
    const uint32_t G = a.groups;
    const uint32_t grp = (blockIdx.x / 8u) % G;
    const uint32_t gblk = (blockIdx.x / (8u * G)) * 8u + blockIdx.x % 8u;
    const uint32_t W = (gridDim.x / G) * WAVES;  // waves of the group
    const uint32_t nbg = (a.nbatches - grp + G - 1u) / G;
    const uint32_t total = tpb * nbg;  // the group's tiles (< 2^32, api.cpp)
    const uint32_t g0 = gblk * WAVES + wave;
    if (g0 >= total) return;
    const uint32_t J = (total - g0 + W - 1u) / W;  // this wave's tiles
    // the fields the loop uses, held in SGPRs: left as kernel-argument
    // reads, the compiler re-loads them from the (4 KiB) argument block
    // inside the loop, each a scalar load and an lgkmcnt wait per tile
    uint64_t n = a.n;
    uint32_t stride = a.stride, policy = a.policy, nb = a.nbatches;
    asm volatile("" : "+s"(n), "+s"(stride), "+s"(policy), "+s"(nb));
    const uint32_t take = stride < WIN ? stride : WIN;
    uint32_t avail = a.published;  // batches [0, avail) are known published
    bool live = true;              // false once this wave gave up waiting

    // Batch b published?  Polls only past `avail`: one system-scope load of
    // the doorbell per wave (one request; every lane gets the word), with
    // backoff sleeps between polls, until the word reaches
    // db_first + b or the wave's wait exceeds timeout_ticks.  On success the
    // wave's caches are invalidated (system-scope acquire) before it stages
    // the new batch, so frames written after the launch started are seen.
    auto ready = [&](uint32_t b) -> bool {
        if (b < avail) return true;
        if (!a.doorbell) return false;
        const uint64_t t0 = wall_clock64();
        uint32_t naps = 1;  // exponential backoff: 1, 2, 4, 8 sleeps between polls
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
            // ~1 us per nap: a waiting wave polls the host word at most
            // every ~8 us once the wait is long, so thousands of waiting
            // waves do not flood PCIe while a producer publishes
            for (uint32_t z = 0; z < naps; ++z) __builtin_amdgcn_s_sleep(32);
            naps = naps < 8u ? 2u * naps : 8u;
        }
    };
    // Cursors of the next tile to stage and to parse: (batch, tile) and that
    // batch's buffers, reloaded from the kernel arguments only when the
    // cursor crosses into the next batch (scalar loads, once per batch).
    struct Cur {
        uint32_t b, t;
        const uint8_t* arena;
        void* out;
    };
    auto setb = [&](Cur& c) {
        if (c.b < nb) {
            c.arena = a.b[c.b].arena;
            c.out = a.b[c.b].out;
            asm volatile("" : "+s"(c.arena), "+s"(c.out));
        }
    };
    auto adv = [&](Cur& c) {
        c.t += W;
        if (c.t >= tpb) {
            do {
                c.t -= tpb;
                c.b += G;
            } while (c.t >= tpb);
            setb(c);
        }
    };
    Cur sc{grp + (g0 / tpb) * G, g0 % tpb, nullptr, nullptr};
    setb(sc);
    Cur pc = sc;
    auto stage = [&](const Cur& c, uint32_t* img) {
#pragma unroll
        for (uint32_t k = 0; k < NCH; ++k) {
            const uint32_t q = k * WAVE + lane;
            const uint32_t pp = q / NCH;
            const uint32_t ch = (q - pp * NCH) ^ swz<NCH>(pp);
            uint64_t slot = (uint64_t)c.t * WAVE + pp;
            if (slot >= n) slot = n - 1u;  // a valid address for the tail tile
            stage16p(c.arena + slot * stride + 16u * ch, img + k * WAVE * 4u, policy);
        }
    };
    auto parse = [&](const Cur& c, const uint32_t* img) {
        const uint64_t i = (uint64_t)c.t * WAVE + lane;
        Frame<NCH> fr{(const lds_u32*)img, lane, 0u, take, stride, c.arena + i * stride};
        Rec r;
        walk<CHAIN, false>(fr, r, nullptr, nullptr);
        if (i < n) {
            if constexpr (MODE == OUT_REC8)
                store_rec(static_cast<uint2*>(c.out) + i, pack8(r), policy);
            else
                store_rec(static_cast<uint4*>(c.out) + i, pack(r), policy);
        }
    };
    // stage the next tile when there is one and its batch is published
    auto issue = [&](uint32_t& js) -> bool {
        if (!live || js >= J) return false;
        if (!ready(sc.b)) {
            live = false;
            return false;
        }
        stage(sc, img0 + (js % DEPTH) * IMG_DW);
        ++js;
        adv(sc);
        return true;
    };

    uint32_t js = 0;  // tiles staged so far
#pragma unroll
    for (uint32_t d = 0; d + 1u < DEPTH; ++d) issue(js);
    for (uint32_t j = 0; j < js; ++j) {
        // tile j's loads have landed: younger than them are the DEPTH-1 later
        // tiles' loads and (pipeline full) the DEPTH-1 earlier tiles' record
        // stores, which may still be in flight (k_parse_pipe)
        if (issue(js) && js - j == DEPTH) {
            if (j + 1u >= DEPTH)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * (NCH + 1u)) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((DEPTH - 1u) * NCH) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // the image is restaged only after every lane's reads of it have
        // returned: the record store consumes them (as in k_parse_pipe)
        parse(pc, img0 + (j % DEPTH) * IMG_DW);
        adv(pc);
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

    // XCD-major block order (a.xcd_remap bit 0), as in k_parse_pipe
    uint32_t bid = blockIdx.x;
    if ((a.xcd_remap & 1u) && gridDim.x % 8u == 0u)
        bid = (bid % 8u) * (gridDim.x / 8u) + bid / 8u;
    uint64_t t = (uint64_t)bid * WAVES + wave;
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

template <uint32_t NCH, uint32_t DEPTH, int MODE, uint32_t POL = 0>
hipError_t launch_pipe(const ParseArgs& a, int chain, uint32_t grid, hipStream_t s) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_UDP_PARSER, MODE, POL>),
                           dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_GENERIC_ULP:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_GENERIC_ULP, MODE, POL>),
                           dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    case INGOT_CHAIN_VLAN_ULP:
        hipLaunchKernelGGL((k_parse_pipe<NCH, DEPTH, INGOT_CHAIN_VLAN_ULP, MODE, POL>),
                           dim3(grid), dim3(BLOCK), 0, s, a);
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

// Ring rewrite kernel defaults (k_modify_pipe; measured).
constexpr uint32_t kModifyRingWb = 64;
constexpr uint32_t kModifyRingPolicy = 3;  // nt staging loads + nt write-back

// C2-style rings (slots >= 64 B, no length array, record output): the
// double-buffered multi-tile kernel.  Its grid is a whole number of blocks
// per CU (default 2), so the tiles spread evenly; measured on MI355X (1 M x
// 64 B, interleaved A/B): 16.6-16.7 vs 18.6-18.8 us per launch on one
// stream, 13.5-13.6 vs 14.2-14.4 us per step on two; 6 or 12 tiles per
// wave (uneven over the CUs) lose most of it.
hipError_t launch_slot_ring(const ParseArgs& args, int chain, int mode, const Tuning& t,
                            hipStream_t s) {
    ParseArgs a = args;
    // tile order: XCD-major by default (measured, DESIGN.md §4.2: 2 streams
    // 12.22 -> 12.03 us/step at 20 steps, 11.91 -> 11.74 at 2,000);
    // INGOT_TUNE_XCD_REMAP 4 = hardware order
    a.xcd_remap = t.xcd_remap == 0   ? 1u
                  : t.xcd_remap == 4 ? 0u
                  : t.xcd_remap == 5 ? 4u
                                     : (uint32_t)t.xcd_remap;
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
    // the default policies (launch_parse: 16-B records 11, 8-B records 3)
    // with their cache bits compiled in
    if (mode == OUT_REC16 && a.policy == 11u) return launch_pipe<4, 2, OUT_REC16, 11u>(a, chain, pg, s);
    if (mode == OUT_REC8 && a.policy == 3u) return launch_pipe<4, 2, OUT_REC8, 3u>(a, chain, pg, s);
    return mode == OUT_REC8 ? launch_pipe<4, 2, OUT_REC8>(a, chain, pg, s)
                            : launch_pipe<4, 2, OUT_REC16>(a, chain, pg, s);
}

// Slot rings (slots >= 64 B, no length array): the multi-tile kernel with
// lane-linear write-back (k_modify_pipe).  Defaults measured on MI355X
// (DESIGN.md §1c): write-back unit WB, plain staging loads.
hipError_t launch_modify_ring(const ModifyArgs& args, int chain, const Tuning& t,
                              hipStream_t s) {
    ModifyArgs a = args;
    a.p.xcd_remap = t.xcd_remap == 0 ? 1u : t.xcd_remap == 4 ? 0u : ((uint32_t)t.xcd_remap & 1u);
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
    // batch groups only on a grid of whole 8-block rows per group
    a.groups = t.ring_groups > 1 ? (uint32_t)t.ring_groups : 1u;
    if (g % (8u * a.groups) != 0 || a.groups > a.nbatches) a.groups = 1;
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

}  // namespace ingot_gpu
