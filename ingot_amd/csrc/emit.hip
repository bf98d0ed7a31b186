// emit.hip — batched Emit (ingot_gpu_emit_packets / ingot_gpu_emit_headers).
//
// ingot's Emit (ingot-types/src/emit.rs:8-120) writes an owned header stack
// field by field (the generated emit_raw, ingot-macros/src/packet/mod.rs:
// 2097-2255), a tuple emits its members back to back and a `&[u8]` member is
// a plain copy.  Here one owned stack, serialised once on the host, goes in
// front of every packet of a batch with per-packet setters applied to it
// (bitfield.rs:188-315: the field's covering bytes read-modify-written
// big-endian) — OPTE's outbound Geneve encapsulation.
//
// The header block sits in LDS once per workgroup.  A wave owns 64 packets:
// lane j loads packet j's descriptors and per-packet set values (coalesced),
// then the wave's groups of G lanes walk the packets (G = 64 for whole
// packets, 16 for header blocks: 4 packets at a time).  A group covers the
// packet's destination span [D, D + T) in aligned 16-B chunks, G per pass;
// each lane builds its chunk from
//   * the header bytes: two template blocks from LDS funnel-shifted by the
//     destination's misalignment, then the setters' bytes that fall in the
//     chunk (every covering byte's new value depends only on its own mask
//     and value bits, so a field split over two chunks needs no exchange);
//   * the payload bytes: one aligned 16-B source block per lane plus the
//     neighbouring lane's block, funnel-shifted by the packet's uniform
//     source-vs-destination misalignment;
// and stores it: a whole chunk as one aligned 16-B store, the two edge chunks
// byte by byte (packed packets share them).
// HBM-bound copy: algorithmic bytes per packet = len + 18 B of descriptors
// read, hdr_len + len written.
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "kernels.h"

namespace ingot_gpu {
namespace {

constexpr uint32_t BLOCK = 256;
constexpr uint32_t WAVE = 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gbl(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl_mut(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

// dword d of the 16 bytes at byte s (uniform 0..15) of the 32-B pair a ++ b
__device__ __forceinline__ uint32_t pick(const u32x4& a, const u32x4& b, uint32_t k) {
    switch (k) {
    case 0: return a.x;
    case 1: return a.y;
    case 2: return a.z;
    case 3: return a.w;
    case 4: return b.x;
    case 5: return b.y;
    case 6: return b.z;
    case 7: return b.w;
    default: return 0u;
    }
}
__device__ __forceinline__ u32x4 funnel(const u32x4& a, const u32x4& b, uint32_t s) {
    const uint32_t q = s >> 2, sh = (s & 3u) * 8u;
    u32x4 r;
    const uint32_t w0 = pick(a, b, q), w1 = pick(a, b, q + 1), w2 = pick(a, b, q + 2),
                   w3 = pick(a, b, q + 3), w4 = pick(a, b, q + 4);
    if (sh == 0) {
        r = u32x4{w0, w1, w2, w3};
    } else {
        r.x = (uint32_t)((((uint64_t)w1 << 32) | w0) >> sh);
        r.y = (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh);
        r.z = (uint32_t)((((uint64_t)w3 << 32) | w2) >> sh);
        r.w = (uint32_t)((((uint64_t)w4 << 32) | w3) >> sh);
    }
    return r;
}

__device__ __forceinline__ uint32_t head_mask(int32_t hc, uint32_t d) {
    // bytes [4d, 4d+4) of a chunk whose first hc bytes are header bytes
    const int32_t k = hc - (int32_t)(4u * d);
    return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : ((1u << (8u * (uint32_t)k)) - 1u);
}

__device__ __forceinline__ uint32_t set_value(const EmitSet& e, uint64_t i, uint32_t total) {
    switch (e.source) {
    case INGOT_EMIT_LENGTH: return total - e.at + (uint32_t)e.add;
    case INGOT_EMIT_U16: return (uint32_t)gbl((const uint16_t*)e.values)[i] + (uint32_t)e.add;
    case INGOT_EMIT_U32: return gbl((const uint32_t*)e.values)[i] + (uint32_t)e.add;
    default: return (uint32_t)e.add;
    }
}

template <uint32_t G, bool COPY>
__global__ __launch_bounds__(BLOCK) void k_emit(EmitArgs a) {
    constexpr uint32_t GPW = WAVE / G;  // groups (packets in flight) per wave
    // the header block with 16 zero bytes before and after it, as 16-B blocks
    __shared__ u32x4 tmpl[INGOT_MAX_EMIT_HDR / 16 + 2];
    for (uint32_t k = threadIdx.x; k < INGOT_MAX_EMIT_HDR / 16 + 2; k += BLOCK) {
        const bool in = k >= 1 && k <= INGOT_MAX_EMIT_HDR / 16;
        tmpl[k] = in ? u32x4{a.hdr[4 * k - 4], a.hdr[4 * k - 3], a.hdr[4 * k - 2],
                             a.hdr[4 * k - 1]}
                     : u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x % WAVE;
    const uint32_t gl = lane % G;  // lane within the group
    const uint32_t gw = lane / G;  // group within the wave
    const uint64_t wave = (uint64_t)blockIdx.x * (BLOCK / WAVE) + threadIdx.x / WAVE;
    const uint64_t base = wave * WAVE;
    if (base >= a.n) return;
    const uint32_t H = a.hdr_len;

    // lane j: packet base + j's descriptors and per-packet set values
    const uint64_t mine = base + lane;
    const bool have = mine < a.n;
    const uint32_t my_len = have ? (uint32_t)gbl(a.len)[mine] : 0u;
    const uint64_t my_dst = have ? (a.dst_off ? gbl(a.dst_off)[mine] : mine * (uint64_t)a.stride)
                                 : 0u;
    const uint64_t my_src = (COPY && have) ? gbl(a.off)[mine] : 0u;
    uint32_t my_val[INGOT_MAX_EMIT_SETS];
#pragma unroll
    for (uint32_t s = 0; s < INGOT_MAX_EMIT_SETS; ++s)
        my_val[s] = (s < a.n_sets && have) ? set_value(a.sets[s], mine, H + my_len) : 0u;

    const uint32_t count = (uint32_t)min<uint64_t>(WAVE, a.n - base);
    for (uint32_t p = 0; p < count; p += GPW) {
        const uint32_t j = p + gw;  // this group's packet within the wave's 64
        const bool live = j < count;
        const uint32_t jj = live ? j : p;
        const uint32_t L = (uint32_t)__shfl((int)my_len, (int)jj);
        const uint64_t doff = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(my_dst >> 32), (int)jj)
                               << 32) |
                              (uint32_t)__shfl((int)(uint32_t)my_dst, (int)jj);
        const uint64_t soff =
            COPY ? ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(my_src >> 32), (int)jj) << 32) |
                       (uint32_t)__shfl((int)(uint32_t)my_src, (int)jj)
                 : 0u;
        uint32_t v[INGOT_MAX_EMIT_SETS];
#pragma unroll
        for (uint32_t s = 0; s < INGOT_MAX_EMIT_SETS; ++s)
            v[s] = s < a.n_sets ? (uint32_t)__shfl((int)my_val[s], (int)jj) : 0u;
        uint8_t* D = a.dst + doff;
        const uint32_t T = H + (COPY ? L : 0u);
        const uint32_t dmis = (uint32_t)((uintptr_t)D & 15u);
        const uint32_t nch = (dmis + T + 15u) / 16u;
        const uint8_t* S = COPY ? a.src + soff : nullptr;
        // chunk c holds destination bytes r0 = 16c - dmis ...; header byte r
        // is template block (r + 16) / 16, payload byte r is S + r - H: both
        // shifts are uniform over the packet's chunks
        const uint32_t t_mis = (16u - dmis) & 15u;
        const uint32_t s_mis = COPY ? (uint32_t)((uintptr_t)(S - H - dmis) & 15u) : 0u;
        uint32_t np = (nch + G - 1) / G;
        // every group of the wave runs the same number of passes (shuffles)
#pragma unroll
        for (uint32_t o = G; o < WAVE; o <<= 1) np = max(np, (uint32_t)__shfl_xor((int)np, (int)o));
        for (uint32_t pass = 0; pass < np; ++pass) {
            const uint32_t c = pass * G + gl;
            const bool valid = live && c < nch;
            const int32_t r0 = (int32_t)(16u * c) - (int32_t)dmis;
            u32x4 out = u32x4{0u, 0u, 0u, 0u};
            if (COPY) {
                // own aligned block: the one holding source byte S + r0 - H
                const uintptr_t X = (uintptr_t)S + (intptr_t)(r0 - (int32_t)H);
                const uintptr_t B = X & ~(uintptr_t)15;
                const uintptr_t S0 = (uintptr_t)S, S1 = (uintptr_t)S + L;
                u32x4 own = u32x4{0u, 0u, 0u, 0u};
                if (valid && B + 16 > S0 && B < S1)
                    own = *(const __attribute__((address_space(1))) u32x4*)B;
                u32x4 nb;
                nb.x = (uint32_t)__shfl_down((int)own.x, 1u, (int)G);
                nb.y = (uint32_t)__shfl_down((int)own.y, 1u, (int)G);
                nb.z = (uint32_t)__shfl_down((int)own.z, 1u, (int)G);
                nb.w = (uint32_t)__shfl_down((int)own.w, 1u, (int)G);
                if (valid && s_mis != 0 && (gl == G - 1 || c + 1 >= nch) && B + 16 < S1 &&
                    B + 32 > S0)
                    nb = *(const __attribute__((address_space(1))) u32x4*)(B + 16);
                out = funnel(own, nb, s_mis);
            }
            if (H && valid && r0 < (int32_t)H) {
                const uint32_t tb = (uint32_t)(r0 + 16) >> 4;
                u32x4 hb = funnel(tmpl[tb], tmpl[tb + 1], t_mis);
                // the setters, byte by byte: each covering byte's new value
                // depends only on its own mask and value bits
#pragma unroll
                for (uint32_t s = 0; s < INGOT_MAX_EMIT_SETS; ++s) {
                    if (s >= a.n_sets) break;
                    const EmitSet& e = a.sets[s];
                    const uint32_t fm = e.bits >= 32 ? 0xffffffffu : ((1u << e.bits) - 1u);
                    const uint32_t m = fm << e.rshift, vb = (v[s] & fm) << e.rshift;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) {
                        if (k >= e.nbytes) break;
                        const int32_t t = (int32_t)(e.pos + k) - r0;
                        if (t < 0 || t >= 16) continue;
                        const uint32_t sh = 8u * (e.nbytes - 1u - k);
                        const uint32_t bm = ((m >> sh) & 0xffu) << (8u * ((uint32_t)t & 3u));
                        const uint32_t bv = ((vb >> sh) & 0xffu) << (8u * ((uint32_t)t & 3u));
                        const uint32_t d = (uint32_t)t >> 2;
                        if (d == 0) hb.x = (hb.x & ~bm) | bv;
                        if (d == 1) hb.y = (hb.y & ~bm) | bv;
                        if (d == 2) hb.z = (hb.z & ~bm) | bv;
                        if (d == 3) hb.w = (hb.w & ~bm) | bv;
                    }
                }
                const int32_t hc = (int32_t)H - r0;
                const uint32_t m0 = head_mask(hc, 0), m1 = head_mask(hc, 1),
                               m2 = head_mask(hc, 2), m3 = head_mask(hc, 3);
                out.x = (hb.x & m0) | (out.x & ~m0);
                out.y = (hb.y & m1) | (out.y & ~m1);
                out.z = (hb.z & m2) | (out.z & ~m2);
                out.w = (hb.w & m3) | (out.w & ~m3);
            }
            if (valid) {
                const int32_t t0 = r0 < 0 ? -r0 : 0;
                const int32_t t1 = (int32_t)T - r0 < 16 ? (int32_t)T - r0 : 16;
                if (t0 == 0 && t1 == 16) {
                    *(__attribute__((address_space(1))) u32x4*)(D + r0) = out;
                } else {
                    for (int32_t t = t0; t < t1; ++t) {
                        const uint32_t d = (uint32_t)t >> 2;
                        const uint32_t w = d == 0 ? out.x : d == 1 ? out.y : d == 2 ? out.z : out.w;
                        gbl_mut(D)[r0 + t] = (uint8_t)(w >> (8 * (t & 3)));
                    }
                }
            }
        }
    }
}

template <uint32_t G, bool COPY>
hipError_t go(const EmitArgs& a, hipStream_t s) {
    const uint64_t waves = (a.n + WAVE - 1) / WAVE;
    const uint64_t blocks = (waves + BLOCK / WAVE - 1) / (BLOCK / WAVE);
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_emit<G, COPY>), dim3((uint32_t)blocks), dim3(BLOCK), 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_emit(const EmitArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    return a.src ? go<64, true>(a, s) : go<16, false>(a, s);
}

}  // namespace ingot_gpu
