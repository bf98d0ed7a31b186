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

constexpr uint32_t BLOCK = 128;  // two waves: <= 40 KiB of LDS at the largest header block
constexpr uint32_t WAVE = 64;
#ifndef INGOT_EMIT_UNROLL
#define INGOT_EMIT_UNROLL 4
#endif
constexpr uint32_t UNROLL = INGOT_EMIT_UNROLL;  // 64-chunk steps whose loads fly together

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gbl(const T* p) {
    return (const __attribute__((address_space(1))) T*)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gbl_mut(T* p) {
    return (__attribute__((address_space(1))) T*)p;
}

// The 16 bytes at byte s (0..15, per lane) of the 32-B pair a ++ b: rotate
// by whole dwords in two select stages (2, then 1), then v_alignbyte.
__device__ __forceinline__ u32x4 funnel(const u32x4& a, const u32x4& b, uint32_t s) {
    const bool r2 = s & 8u, r1 = s & 4u;
    const uint32_t c0 = r2 ? a.z : a.x, c1 = r2 ? a.w : a.y, c2 = r2 ? b.x : a.z,
                   c3 = r2 ? b.y : a.w, c4 = r2 ? b.z : b.x, c5 = r2 ? b.w : b.y;
    const uint32_t d0 = r1 ? c1 : c0, d1 = r1 ? c2 : c1, d2 = r1 ? c3 : c2, d3 = r1 ? c4 : c3,
                   d4 = r1 ? c5 : c4;
    const uint32_t sh = s & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                 __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh)};
}

// The value of the next lane (lane 63: 0): DPP wave_shl:1, no LDS traffic.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
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

// Per-wave LDS: the 64 packets' descriptors, the inclusive prefix of their
// chunk counts, and each packet's patched header block at its destination's
// 16-B alignment (RS bytes per packet).
struct WaveDesc {
    uint64_t dst[WAVE];   // destination address of packet j
    uint64_t src[WAVE];   // source address of its payload
    uint32_t pfx[WAVE];   // inclusive prefix of chunk counts
    uint32_t len[WAVE];   // payload bytes
    uint32_t mis[WAVE];   // dmis | s_mis << 8
    uint32_t _pad[WAVE];
};

__host__ __device__ constexpr uint32_t region_bytes(uint32_t H) { return (H + 15u + 15u) / 16u * 16u; }

template <bool COPY>
__global__ __launch_bounds__(BLOCK) void k_emit(EmitArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    // the header block between zero bytes, as 16-B blocks
    u32x4* tmpl = reinterpret_cast<u32x4*>(smem);
    constexpr uint32_t TB = INGOT_MAX_EMIT_HDR / 16 + 4;  // 16 B before, 48 B after
    for (uint32_t k = threadIdx.x; k < TB; k += BLOCK) {
        const bool in = k >= 1 && k <= INGOT_MAX_EMIT_HDR / 16;
        tmpl[k] = in ? u32x4{a.hdr[4 * k - 4], a.hdr[4 * k - 3], a.hdr[4 * k - 2],
                             a.hdr[4 * k - 1]}
                     : u32x4{0u, 0u, 0u, 0u};
    }
    const uint32_t H = a.hdr_len;
    const uint32_t RS = region_bytes(H);
    const uint32_t lane = threadIdx.x % WAVE, w = threadIdx.x / WAVE;
    WaveDesc& wd = reinterpret_cast<WaveDesc*>(smem + TB * 16)[w];
    uint8_t* regions = smem + TB * 16 + (BLOCK / WAVE) * sizeof(WaveDesc) + w * WAVE * RS;
    __syncthreads();
    const uint64_t base = ((uint64_t)blockIdx.x * (BLOCK / WAVE) + w) * WAVE;
    if (base >= a.n) return;

    // 1. lane j: packet base + j (coalesced descriptor and set-value loads)
    const uint64_t i = base + lane;
    const bool live = i < a.n;
    const uint32_t L = live ? (uint32_t)gbl(a.len)[i] : 0u;
    const uint64_t doff = live ? (a.dst_off ? gbl(a.dst_off)[i] : i * (uint64_t)a.stride) : 0u;
    const uint64_t soff = (COPY && live) ? gbl(a.off)[i] : 0u;
    uint32_t v[INGOT_MAX_EMIT_SETS];
#pragma unroll
    for (uint32_t s = 0; s < INGOT_MAX_EMIT_SETS; ++s)
        v[s] = (s < a.n_sets && live) ? set_value(a.sets[s], i, H + L) : 0u;
    uint8_t* D = a.dst + doff;
    const uint8_t* S = COPY ? a.src + soff : nullptr;
    const uint32_t T = H + (COPY ? L : 0u);
    const uint32_t dmis = (uint32_t)((uintptr_t)D & 15u);
    const uint32_t s_mis = COPY ? (uint32_t)((uintptr_t)(S - H - dmis) & 15u) : 0u;
    const uint32_t nch = live ? (dmis + T + 15u) / 16u : 0u;

    // 2. the packet's header block in its region: template bytes shifted to
    //    the destination's alignment (region byte b = header byte b - dmis),
    //    then the setters byte by byte (neighbouring bits kept)
    uint8_t* R = regions + lane * RS;
    if (H && live) {
        const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tmpl);
        const uint32_t sh = 8u * ((16u - dmis) & 3u);
        for (uint32_t m = 0; m < RS / 4u; ++m) {
            const uint32_t tb = 16u + 4u * m - dmis;  // template byte of region byte 4m (+16)
            const uint32_t lo = t32[tb >> 2], hi = t32[(tb >> 2) + 1];
            reinterpret_cast<uint32_t*>(R)[m] =
                sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) : lo;
        }
#pragma unroll
        for (uint32_t s = 0; s < INGOT_MAX_EMIT_SETS; ++s) {
            if (s >= a.n_sets) break;
            const EmitSet& e = a.sets[s];
            const uint32_t fm = e.bits >= 32 ? 0xffffffffu : ((1u << e.bits) - 1u);
            const uint32_t m = fm << e.rshift, vb = (v[s] & fm) << e.rshift;
            for (uint32_t k = 0; k < e.nbytes; ++k) {
                const uint32_t shb = 8u * (e.nbytes - 1u - k);
                uint8_t& b = R[dmis + e.pos + k];
                b = (uint8_t)((b & ~(m >> shb)) | ((vb >> shb) & (m >> shb)));
            }
        }
    }

    // 3. chunk counts -> inclusive prefix over the wave
    uint32_t P = nch;
#pragma unroll
    for (uint32_t o = 1; o < WAVE; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)P, o);
        if (lane >= o) P += y;
    }
    wd.dst[lane] = (uint64_t)(uintptr_t)D;
    wd.src[lane] = (uint64_t)(uintptr_t)S;
    wd.pfx[lane] = P;
    wd.len[lane] = L;
    wd.mis[lane] = dmis | (s_mis << 8);
    const uint32_t total = (uint32_t)__shfl((int)P, (int)WAVE - 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // 4. the wave's chunks, 64 per step and UNROLL steps at a time (all their
    //    loads are issued before the first store: bytes in flight): chunk k
    //    belongs to the first packet whose inclusive prefix exceeds k
    for (uint32_t k0 = 0; k0 < total; k0 += WAVE * UNROLL) {
        uint32_t q[UNROLL], c[UNROLL];
        u32x4 own[UNROLL], nb[UNROLL];
        bool extra[UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < UNROLL; ++u) {
            const uint32_t k = k0 + u * WAVE + lane;
            const bool valid = k < total;
            uint32_t qq = 0;
#pragma unroll
            for (uint32_t step = WAVE / 2; step; step >>= 1)
                if (wd.pfx[qq + step - 1] <= k) qq += step;
            qq = valid ? qq : 0u;
            const uint32_t end = wd.pfx[qq];
            c[u] = valid ? k - (qq ? wd.pfx[qq - 1] : 0u) : 0xffffu;
            q[u] = qq;
            own[u] = u32x4{0u, 0u, 0u, 0u};
            nb[u] = u32x4{0u, 0u, 0u, 0u};
            extra[u] = false;
            if (COPY && valid) {
                const uint32_t mis = wd.mis[qq];
                const uint32_t qd = mis & 0xffu, qs = mis >> 8;
                const uint8_t* QS = (const uint8_t*)(uintptr_t)wd.src[qq];
                const int32_t r0 = (int32_t)(16u * c[u]) - (int32_t)qd;
                const uintptr_t X = (uintptr_t)QS + (intptr_t)(r0 - (int32_t)H);
                const uintptr_t B = X & ~(uintptr_t)15;
                const uintptr_t S0 = (uintptr_t)QS, S1 = (uintptr_t)QS + wd.len[qq];
                if (B + 16 > S0 && B < S1) own[u] = *(const __attribute__((address_space(1))) u32x4*)B;
                // the next lane holds block B + 16 only if it has this packet's next chunk
                if (qs != 0 && (lane == WAVE - 1 || k + 1 >= end) && B + 16 < S1 && B + 32 > S0) {
                    nb[u] = *(const __attribute__((address_space(1))) u32x4*)(B + 16);
                    extra[u] = true;
                }
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < UNROLL; ++u) {
            const bool valid = c[u] != 0xffffu;
            const uint32_t qq = q[u];
            const uint32_t mis = wd.mis[qq];
            const uint32_t qd = mis & 0xffu, qs = mis >> 8;
            uint8_t* QD = (uint8_t*)(uintptr_t)wd.dst[qq];
            const uint32_t QT = H + (COPY ? wd.len[qq] : 0u);
            const int32_t r0 = (int32_t)(16u * c[u]) - (int32_t)qd;
            u32x4 out = u32x4{0u, 0u, 0u, 0u};
            if (COPY) {
                u32x4 n2;
                n2.x = from_next_lane(own[u].x);
                n2.y = from_next_lane(own[u].y);
                n2.z = from_next_lane(own[u].z);
                n2.w = from_next_lane(own[u].w);
                out = funnel(own[u], extra[u] ? nb[u] : n2, qs);
            }
            if (H && valid && r0 < (int32_t)H) {
                const u32x4 hb = *reinterpret_cast<const u32x4*>(regions + qq * RS + 16u * c[u]);
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
                const int32_t t1 = (int32_t)QT - r0 < 16 ? (int32_t)QT - r0 : 16;
                if (t0 == 0 && t1 == 16) {
                    *(__attribute__((address_space(1))) u32x4*)(QD + r0) = out;
                } else {
                    // an edge chunk (packets share it): whole dwords inside
                    // [t0, t1) as dword stores, the rest byte by byte
                    const uint32_t wv[4] = {out.x, out.y, out.z, out.w};
#pragma unroll
                    for (int32_t d = 0; d < 4; ++d) {
                        if (4 * d >= t0 && 4 * d + 4 <= t1) {
                            *(__attribute__((address_space(1))) uint32_t*)(QD + r0 + 4 * d) = wv[d];
                        } else {
#pragma unroll
                            for (int32_t b = 0; b < 4; ++b)
                                if (4 * d + b >= t0 && 4 * d + b < t1)
                                    gbl_mut(QD)[r0 + 4 * d + b] = (uint8_t)(wv[d] >> (8 * b));
                        }
                    }
                }
            }
        }
    }
}

template <bool COPY>
hipError_t go(const EmitArgs& a, hipStream_t s) {
    const uint64_t waves = (a.n + WAVE - 1) / WAVE;
    const uint64_t blocks = (waves + BLOCK / WAVE - 1) / (BLOCK / WAVE);
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const size_t smem = (INGOT_MAX_EMIT_HDR / 16 + 4) * 16 +
                        (BLOCK / WAVE) * (sizeof(WaveDesc) + WAVE * region_bytes(a.hdr_len));
    hipLaunchKernelGGL((k_emit<COPY>), dim3((uint32_t)blocks), dim3(BLOCK), smem, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_emit(const EmitArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    return a.src ? go<true>(a, s) : go<false>(a, s);
}

}  // namespace ingot_gpu
