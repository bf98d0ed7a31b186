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
// The header block sits in LDS once per workgroup.  A group of 4 x 64
// packets: lane j of the group's wave w < 4 loads packet 64 w + j's
// descriptors and set values (coalesced) and patches the header block for it
// into an LDS region
// at its destination's 16-B alignment (template funnel-shifted, then the
// setters byte by byte: every covering byte's new value depends only on its
// own mask and value bits); a scan of the packets' chunk counts turns the
// group into one flat run of aligned 16-B destination chunks, which the
// group's 16 waves take in turns, 64 chunks per step.  A lane's chunk: its
// packet by binary search of the scan; the payload bytes as one aligned
// 16-B source block plus the next lane's (DPP), funnel-shifted by the
// packet's source-vs-destination misalignment; the header bytes from the
// region; a whole chunk leaves as one 16-B store, the two edge chunks a
// packet shares with its neighbours as predicated pieces (store_edge).
// HBM-bound copy: algorithmic bytes per packet = len + 24 B of descriptors
// and set values read, hdr_len + len written.
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "kernels.h"

namespace ingot_gpu {
namespace {

constexpr uint32_t WAVE = 64;
#ifndef INGOT_EMIT_GROUP_WAVES
#define INGOT_EMIT_GROUP_WAVES 16
#endif
// Whole packets: the W waves of a workgroup share one group of packets and
// take turns over its chunks, so a group's span is written by W waves at once
// and the spans in flight sit closer together (a plain copy of this shape:
// 4.87 TB/s one wave per span, 5.40 four).  A group is PW subgroups of 64
// packets whose descriptors PW waves load and patch in parallel, so the
// walkers wait on one subgroup's prologue, not PW of them.  Measured with
// equal output checksums (profiles/r05_emit_probe_history.json, r05aj /
// r05am / r05an): one wave per 64 packets 2.91 ms, W = 4 2.78-2.81, W = 16
// over four subgroups 2.65-2.77 (the best of W in {4, 6, 8, 10, 12, 16} with
// 1, 2, 3, 4, 8 or 16 subgroups).
// Header blocks: two one-wave groups.
#ifndef INGOT_EMIT_GROUP_SUBS
#define INGOT_EMIT_GROUP_SUBS 4
#endif
template <bool COPY> struct Shape {
    static constexpr uint32_t W = COPY ? INGOT_EMIT_GROUP_WAVES : 1u;  // waves per group
    static constexpr uint32_t PW = COPY ? INGOT_EMIT_GROUP_SUBS : 1u;  // 64-packet subgroups
    static constexpr uint32_t NP = PW * WAVE;                          // packets per group
    static constexpr uint32_t BLOCK = COPY ? W * WAVE : 2u * WAVE;
    static constexpr uint32_t G = BLOCK / (W * WAVE);                 // groups per block
    static_assert(PW <= W && PW <= 4, "one prologue wave per subgroup");
};
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
template <uint32_t NP>
struct WaveDesc {
    uint64_t dst[NP];     // destination address of packet j
    uint64_t src[NP];     // source address of its payload
    uint32_t pfx[NP];     // inclusive prefix of chunk counts
    uint32_t len[NP];     // payload bytes
    uint32_t mis[NP];     // dmis | s_mis << 8
    uint32_t sub[4];      // chunks of each 64-packet subgroup
    uint32_t cp, cp_inv;  // header blocks: chunk slots per packet, its reciprocal
    uint32_t _pad[WAVE - 6];
};

__host__ __device__ constexpr uint32_t region_bytes(uint32_t H) { return (H + 15u + 15u) / 16u * 16u; }

__device__ __forceinline__ uint32_t dword_at(const u32x4& v, uint32_t d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

// Bytes [t0, t1) of the 16-B chunk v at p (16-B aligned; neighbouring packets
// own the rest).  An edge chunk is cut on one side: a packet's first chunk
// keeps [t0, 16), its last [0, t1).  The whole dwords go as predicated dword
// stores at constant offsets, the one cut dword as a byte / short piece at
// p + 4 * (its index); a chunk cut on both sides (a packet shorter than a
// chunk) takes the byte loop.
__device__ __forceinline__ void store_edge(uint8_t* p, const u32x4& v, int32_t t0, int32_t t1) {
    auto* g32 = (__attribute__((address_space(1))) uint32_t*)p;
    if (t0 >= t1) return;
    if (t0 > 0 && t1 < 16) {
        for (int32_t t = t0; t < t1; ++t)
            gbl_mut(p)[t] = (uint8_t)(dword_at(v, (uint32_t)t >> 2) >> (8 * (t & 3)));
        return;
    }
    // whole dwords inside [t0, t1)
    if (0 >= t0 && 4 <= t1) g32[0] = v.x;
    if (4 >= t0 && 8 <= t1) g32[1] = v.y;
    if (8 >= t0 && 12 <= t1) g32[2] = v.z;
    if (12 >= t0 && 16 <= t1) g32[3] = v.w;
    // the cut dword: bytes [t0 & 3, 4) of dword t0 >> 2, or [0, t1 & 3) of t1 >> 2
    const bool head = t0 > 0;
    const uint32_t cut = head ? (uint32_t)t0 & 3u : (uint32_t)t1 & 3u;
    if (cut == 0) return;
    const uint32_t d = head ? (uint32_t)t0 >> 2 : (uint32_t)t1 >> 2;
    const uint32_t w = dword_at(v, d);
    auto* q8 = gbl_mut(p + 4 * d);
    auto* q16 = (__attribute__((address_space(1))) uint16_t*)(p + 4 * d);
    if (head) {  // bytes cut..3
        if (cut == 1) q8[1] = (uint8_t)(w >> 8);
        if (cut <= 2) q16[1] = (uint16_t)(w >> 16);
        if (cut == 3) q8[3] = (uint8_t)(w >> 24);
    } else {     // bytes 0..cut-1
        if (cut >= 2) q16[0] = (uint16_t)w;
        if (cut != 2) q8[cut == 1 ? 0 : 2] = (uint8_t)(cut == 1 ? w : w >> 16);
    }
}

template <bool COPY>
__global__ __launch_bounds__(Shape<COPY>::BLOCK) void k_emit(EmitArgs a) {
    constexpr uint32_t BLOCK = Shape<COPY>::BLOCK, W = Shape<COPY>::W, G = Shape<COPY>::G;
    constexpr uint32_t PW = Shape<COPY>::PW, NP = Shape<COPY>::NP;
    constexpr uint32_t NPOW = NP <= 64 ? 64 : NP <= 128 ? 128 : 256;  // search span
    using Desc = WaveDesc<NP>;
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
    const uint32_t lane = threadIdx.x % WAVE, g = threadIdx.x / (W * WAVE);
    const uint32_t wg = (threadIdx.x / WAVE) % W;  // this wave's turn in its group
    Desc& wd = reinterpret_cast<Desc*>(smem + TB * 16)[g];
    uint8_t* regions = smem + TB * 16 + G * sizeof(Desc) + g * NP * RS;
    __syncthreads();
    const uint64_t base = ((uint64_t)blockIdx.x * G + g) * NP;
    if (wg < PW) {
        // 1. wave wg of the group, lane j: packet base + 64 wg + j (coalesced
        //    descriptor and set-value loads)
        const uint32_t j = wg * WAVE + lane;  // the packet's index in the group
        const uint64_t i = base + j;
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
        uint8_t* R = regions + j * RS;
        if (H && live) {
            for (uint32_t m = 0; m < RS / 16u; ++m) {
                const uint32_t tb = 16u + 16u * m - dmis;  // template byte of region byte 16m (+16)
                reinterpret_cast<u32x4*>(R)[m] = funnel(tmpl[tb >> 4], tmpl[(tb >> 4) + 1], tb & 15u);
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
        wd.dst[j] = (uint64_t)(uintptr_t)D;
        wd.src[j] = (uint64_t)(uintptr_t)S;
        wd.pfx[j] = P;
        wd.len[j] = L;
        wd.mis[j] = dmis | (s_mis << 8);
        // header blocks: every packet takes CP chunk slots, the most any packet
        // of this wave needs (5 for 74 B at 16-B aligned slots, 6 unaligned)
        uint32_t CP = nch;
#pragma unroll
        for (uint32_t o = 1; o < WAVE; o <<= 1) CP = max(CP, (uint32_t)__shfl_xor((int)CP, (int)o));
        CP = max(CP, 1u);
        const uint32_t cp_inv = CP > 1u ? 0xffffffffu / CP + 1u : 0u;  // CP == 1: q = k
        const uint32_t wtotal = COPY ? (uint32_t)__shfl((int)P, (int)WAVE - 1)
                                     : (base < a.n ? (uint32_t)min<uint64_t>(WAVE, a.n - base) * CP : 0u);
        if (lane == 0) {
            wd.sub[wg] = wtotal;
            wd.cp = CP;
            wd.cp_inv = cp_inv;
        }
    }  // wg < PW
    __syncthreads();
    if (PW > 1) {
        // subgroups 1.. continue the prefix of the ones before them
        if (wg > 0 && wg < PW) {
            uint32_t before = 0;
            for (uint32_t t = 0; t < wg; ++t) before += wd.sub[t];
            wd.pfx[wg * WAVE + lane] += before;
        }
        __syncthreads();
    }
    uint32_t total = 0;
#pragma unroll
    for (uint32_t t = 0; t < PW; ++t) total += wd.sub[t];
    const uint32_t CP = wd.cp, cp_inv = wd.cp_inv;

    // 4. the wave's chunks, 64 per step and UNROLL steps at a time (all their
    //    loads are issued before the first store: bytes in flight): chunk k
    //    belongs to the first packet whose inclusive prefix exceeds k
    constexpr uint32_t U = COPY ? UNROLL : 2u;  // header blocks: no loads to overlap
    for (uint32_t k0 = wg * WAVE * U; k0 < total; k0 += W * WAVE * U) {
        uint32_t q[U], c[U];
        u32x4 own[U], nb[U];
        bool extra[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * WAVE + lane;
            const bool valid = k < total;
            uint32_t qq = 0, end = 0;
            if (COPY) {
#pragma unroll
                for (uint32_t step = NPOW / 2; step; step >>= 1)
                    if ((NP == NPOW || qq + step <= NP) && wd.pfx[qq + step - 1] <= k) qq += step;
                qq = valid ? qq : 0u;
                end = wd.pfx[qq];
                c[u] = valid ? k - (qq ? wd.pfx[qq - 1] : 0u) : 0xffffu;
            } else {
                // header blocks: CP chunks per packet (the most any packet of
                // the wave needs); the ones past a packet's own count write
                // nothing.  k / CP as a multiply-high by the wave's reciprocal
                // (exact: k < 64 * CP)
                qq = valid ? (CP == 1u ? k : __umulhi(k, cp_inv)) : 0u;
                c[u] = valid ? k - qq * CP : 0xffffu;
            }
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
        for (uint32_t u = 0; u < U; ++u) {
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
                    store_edge(QD + r0, out, t0, t1);
                }
            }
        }
    }
}

// Dynamic LDS of one k_emit block for a header block of H bytes.
template <bool COPY>
constexpr size_t emit_smem(uint32_t H) {
    return (INGOT_MAX_EMIT_HDR / 16 + 4) * 16 +
           Shape<COPY>::G * (sizeof(WaveDesc<Shape<COPY>::NP>) + Shape<COPY>::NP * region_bytes(H));
}
// gfx950: 160 KiB of LDS per workgroup.  A build with other group shapes
// (INGOT_EMIT_GROUP_SUBS / _WAVES) must still fit the largest header block.
static_assert(emit_smem<true>(INGOT_MAX_EMIT_HDR) <= 160u * 1024u, "k_emit<copy> LDS > 160 KiB");
static_assert(emit_smem<false>(INGOT_MAX_EMIT_HDR) <= 160u * 1024u, "k_emit LDS > 160 KiB");

template <bool COPY>
hipError_t go(const EmitArgs& a, hipStream_t s) {
    constexpr uint32_t G = Shape<COPY>::G, NP = Shape<COPY>::NP;
    const uint64_t groups = (a.n + NP - 1) / NP;
    const uint64_t blocks = (groups + G - 1) / G;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    const size_t smem = emit_smem<COPY>(a.hdr_len);
    hipLaunchKernelGGL((k_emit<COPY>), dim3((uint32_t)blocks), dim3(Shape<COPY>::BLOCK), smem, s, a);
    return hipGetLastError();
}

}  // namespace

size_t emit_lds_bytes(const EmitArgs& a) {
    return a.src ? emit_smem<true>(a.hdr_len) : emit_smem<false>(a.hdr_len);
}

hipError_t launch_emit(const EmitArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    return a.src ? go<true>(a, s) : go<false>(a, s);
}

}  // namespace ingot_gpu
