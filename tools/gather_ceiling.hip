// Measurement tool (not product code): how fast can the chip pull the 128-B
// lines a header parse of packed frames needs, with nothing else to do?
// Built by tools/gather_ceiling.py into tools/bin/libgather_ceiling.so and
// driven from there (torch buffers, HIP events).
//
//   k_touch   one lane per frame, one 4-B load per distinct 128-B line of the
//             frame bytes [skip, skip + span[i]) (clipped to the frame): the
//             fewest instructions that make HBM deliver exactly those lines;
//             a 4-B store per frame keeps the loads alive.
//   k_stage   the parse kernels' staging alone: a line-completing window of
//             2..5 16-B chunks from the chunk holding byte 12 (k_parse's
//             linewin = 2), copied into a per-wave LDS image by LDS-DMA, one
//             tile of 64 frames per wave, then one LDS dword per lane and a
//             4-B store (no walk, no record).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr uint32_t WAVE = 64, WAVES = 4, BLOCK = WAVE * WAVES, NCH = 5;
typedef __attribute__((address_space(3))) void lds_void;

__global__ __launch_bounds__(BLOCK) void k_touch(const uint8_t* arena, const uint64_t* off,
                                                 const uint16_t* len, uint64_t n, uint32_t skip,
                                                 const uint16_t* span, uint32_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint32_t l = len[i];
    const uint32_t sp = span[i];
    uint32_t acc = 0;
    if (l > skip && sp) {
        const uint32_t e = l < skip + sp ? l : skip + sp;
        const uintptr_t a = (uintptr_t)(arena + o + skip);
        const uintptr_t b = (uintptr_t)(arena + o + e - 1u);
        const uintptr_t l0 = a & ~(uintptr_t)127, l1 = b & ~(uintptr_t)127;
        acc = *reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        for (uintptr_t x = l0 + 128; x <= l1; x += 128) acc ^= *reinterpret_cast<const uint32_t*>(x);
    }
    out[i] = acc;
}

__global__ __launch_bounds__(BLOCK) void k_stage(const uint8_t* arena, const uint64_t* off,
                                                 const uint16_t* len, uint64_t n, uint32_t* out) {
    constexpr uint32_t SKIP = 12, WAVE_DW = WAVE * NCH * 4;
    __shared__ __attribute__((aligned(16))) uint32_t s_win[WAVES * WAVE_DW];
    const uint32_t lane = threadIdx.x & (WAVE - 1u), wave = threadIdx.x / WAVE;
    uint32_t* img = s_win + wave * WAVE_DW;
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const bool valid = i < n;
    const uint64_t o = valid ? off[i] : 0u;
    const uint32_t l = valid ? len[i] : 0u;
    const uint32_t mis = (uint32_t)((uintptr_t)arena & 31u);
    const uint32_t sh = (uint32_t)((o + SKIP + mis) & 15u);
    const int64_t base = (int64_t)o + SKIP - sh;
    const uint32_t lp = (uint32_t)((uintptr_t)(arena + base) >> 4) & 7u;
    uint32_t want = ((lp + 2u + 7u) & ~7u) - lp;
    if (want > NCH) want = NCH;
    const uint32_t wend = SKIP + 16u * want - sh;
    const uint32_t take = l < wend ? l : wend;
    const int32_t staged = (int32_t)take - ((int32_t)SKIP - (int32_t)sh);
    const uint32_t nch = staged > 0 ? ((uint32_t)staged + 15u) >> 4 : 0u;
#pragma unroll
    for (uint32_t k = 0; k < NCH; ++k) {
        const uint32_t q = k * WAVE + lane;
        const uint32_t pp = q / NCH, c = q - pp * NCH;
        const uint32_t np = (uint32_t)__shfl((int)nch, (int)pp);
        const int64_t bp = (int64_t)__shfl((long long)base, (int)pp);
        if (c < np)
            __builtin_amdgcn_global_load_lds((const void*)(arena + bp + 16u * c),
                                             (lds_void*)(img + k * WAVE * 4u), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (valid) out[i] = img[lane * NCH * 4u];
}

}  // namespace

extern "C" int gc_touch(const uint8_t* arena, const uint64_t* off, const uint16_t* len, uint64_t n,
                        uint32_t skip, const uint16_t* span, uint32_t* out, hipStream_t s) {
    const uint32_t g = (uint32_t)((n + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_touch, dim3(g), dim3(BLOCK), 0, s, arena, off, len, n, skip, span, out);
    return (int)hipGetLastError();
}

extern "C" int gc_stage(const uint8_t* arena, const uint64_t* off, const uint16_t* len, uint64_t n,
                        uint32_t* out, hipStream_t s) {
    const uint32_t g = (uint32_t)((n + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_stage, dim3(g), dim3(BLOCK), 0, s, arena, off, len, n, out);
    return (int)hipGetLastError();
}
