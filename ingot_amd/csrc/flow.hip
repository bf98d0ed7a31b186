// flow.hip — per-flow histogram pass (second launch of ingot_gpu_flow_hist).
//
// Counting straight from the parse kernel with global atomics serialises on
// the Zipf head (one hot flow = ~14% of packets at one address; measured
// 1.87 ms/step vs 0.32 ms for the parse alone on config 5).  Instead the parse
// kernel writes each packet's flow bin, and this pass builds the histogram
// without contention:
//  * with a caller workspace (ingot_gpu_flow_hist_ws, <= 65,536 bins): each
//    1024-thread block counts a contiguous slice of <= 65,535 flow ids into
//    packed 16-bit LDS counters (two bins per dword, 128 KiB; the slice bound
//    means no counter can wrap) and stores them as its row of the workspace;
//    a reduce pass sums the rows per bin and adds to the histogram — every
//    bin owned by one thread, no atomics.  Flow ids are read once.  Measured
//    on config 5 (tools/histbench.py): counting 9-14 us, atomic flush of the
//    same counters 73-102 us, row flush + reduce ~20 us;
//  * without one: block (x, y) owns bin range y (16,384 bins = 64 KiB of
//    32-bit LDS counters), scans packet slice x, and adds its non-zero
//    counters with global atomics (64 us on config 5);
//  * > 16 ranges: wave-aggregated global atomics.
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "kernels.h"

namespace ingot_gpu {
namespace {

constexpr uint32_t RANGE = 16384;
constexpr uint32_t THREADS = 1024;

__global__ __launch_bounds__(THREADS) void k_flow_hist(const uint32_t* __restrict__ flow,
                                                       uint64_t n, uint32_t* __restrict__ hist,
                                                       uint32_t range_bins) {
    __shared__ uint32_t cnt[RANGE];
    const uint32_t base = blockIdx.y * range_bins;
    for (uint32_t b = threadIdx.x; b < range_bins; b += THREADS) cnt[b] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * THREADS;
    for (uint64_t i = (uint64_t)blockIdx.x * THREADS + threadIdx.x; i < n; i += stride) {
        const uint32_t d = flow[i] - base;  // INGOT_FLOW_NONE and other ranges wrap out
        if (d < range_bins) atomicAdd(&cnt[d], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < range_bins; b += THREADS) {
        const uint32_t c = cnt[b];
        if (c) atomicAdd(hist + base + b, c);
    }
}

constexpr uint32_t WORDS16 = 32768;  // packed 16-bit counters for 65,536 bins: 128 KiB
constexpr uint64_t SLICE16 = 65532;  // flow ids per block (a multiple of 4): no counter wraps

__global__ __launch_bounds__(THREADS) void k_flow_count16(const uint32_t* __restrict__ flow,
                                                          uint64_t n, uint32_t bins,
                                                          uint64_t slice, bool vec,
                                                          uint32_t* __restrict__ rows) {
    __shared__ __attribute__((aligned(16))) uint32_t cnt[WORDS16];
    const uint32_t words = (bins + 1u) / 2u;
    for (uint32_t b = 4u * threadIdx.x; b < words; b += 4u * THREADS)
        *reinterpret_cast<uint4*>(cnt + b) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    auto count = [&](uint32_t d) {
        if (d < bins) atomicAdd(&cnt[d >> 1], 1u << ((d & 1u) * 16u));
    };
    const uint64_t lo = (uint64_t)blockIdx.x * slice;
    const uint64_t hi = lo + slice < n ? lo + slice : n;
    // slices start 16-B aligned (slice % 4 == 0; vec: flow 16-B aligned): 16-B
    // loads, UNROLL of them in flight per thread before the LDS atomics
    constexpr uint32_t UNROLL = 4;
    const uint64_t nv = vec && lo < hi ? (hi - lo) / 4u : 0u;
    const uint4* fv = reinterpret_cast<const uint4*>(flow + lo);
    uint64_t v = threadIdx.x;
    for (; v + (UNROLL - 1u) * THREADS < nv; v += UNROLL * THREADS) {
        uint4 x[UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < UNROLL; ++u) x[u] = fv[v + u * THREADS];
#pragma unroll
        for (uint32_t u = 0; u < UNROLL; ++u) {
            count(x[u].x);
            count(x[u].y);
            count(x[u].z);
            count(x[u].w);
        }
    }
    for (; v < nv; v += THREADS) {
        const uint4 x = fv[v];
        count(x.x);
        count(x.y);
        count(x.z);
        count(x.w);
    }
    for (uint64_t i = lo + 4u * nv + threadIdx.x; i < hi; i += THREADS) count(flow[i]);
    __syncthreads();
    uint32_t* row = rows + (uint64_t)blockIdx.x * words;
    for (uint32_t b = 4u * threadIdx.x; b < words; b += 4u * THREADS) {
        if (b + 4u <= words) {
            *reinterpret_cast<uint4*>(row + b) = *reinterpret_cast<const uint4*>(cnt + b);
        } else {
            for (uint32_t q = b; q < words; ++q) row[q] = cnt[q];
        }
    }
}

// hist[bin] += sum over the g rows.  Block: 64 words x 4 row groups; every
// bin pair is owned by one thread of the final step.
__global__ __launch_bounds__(256) void k_flow_reduce16(const uint32_t* __restrict__ rows,
                                                       uint32_t g, uint32_t words,
                                                       uint32_t* __restrict__ hist,
                                                       uint32_t bins) {
    __shared__ uint32_t part[2][4][64];
    const uint32_t lw = threadIdx.x & 63u, grp = threadIdx.x >> 6;
    const uint32_t w = blockIdx.x * 64u + lw;
    uint32_t a0 = 0, a1 = 0;
    if (w < words) {
#pragma unroll 8
        for (uint32_t r = grp; r < g; r += 4) {
            const uint32_t c = rows[(uint64_t)r * words + w];
            a0 += c & 0xffffu;
            a1 += c >> 16;
        }
    }
    part[0][grp][lw] = a0;
    part[1][grp][lw] = a1;
    __syncthreads();
    if (grp == 0 && w < words) {
        a0 += part[0][1][lw] + part[0][2][lw] + part[0][3][lw];
        a1 += part[1][1][lw] + part[1][2][lw] + part[1][3][lw];
        hist[2u * w] += a0;
        if (2u * w + 1u < bins) hist[2u * w + 1u] += a1;
    }
}

// Blocks of the workspace pass: enough slices that none exceeds SLICE16, and
// ~128 (measured best on config 5 vs 256 / 512: the rows are half as many);
// 0 = too many slices (> 256): use the range pass.
uint32_t rows_grid(uint64_t n) {
    uint64_t g = (n + SLICE16 - 1) / SLICE16;
    const uint64_t by_n = (n + 8191) / 8192;
    const uint64_t want = by_n < 128 ? by_n : 128;
    if (g < want) g = want;
    if (g < 1) g = 1;
    return g <= 256 ? (uint32_t)g : 0u;
}

// Many bins (> 16 ranges): re-scanning the flow ids once per range would cost
// more than atomics, and hot flows are then the only contention.  Lanes of a
// wave that share a bin are merged by ballot first (one atomic per bin per
// wave).
__global__ __launch_bounds__(256) void k_flow_hist_atomic(const uint32_t* __restrict__ flow,
                                                          uint64_t n, uint32_t* __restrict__ hist,
                                                          uint32_t bins) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    const uint64_t n_up = (n + 63u) & ~(uint64_t)63u;  // whole waves iterate together
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n_up; i += stride) {
        const uint32_t f = i < n ? flow[i] : INGOT_FLOW_NONE;
        const bool counted = f < bins;
        uint64_t pending = __ballot(counted);
        while (pending) {
            const int leader = __ffsll((long long)pending) - 1;
            const uint32_t b = (uint32_t)__shfl((int)f, leader);
            const uint64_t same = __ballot(counted && f == b) & pending;
            if ((int)lane == leader) atomicAdd(hist + b, (uint32_t)__popcll(same));
            pending &= ~same;
        }
    }
}

}  // namespace

size_t flow_hist_workspace(uint64_t n, uint32_t bins) {
    if (n == 0 || bins > 2u * WORDS16) return 0;
    const uint32_t g = rows_grid(n);
    return (size_t)g * ((bins + 1u) / 2u) * sizeof(uint32_t);
}

hipError_t launch_flow_hist(const uint32_t* flow, uint64_t n, uint32_t* hist, uint32_t bins,
                            void* work, size_t work_bytes, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t need = flow_hist_workspace(n, bins);
    if (need && work && work_bytes >= need) {
        const uint32_t g = rows_grid(n);
        const uint32_t words = (bins + 1u) / 2u;
        const uint64_t slice = ((n + g - 1) / g + 3u) & ~(uint64_t)3u;  // <= SLICE16
        auto* rows = static_cast<uint32_t*>(work);
        const bool vec = ((uintptr_t)flow & 15u) == 0;
        hipLaunchKernelGGL(k_flow_count16, dim3(g), dim3(THREADS), 0, s, flow, n, bins, slice,
                           vec, rows);
        hipLaunchKernelGGL(k_flow_reduce16, dim3((words + 63u) / 64u), dim3(256), 0, s,
                           (const uint32_t*)rows, g, words, hist, bins);
        return hipGetLastError();
    }
    const uint32_t range_bins = bins < RANGE ? bins : RANGE;
    const uint32_t ranges = bins / range_bins;
    if (ranges > 16) {
        uint64_t g = (n + 255) / 256;
        if (g > 4096) g = 4096;
        hipLaunchKernelGGL(k_flow_hist_atomic, dim3((uint32_t)g), dim3(256), 0, s, flow, n, hist,
                           bins);
        return hipGetLastError();
    }
    // ~256 blocks in flight (one 1024-thread block per CU), at least ~8 K
    // packets per block.
    uint64_t x = 256 / (ranges < 256 ? ranges : 256);
    const uint64_t by_n = (n + 8191) / 8192;
    if (x > by_n) x = by_n;
    if (x < 1) x = 1;
    hipLaunchKernelGGL(k_flow_hist, dim3((uint32_t)x, ranges), dim3(THREADS), 0, s, flow, n, hist,
                       range_bins);
    return hipGetLastError();
}

}  // namespace ingot_gpu
