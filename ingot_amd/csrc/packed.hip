// packed.hip — offsets for frames stored back to back with only a length
// array (a capture buffer / ring without a descriptor table;
// ingot_gpu_parse_packed).  Frame i starts at sum(len[0..i)).
//
// Two small passes give every 64-packet tile its base offset; the parse
// kernel (k_parse, LAYOUT_PACKED) then derives each lane's offset with a
// wavefront prefix scan of its tile's lengths, so no per-packet offset array
// is ever written or read:
//   k_tile_sums   a 256-thread block covers GROUP = 128 tiles: each lane
//                 loads 8 lengths (16 B) per instruction, groups of 8 lanes
//                 reduce to one tile sum, then the block's 128 sums are
//                 scanned in LDS -> the tile's u32 offset within its group
//                 and the group total;
//   k_group_scan  one 1024-thread block: exclusive scan of the group totals
//                 -> u64 group bases.
// The parse adds the two (tile base = group base + local prefix).
// Workspace: u64 group bases, then u32 local prefixes (one per tile).
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "kernels.h"

namespace ingot_gpu {
namespace {

constexpr uint32_t WAVE = 64;
constexpr uint32_t GROUP = PACKED_GROUP;       // tiles per k_tile_sums block
constexpr uint32_t SCAN_THREADS = 1024;
constexpr uint32_t SCAN_K = 8;                 // groups per thread per chunk

// len[] may be any length: reads past n return 0 (16-B loads only when the
// whole vector is in range).
__global__ __launch_bounds__(256) void k_tile_sums(const uint16_t* __restrict__ len, uint64_t n,
                                                   uint32_t* __restrict__ local,
                                                   uint64_t* __restrict__ totals) {
    __shared__ uint32_t sums[GROUP];
    const uint32_t lane = threadIdx.x & (WAVE - 1u), wave = threadIdx.x / WAVE;
    const uint64_t g0 = (uint64_t)blockIdx.x * GROUP;  // first tile of the group
    const bool vec = ((uintptr_t)len & 15u) == 0;
    // 4 waves x 4 iterations x 8 tiles = 128 tiles; lane L of an iteration
    // covers lengths [8L, 8L + 8) of 8 consecutive tiles (512 lengths)
#pragma unroll
    for (uint32_t it = 0; it < 4; ++it) {
        const uint64_t tile0 = g0 + (wave * 4u + it) * 8u;
        const uint64_t i = tile0 * WAVE + 8u * lane;
        uint32_t x = 0;
        if (vec && i + 8u <= n) {
            const uint4 v = *reinterpret_cast<const uint4*>(len + i);
            x = (v.x & 0xffffu) + (v.x >> 16) + (v.y & 0xffffu) + (v.y >> 16) + (v.z & 0xffffu) +
                (v.z >> 16) + (v.w & 0xffffu) + (v.w >> 16);
        } else {
            for (uint32_t k = 0; k < 8; ++k)
                if (i + k < n) x += len[i + k];
        }
#pragma unroll
        for (uint32_t d = 4; d > 0; d >>= 1) x += (uint32_t)__shfl_xor((int)x, (int)d);
        if ((lane & 7u) == 0) sums[(wave * 4u + it) * 8u + lane / 8u] = x;
    }
    __syncthreads();
    // exclusive scan of the 128 sums by the first 128 threads (Hillis-Steele)
    uint32_t v = threadIdx.x < GROUP ? sums[threadIdx.x] : 0u;
    uint32_t incl = v;
    for (uint32_t d = 1; d < GROUP; d <<= 1) {
        const uint32_t y = threadIdx.x >= d && threadIdx.x < GROUP ? sums[threadIdx.x - d] : 0u;
        __syncthreads();
        if (threadIdx.x < GROUP) sums[threadIdx.x] = incl = incl + y;
        __syncthreads();
    }
    const uint64_t ntiles = (n + WAVE - 1) / WAVE;
    if (threadIdx.x < GROUP && g0 + threadIdx.x < ntiles) local[g0 + threadIdx.x] = incl - v;
    if (threadIdx.x == GROUP - 1) totals[blockIdx.x] = incl;  // <= 2^31: fits u32 sums
}

__global__ __launch_bounds__(SCAN_THREADS) void k_group_scan(uint64_t* __restrict__ base,
                                                             uint64_t ngroups) {
    // in place: totals -> exclusive prefix
    __shared__ uint64_t part[SCAN_THREADS];
    const uint32_t tid = threadIdx.x;
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < ngroups; c0 += (uint64_t)SCAN_THREADS * SCAN_K) {
        const uint64_t first = c0 + (uint64_t)tid * SCAN_K;
        uint64_t v[SCAN_K];
        uint64_t loc = 0;
#pragma unroll
        for (uint32_t k = 0; k < SCAN_K; ++k) {
            v[k] = first + k < ngroups ? base[first + k] : 0u;
            loc += v[k];
        }
        part[tid] = loc;
        __syncthreads();
        for (uint32_t d = 1; d < SCAN_THREADS; d <<= 1) {
            const uint64_t y = tid >= d ? part[tid - d] : 0u;
            __syncthreads();
            part[tid] += y;
            __syncthreads();
        }
        uint64_t x = carry + part[tid] - loc;
#pragma unroll
        for (uint32_t k = 0; k < SCAN_K; ++k) {
            if (first + k < ngroups) base[first + k] = x;
            x += v[k];
        }
        carry += part[SCAN_THREADS - 1];
        __syncthreads();
    }
}

}  // namespace

size_t packed_workspace(uint64_t n) {
    const uint64_t ntiles = (n + WAVE - 1) / WAVE;
    const uint64_t ngroups = (ntiles + GROUP - 1) / GROUP;
    return (size_t)ngroups * sizeof(uint64_t) + (size_t)ntiles * sizeof(uint32_t) + 64;
}

hipError_t launch_tile_bases(const uint16_t* len, uint64_t n, void* work, hipStream_t s) {
    const uint64_t ntiles = (n + WAVE - 1) / WAVE;
    const uint64_t ngroups = (ntiles + GROUP - 1) / GROUP;
    if (ngroups > 0x7fffffffull) return hipErrorInvalidValue;
    uint64_t* base = static_cast<uint64_t*>(work);
    uint32_t* local = reinterpret_cast<uint32_t*>(base + ngroups);
    hipLaunchKernelGGL(k_tile_sums, dim3((uint32_t)ngroups), dim3(256), 0, s, len, n, local,
                       base);
    hipLaunchKernelGGL(k_group_scan, dim3(1), dim3(SCAN_THREADS), 0, s, base, ngroups);
    return hipGetLastError();
}

}  // namespace ingot_gpu
