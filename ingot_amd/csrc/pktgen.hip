// pktgen.hip — deterministic synthetic traffic on the device
// (include/ingot_pktgen.h; the generator itself is pktgen_core.h, shared
// with the host build).
//
// Bench/test infrastructure, not the parse path.  Two passes: a coalesced
// pattern fill of the whole arena (payload and gaps), then one lane per frame
// writing its header bytes (clipped to the frame length, so truncated frames
// never spill into their neighbours).
#include <hip/hip_runtime.h>

#include "../../include/ingot_gpu.h"
#include "pktgen_core.h"

namespace {

using namespace ingot_pktgen;

__global__ void k_lengths(int profile, uint64_t seed, uint64_t first, uint64_t n, uint16_t* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint16_t)plan(profile, seed, first + i).len;
}

__global__ void k_pattern(int profile, uint64_t seed, uint8_t* arena, uint64_t bytes) {
    const uint64_t words = bytes / 16;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t v[4];
        pattern_word(profile, seed, w, v);
        reinterpret_cast<uint4*>(arena)[w] = make_uint4(v[0], v[1], v[2], v[3]);
    }
    const uint64_t tail = words * 16;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < bytes - tail) arena[tail + t] = (uint8_t)(t * 13 + 7);
}

__global__ void k_headers(int profile, uint64_t seed, uint64_t first, uint64_t n,
                          const uint64_t* off, uint32_t stride, const uint16_t* lens,
                          uint8_t* arena, uint64_t arena_bytes) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Plan p = plan(profile, seed, first + i);
    const uint64_t o = off ? off[i] : i * (uint64_t)stride;
    uint32_t len = lens ? lens[i] : stride;
    if (o >= arena_bytes) return;
    if (o + len > arena_bytes) len = (uint32_t)(arena_bytes - o);
    write_frame(profile, seed, first + i, p, arena + o, len);
}

int err(hipError_t e) { return e == hipSuccess ? INGOT_GPU_SUCCESS : INGOT_GPU_EHIP; }

}  // namespace

extern "C" int ingot_pktgen_lengths(int profile, uint64_t seed, uint64_t first, uint64_t n,
                                    uint16_t* d_len, void* stream) {
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_len) return INGOT_GPU_EINVAL;
    const uint32_t grid = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_lengths, dim3(grid), dim3(256), 0, (hipStream_t)stream, profile, seed,
                       first, n, d_len);
    return err(hipGetLastError());
}

extern "C" int ingot_pktgen_fill(int profile, uint64_t seed, uint64_t first, uint64_t n,
                                 const uint64_t* d_off, uint32_t stride, const uint16_t* d_len,
                                 uint8_t* d_arena, uint64_t arena_bytes, void* stream) {
    if (!d_arena || (!d_off && stride == 0) || (d_off && !d_len)) return INGOT_GPU_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (((uintptr_t)d_arena & 15u) != 0) return INGOT_GPU_EINVAL;
    if (arena_bytes) {
        hipLaunchKernelGGL(k_pattern, dim3(4096), dim3(256), 0, s, profile, seed, d_arena,
                           arena_bytes);
        if (hipGetLastError() != hipSuccess) return INGOT_GPU_EHIP;
    }
    if (n == 0) return INGOT_GPU_SUCCESS;
    const uint32_t grid = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_headers, dim3(grid), dim3(256), 0, s, profile, seed, first, n, d_off,
                       stride, d_len, d_arena, arena_bytes);
    return err(hipGetLastError());
}
