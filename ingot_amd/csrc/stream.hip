// stream.hip — stream scheduling helpers for multi-stream ring consumers.
//
// k_delay holds its stream for a fixed span of the device's constant-rate
// wall clock (s_memrealtime via wall_clock64(), `hipDeviceAttributeWallClockRate`
// kHz): one wave on one CU, sleeping between clock reads.  A consumer that
// alternates batches over two streams uses it to start the second stream
// about half a launch behind the first, so the two streams' launches do not
// ramp up and drain in lockstep ("Staggered streams").
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace ingot_gpu {
namespace {

__global__ __launch_bounds__(64) void k_delay(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
}

}  // namespace

hipError_t launch_delay(uint64_t ticks, hipStream_t s) {
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, ticks);
    return hipGetLastError();
}

}  // namespace ingot_gpu
