// kernels.h — internal interface between the C ABI (api.cpp) and the HIP
// kernels (parse.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ingot_gpu.h"

namespace ingot_gpu {

enum LayoutKind { LAYOUT_STRIDED = 0, LAYOUT_INDEXED = 1 };

struct ParseArgs {
    const uint8_t* arena;
    const uint64_t* off;   // LAYOUT_INDEXED
    const uint16_t* len;   // optional for LAYOUT_STRIDED
    uint32_t stride;       // LAYOUT_STRIDED
    uint64_t n;
    ingot_rec* out;        // record mode
    ingot_fields* fields;  // parity mode
};

// max_blocks = 0 lets the launcher size the grid (persistent, LDS-limited).
hipError_t launch_parse(const ParseArgs& a, int layout_kind, int chain, bool fields,
                        uint32_t max_blocks, hipStream_t s);

}  // namespace ingot_gpu
