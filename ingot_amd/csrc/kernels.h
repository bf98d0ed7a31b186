// kernels.h — internal interface between the C ABI (api.cpp) and the HIP
// kernels (parse.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ingot_gpu.h"

namespace ingot_gpu {

enum LayoutKind { LAYOUT_STRIDED = 0, LAYOUT_INDEXED = 1 };

// Output mode: 16-B ingot_rec, 8-B ingot_rec8, or 256-B ingot_fields.
enum OutMode { OUT_REC16 = 0, OUT_REC8 = 1, OUT_FIELDS = 2 };

struct ParseArgs {
    const uint8_t* arena;
    const uint64_t* off;   // LAYOUT_INDEXED
    const uint16_t* len;   // optional for LAYOUT_STRIDED
    uint32_t stride;       // LAYOUT_STRIDED
    uint64_t n;
    void* out;             // n records of the OutMode's type
};

// Per-context tuning (0 = measured default); see INGOT_TUNE_* in ingot_gpu.h.
struct Tuning {
    int window_indexed = 0;
    int window_strided = 0;
    uint32_t max_blocks = 0;
};

hipError_t launch_parse(const ParseArgs& a, int layout_kind, int chain, int mode,
                        const Tuning& t, hipStream_t s);
bool tuning_valid(int key, int value);

}  // namespace ingot_gpu
