// pktgen_host.cpp — the synthetic traffic generator on the host
// (ingot_pktgen_*_host, include/ingot_pktgen.h), built with g++ into
// libingot_pktgen_host.so: no HIP dependency, so bench.py can build its CPU
// baseline's sample before the process touches the GPU.  Same bytes as the
// device generator for the same (profile, seed, first, n, layout, length of
// arena) — tests/test_pktgen_host.py checks that on the GPU.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/ingot_gpu.h"
#include "pktgen_core.h"

using namespace ingot_pktgen;

namespace {

// [lo, hi) of n split into `threads` contiguous ranges, fn(lo, hi) each.
template <class F>
void parallel(uint64_t n, int threads, F fn) {
    if (threads <= 1 || n < 4096) {
        fn(0, n);
        return;
    }
    std::vector<std::thread> ts;
    const uint64_t step = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const uint64_t lo = std::min<uint64_t>(n, t * step), hi = std::min<uint64_t>(n, lo + step);
        if (lo < hi) ts.emplace_back([=] { fn(lo, hi); });
    }
    for (auto& t : ts) t.join();
}

}  // namespace

extern "C" int ingot_pktgen_lengths_host(int profile, uint64_t seed, uint64_t first, uint64_t n,
                                         uint16_t* h_len, int threads) {
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!h_len) return INGOT_GPU_EINVAL;
    parallel(n, threads, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) h_len[i] = (uint16_t)plan(profile, seed, first + i).len;
    });
    return INGOT_GPU_SUCCESS;
}

extern "C" int ingot_pktgen_fill_host(int profile, uint64_t seed, uint64_t first, uint64_t n,
                                      const uint64_t* h_off, uint32_t stride,
                                      const uint16_t* h_len, uint8_t* h_arena,
                                      uint64_t arena_bytes, int threads) {
    if (!h_arena || (!h_off && stride == 0) || (h_off && !h_len)) return INGOT_GPU_EINVAL;
    if (((uintptr_t)h_arena & 15u) != 0) return INGOT_GPU_EINVAL;
    const uint64_t words = arena_bytes / 16;
    parallel(words, threads, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t w = lo; w < hi; ++w) {
            uint32_t v[4];
            pattern_word(profile, seed, w, v);
            memcpy(h_arena + 16 * w, v, 16);  // little-endian, as the device's uint4 store
        }
    });
    for (uint64_t t = 0; t < arena_bytes - words * 16; ++t)
        h_arena[words * 16 + t] = (uint8_t)(t * 13 + 7);
    parallel(n, threads, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) {
            const Plan p = plan(profile, seed, first + i);
            const uint64_t o = h_off ? h_off[i] : i * (uint64_t)stride;
            uint32_t len = h_len ? h_len[i] : stride;
            if (o >= arena_bytes) continue;
            if (o + len > arena_bytes) len = (uint32_t)(arena_bytes - o);
            write_frame(profile, seed, first + i, p, h_arena + o, len);
        }
    });
    return INGOT_GPU_SUCCESS;
}
