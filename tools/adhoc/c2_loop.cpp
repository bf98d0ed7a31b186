// c2_loop.cpp — measurement tool: the C2 step loop (1 M x 64-B slots,
// UdpParser, 16-B records) driven from C++ instead of Python, to check that
// bench.py's Python launch loop does not limit the pipelined rate.  Same
// shape as bench.py: R rotated arena copies, step k on stream k % S, HIP
// events around K steps.
//
//   hipcc --offload-arch=gfx950 -O2 -Iinclude tools/c2_loop.cpp \
//       -Lingot_amd/lib -lingot_gpu -Wl,-rpath,$PWD/ingot_amd/lib -o /tmp/c2_loop
//   /tmp/c2_loop [streams] [steps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ingot_gpu.h"
#include "ingot_pktgen.h"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int S = argc > 1 ? std::atoi(argv[1]) : 2;
    const int K = argc > 2 ? std::atoi(argv[2]) : 2000;
    const uint64_t n = 1u << 20;
    const uint32_t stride = 64;
    const int R = 8;
    ingot_gpu_ctx* ctx = nullptr;
    if (ingot_gpu_ctx_create(0, &ctx)) return 1;
    std::vector<uint8_t*> arena(R);
    std::vector<ingot_rec*> out(R);
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&arena[r], n * stride + 256));
        CK(hipMalloc(&out[r], n * sizeof(ingot_rec)));
        if (ingot_pktgen_fill(2 /*V4UDP64*/, 20250808, 0, n, nullptr, stride, nullptr, arena[r],
                              n * stride + 256, nullptr))
            return 1;
    }
    std::vector<hipStream_t> st(S);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](int steps) -> float {
        hipEventRecord(e0, st[0]);
        for (int s = 1; s < S; ++s) hipStreamWaitEvent(st[s], e0, 0);
        for (int k = 0; k < steps; ++k)
            ingot_gpu_parse_strided(ctx, arena[k % R], stride, nullptr, n,
                                    INGOT_CHAIN_UDP_PARSER, out[k % R], st[k % S]);
        for (int s = 1; s < S; ++s) {
            hipEvent_t j;
            hipEventCreateWithFlags(&j, hipEventDisableTiming);
            hipEventRecord(j, st[s]);
            hipStreamWaitEvent(st[0], j, 0);
            hipEventDestroy(j);
        }
        hipEventRecord(e1, st[0]);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return ms;
    };
    run(100);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        const float ms = run(K);
        if (ms < best) best = ms;
    }
    const double us = best * 1e3 / K;
    std::printf("{\"streams\": %d, \"steps\": %d, \"us_per_step\": %.3f, \"Gpkt_s\": %.2f}\n", S,
                K, us, n / us / 1e3);
    ingot_gpu_ctx_destroy(ctx);
    return 0;
}
