// census.hip — where does the hardware place the blocks of a persistent grid?
// Measurement tool (not product code).  Launches `blocks` 256-thread blocks
// with `lds` bytes of LDS each (the ring kernel's footprint: 32,896 B), each
// block recording its XCC, shader engine, CU and wave slot from the hardware
// ID registers and then holding its CU for `hold_us` of wall clock (so every
// block of the grid is resident at once, as in a persistent kernel).  Prints
// the histogram of blocks per CU.
//
//   hipcc --offload-arch=gfx950 -O2 tools/census.hip -o /tmp/census
//   /tmp/census 512 32896 200
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ __launch_bounds__(256) void k_census(uint32_t* out, uint64_t hold_ticks) {
    extern __shared__ uint32_t lds[];
    if (threadIdx.x == 0) {
        uint32_t hw = 0, xcc = 0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        lds[0] = hw;
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < hold_ticks) __builtin_amdgcn_s_sleep(8);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 512;
    const int lds = argc > 2 ? atoi(argv[2]) : 32896;
    const int hold_us = argc > 3 ? atoi(argv[3]) : 200;
    int khz = 0;
    hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    uint32_t* d = nullptr;
    hipMalloc(&d, sizeof(uint32_t) * 2 * blocks);
    hipFuncSetAttribute((const void*)k_census, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(k_census, dim3(blocks), dim3(256), lds, 0, d,
                       (uint64_t)hold_us * (uint64_t)khz / 1000u);
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "launch failed\n");
        return 1;
    }
    std::vector<uint32_t> h(2 * blocks);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // HW_ID (gfx9): wave_id [3:0], simd_id [5:4], cu_id [11:8], sh_id [12],
    // se_id [15:13]
    std::map<uint32_t, int> per_cu;
    for (int b = 0; b < blocks; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
        const uint32_t cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        per_cu[(xcc << 12) | (se << 8) | (sh << 4) | cu]++;
    }
    std::map<int, int> hist;
    for (auto& kv : per_cu) hist[kv.second]++;
    printf("{\"blocks\": %d, \"lds\": %d, \"cus_used\": %zu, \"blocks_per_cu_hist\": {", blocks, lds,
           per_cu.size());
    bool first = true;
    for (auto& kv : hist) {
        printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
        first = false;
    }
    printf("}}\n");
    hipFree(d);
    return 0;
}
