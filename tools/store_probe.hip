// store_probe.hip — measurement tool: HBM write rate of the store shapes the
// header-block emit can take (ingot_gpu_emit_headers into slots).
//   hipcc --offload-arch=gfx950 -O3 -o tools/variants/store_probe tools/store_probe.hip
//   tools/variants/store_probe [n_slots]
// Each variant writes H bytes of every slot i at i * stride (H <= stride):
//   flat16   lanes cover the slots' bytes as one flat run of 16-B chunks
//            (full chunks whole, edge chunks cut), consecutive lanes ->
//            consecutive chunks (the chunk walk);
//   lane16   lane = slot, its chunks one 16-B store each, chunk c of 64
//            slots per instruction;
//   lane16f  lane16 with the whole slot stored (H rounded up to 16) — the
//            bound if the tail bytes were the kernel's to write;
//   memset   the slots' whole span written contiguously, 16 B per lane;
//   edit8    dwords 5 and 6 of every 64-B slot (bytes 20..27: an IPv4 TTL /
//            checksum edit behind a 14-B Ethernet header), the rest of the
//            line left alone — against memset of the same span, the choice
//            an in-place rewrite (k_modify_pipe) makes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G(p) ((__attribute__((address_space(1))) u32x4*)(p))

__global__ void k_memset(uint8_t* d, uint64_t nchunks) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nchunks) *G(d + 16 * i) = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

__device__ __forceinline__ void store_piece(uint8_t* p, u32x4 v, int t0, int t1) {
    if (t0 == 0 && t1 == 16) {
        *G(p) = v;
        return;
    }
    for (int t = t0; t < t1; ++t) p[t] = (uint8_t)(v[t >> 2] >> (8 * (t & 3)));
}

__global__ void k_edit8(uint8_t* d, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    auto* p = (__attribute__((address_space(1))) uint32_t*)(d + 64 * i);
    p[5] = (uint32_t)i;
    p[6] = 7u;
}

template <bool FULL>
__global__ void k_lane16(uint8_t* d, uint64_t n, uint32_t stride, uint32_t H) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* D = d + i * stride;
    const uint32_t dmis = (uint32_t)((uintptr_t)D & 15u);
    uint8_t* A = D - dmis;
    const uint32_t T = FULL ? (H + 15u) / 16u * 16u : H;
    for (uint32_t c = 0; 16 * c < dmis + T; ++c) {
        const int r0 = (int)(16 * c) - (int)dmis;
        const int t0 = r0 < 0 ? -r0 : 0, t1 = (int)T - r0 < 16 ? (int)T - r0 : 16;
        store_piece(A + 16 * c, u32x4{(uint32_t)i, c, 2u, 3u}, t0, t1);
    }
}

// chunks per slot when every slot has the same alignment (stride % 16 == 0)
__global__ void k_flat16(uint8_t* d, uint64_t n, uint32_t stride, uint32_t H) {
    const uint32_t cp = (H + 15u) / 16u;
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n * cp) return;
    const uint64_t i = k / cp;
    const uint32_t c = (uint32_t)(k - i * cp);
    const int t1 = (int)H - (int)(16 * c) < 16 ? (int)H - (int)(16 * c) : 16;
    store_piece(d + i * stride + 16 * c, u32x4{(uint32_t)i, c, 2u, 3u}, 0, t1);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : (1ull << 23);
    const uint32_t H = 74;
    const uint32_t strides[] = {74, 80, 96, 128, 256};
    uint8_t* d;
    if (hipMalloc(&d, n * 256 + 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, uint32_t stride, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            hipEventRecord(e0, 0);
            for (int k = 0; k < 10; ++k) launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 10 < best ? ms / 10 : best;
        }
        const hipError_t err = hipGetLastError();
        printf("{\"variant\": \"%s\", \"stride\": %u, \"hdr_len\": %u, \"slots\": %llu, \"us\": %.1f, "
               "\"hdr_GB_s\": %.1f, \"span_GB_s\": %.1f, \"err\": %d}\n",
               name, stride, H, (unsigned long long)n, best * 1e3, n * (double)H / best / 1e6,
               n * (double)stride / best / 1e6, (int)err);
        fflush(stdout);
    };
    for (uint32_t st : strides) {
        const uint64_t nch = (n * st + 15) / 16;
        timeit("memset", st, [&] { k_memset<<<(nch + 255) / 256, 256>>>(d, nch); });
        timeit("lane16", st, [&] { k_lane16<false><<<(n + 255) / 256, 256>>>(d, n, st, H); });
        timeit("lane16f", st, [&] { k_lane16<true><<<(n + 255) / 256, 256>>>(d, n, st, H); });
        if (st % 16 == 0) {
            const uint64_t k = n * ((H + 15) / 16);
            timeit("flat16", st, [&] { k_flat16<<<(k + 255) / 256, 256>>>(d, n, st, H); });
        }
    }
    timeit("edit8", 64, [&] { k_edit8<<<(n + 255) / 256, 256>>>(d, n); });
    timeit("memset", 64, [&] { k_memset<<<(n * 4 + 255) / 256, 256>>>(d, n * 4); });
    hipFree(d);
    return 0;
}
