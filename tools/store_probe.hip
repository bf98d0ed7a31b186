// store_probe.hip — measurement tool: HBM write rate of the store shapes the
// header-block emit can take (ingot_gpu_emit_headers into slots).
//   hipcc --offload-arch=gfx950 -O3 -o tools/variants/store_probe tools/store_probe.hip
//   tools/variants/store_probe [n_slots]
//   tools/variants/store_probe copy [bytes]   (device copy ceiling instead)
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

// one 16-B block per lane per step, U steps' loads in flight before the stores
template <int U>
__global__ void k_copy(const uint8_t* s, uint8_t* d, uint64_t nblk) {
    const uint64_t i0 = ((uint64_t)blockIdx.x * U) * blockDim.x + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t i = i0 + (uint64_t)u * blockDim.x;
        if (i < nblk) v[u] = *(const __attribute__((address_space(1))) u32x4*)(s + 16 * i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t i = i0 + (uint64_t)u * blockDim.x;
        if (i < nblk) *G(d + 16 * i) = v[u];
    }
}

// each wave copies a contiguous run of `per_wave` 16-B blocks, 64 per step, U
// steps' loads before their stores (the emit walk's shape without its math);
// dynamic LDS only limits how many waves share a CU
template <int U>
__global__ void k_copy_walk(const uint8_t* s, uint8_t* d, uint64_t nblk, uint32_t per_wave) {
    extern __shared__ uint8_t lds_pad[];
    const uint32_t lane = threadIdx.x % 64;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint64_t b0 = wave * per_wave;
    if (threadIdx.x == 1u << 20) lds_pad[0] = 0;
    for (uint32_t k0 = 0; k0 < per_wave; k0 += 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b0 + k0 + u * 64 + lane;
            if (k0 + u * 64 + lane < per_wave && i < nblk)
                v[u] = *(const __attribute__((address_space(1))) u32x4*)(s + 16 * i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b0 + k0 + u * 64 + lane;
            if (k0 + u * 64 + lane < per_wave && i < nblk) *G(d + 16 * i) = v[u];
        }
    }
}

// windows of 64 * U consecutive blocks; window w is taken by wave w % nwaves
// in its (w / nwaves)-th iteration, so the waves in flight at any time work
// on neighbouring windows (persistent waves, grid-interleaved windows)
template <int U>
__global__ void k_copy_interleaved(const uint8_t* s, uint8_t* d, uint64_t nblk) {
    extern __shared__ uint8_t lds_pad[];
    const uint32_t lane = threadIdx.x % 64;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / 64;
    if (threadIdx.x == 1u << 20) lds_pad[0] = 0;
    for (uint64_t w = wave; w * 64 * U < nblk; w += nwaves) {
        u32x4 v[U];
        const uint64_t b0 = w * 64 * U + lane;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b0 + u * 64 < nblk) v[u] = *(const __attribute__((address_space(1))) u32x4*)(s + 16 * (b0 + u * 64));
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b0 + u * 64 < nblk) *G(d + 16 * (b0 + u * 64)) = v[u];
    }
}

// the persistent interleaved loop as a two-stage pipeline: window t + 1's
// loads go out before window t's stores, every load and store unconditional
// (indices clamped), so the compiler's vmcnt waits never cover the stores
template <int U>
__global__ void k_copy_pipe(const uint8_t* s, uint8_t* d, uint64_t nblk) {
    extern __shared__ uint8_t lds_pad[];
    const uint32_t lane = threadIdx.x % 64;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / 64;
    if (threadIdx.x == 1u << 20) lds_pad[0] = 0;
    const uint64_t nwin = nblk / (64 * U);  // whole windows only (the probe's sizes)
    auto ld = [&](uint64_t w, u32x4* v) {
        const uint64_t b0 = (w < nwin ? w : 0) * 64 * U + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *(const __attribute__((address_space(1))) u32x4*)(s + 16 * (b0 + u * 64));
    };
    auto st = [&](uint64_t w, const u32x4* v) {
        const uint64_t b0 = w * 64 * U + lane;
#pragma unroll
        for (int u = 0; u < U; ++u) *G(d + 16 * (b0 + u * 64)) = v[u];
    };
    u32x4 a[U], b[U];
    uint64_t w = wave;
    if (w >= nwin) return;
    ld(w, a);
    while (true) {
        ld(w + nwaves, b);
        st(w, a);
        w += nwaves;
        if (w >= nwin) break;
        ld(w + nwaves, a);
        st(w, b);
        w += nwaves;
        if (w >= nwin) break;
    }
}

// a workgroup of W waves shares one contiguous run of `per_group` 16-B blocks
// (the emit walk's 64 packets), wave w taking steps w, w + W, ... of 64 * U
template <int U>
__global__ void k_copy_group(const uint8_t* s, uint8_t* d, uint64_t nblk, uint32_t per_group) {
    extern __shared__ uint8_t lds_pad[];
    const uint32_t lane = threadIdx.x % 64, w = threadIdx.x / 64, W = blockDim.x / 64;
    const uint64_t b0 = (uint64_t)blockIdx.x * per_group;
    if (threadIdx.x == 1u << 20) lds_pad[0] = 0;
    for (uint32_t k0 = w * 64 * U; k0 < per_group; k0 += W * 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b0 + k0 + u * 64 + lane;
            if (k0 + u * 64 + lane < per_group && i < nblk)
                v[u] = *(const __attribute__((address_space(1))) u32x4*)(s + 16 * i);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b0 + k0 + u * 64 + lane;
            if (k0 + u * 64 + lane < per_group && i < nblk) *G(d + 16 * i) = v[u];
        }
    }
}

static int copy_ceiling(uint64_t bytes) {
    uint8_t *s, *d;
    if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipMemset(s, 1, bytes);
    const uint64_t nblk = bytes / 16;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 3; ++r) {
            hipEventRecord(e0, 0);
            for (int k = 0; k < 5; ++k) launch();
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms / 5 < best ? ms / 5 : best;
        }
        printf("{\"variant\": \"%s\", \"bytes\": %llu, \"us\": %.1f, \"rw_GB_s\": %.1f, \"err\": %d}\n",
               name, (unsigned long long)bytes, best * 1e3, 2.0 * bytes / best / 1e6,
               (int)hipGetLastError());
        fflush(stdout);
    };
    timeit("copy_u1_b256", [&] { k_copy<1><<<(nblk + 255) / 256, 256>>>(s, d, nblk); });
    timeit("copy_u4_b256", [&] { k_copy<4><<<(nblk + 1023) / 1024, 256>>>(s, d, nblk); });
    timeit("copy_u8_b256", [&] { k_copy<8><<<(nblk + 2047) / 2048, 256>>>(s, d, nblk); });
    timeit("copy_u4_b128", [&] { k_copy<4><<<(nblk + 511) / 512, 128>>>(s, d, nblk); });
    const uint32_t pw = 3424;  // the emit wave's chunks (C6e: 64 packets, ~856 B each)
    const uint64_t waves = (nblk + pw - 1) / pw, blocks = (waves + 1) / 2;
    timeit("walk_u4_lds20k", [&] { k_copy_walk<4><<<blocks, 128, 20 * 1024>>>(s, d, nblk, pw); });
    timeit("walk_u4_lds0", [&] { k_copy_walk<4><<<blocks, 128, 0>>>(s, d, nblk, pw); });
    timeit("walk_u1_lds0", [&] { k_copy_walk<1><<<blocks, 128, 0>>>(s, d, nblk, pw); });
    timeit("walk_u8_lds0", [&] { k_copy_walk<8><<<blocks, 128, 0>>>(s, d, nblk, pw); });
    timeit("walk_u4_lds10k", [&] { k_copy_walk<4><<<blocks, 128, 10 * 1024>>>(s, d, nblk, pw); });
    timeit("win_u4_oneshot", [&] { k_copy_interleaved<4><<<(nblk + 511) / 512, 128, 0>>>(s, d, nblk); });
    timeit("win_u1_oneshot", [&] { k_copy_interleaved<1><<<(nblk + 127) / 128, 128, 0>>>(s, d, nblk); });
    timeit("persist_u4_4096w_lds20k", [&] { k_copy_interleaved<4><<<2048, 128, 20 * 1024>>>(s, d, nblk); });
    timeit("persist_u4_8192w", [&] { k_copy_interleaved<4><<<4096, 128, 0>>>(s, d, nblk); });
    timeit("persist_u2_4096w_lds20k", [&] { k_copy_interleaved<2><<<2048, 128, 20 * 1024>>>(s, d, nblk); });
    timeit("persist_u1_4096w_lds20k", [&] { k_copy_interleaved<1><<<2048, 128, 20 * 1024>>>(s, d, nblk); });
    timeit("pipe_u4_4096w_lds20k", [&] { k_copy_pipe<4><<<2048, 128, 20 * 1024>>>(s, d, nblk); });
    timeit("pipe_u2_4096w_lds20k", [&] { k_copy_pipe<2><<<2048, 128, 20 * 1024>>>(s, d, nblk); });
    timeit("pipe_u4_8192w", [&] { k_copy_pipe<4><<<4096, 128, 0>>>(s, d, nblk); });
    {
        const uint64_t groups = (nblk + pw - 1) / pw;
        timeit("group_w4_u4_lds12k", [&] { k_copy_group<4><<<groups, 256, 12 * 1024>>>(s, d, nblk, pw); });
        timeit("group_w8_u4_lds12k", [&] { k_copy_group<4><<<groups, 512, 12 * 1024>>>(s, d, nblk, pw); });
        timeit("group_w8_u2_lds12k", [&] { k_copy_group<2><<<groups, 512, 12 * 1024>>>(s, d, nblk, pw); });
        timeit("group_w16_u2_lds12k", [&] { k_copy_group<2><<<groups, 1024, 12 * 1024>>>(s, d, nblk, pw); });
        timeit("group_w16_u1_lds12k", [&] { k_copy_group<1><<<groups, 1024, 12 * 1024>>>(s, d, nblk, pw); });
    }
    timeit("hipMemcpyDtoD", [&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
    hipFree(s);
    hipFree(d);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'c')
        return copy_ceiling(argc > 2 ? strtoull(argv[2], 0, 10) : 6561093376ull);
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
