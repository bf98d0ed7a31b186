// stream_ceiling.hip — measurement tool (not product): the practical HBM
// ceiling for the parse's exact byte pattern at config-2 size, i.e. read
// 64 B + write 16 B per "packet", 1M packets per launch, no parsing.
//   k_reg:  each lane reads 16-B chunks fully coalesced (4 x dwordx4 per
//           64 packets per wave), folds, writes one 16-B record per packet.
//   k_glds: the same bytes staged HBM->LDS with global_load_lds_dwordx4, as
//           the parse kernel does, then one ds_read_b128 x4 per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void lds_void;

__global__ __launch_bounds__(256) void k_reg(const uint4* __restrict__ in, uint4* __restrict__ out,
                                             uint64_t n) {
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wave; t < ntiles; t += (uint64_t)gridDim.x * 4) {
        const uint4* base = in + t * 256;
        uint4 a = base[lane], b = base[64 + lane], c = base[128 + lane], d = base[192 + lane];
        uint4 r;
        r.x = a.x ^ b.y ^ c.z ^ d.w;
        r.y = a.y ^ b.z ^ c.w ^ d.x;
        r.z = a.z ^ b.w ^ c.x ^ d.y;
        r.w = a.w ^ b.x ^ c.y ^ d.z;
        if (t * 64 + lane < n) out[t * 64 + lane] = r;
    }
}

__global__ __launch_bounds__(256) void k_glds(const uint8_t* __restrict__ in, uint4* __restrict__ out,
                                              uint64_t n) {
    __shared__ __attribute__((aligned(16))) uint4 s[4 * 256];
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4* img = s + wave * 256;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wave; t < ntiles; t += (uint64_t)gridDim.x * 4) {
        const uint8_t* base = in + t * 4096;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_global_load_lds((const void*)(base + (k * 64 + lane) * 16),
                                             (lds_void*)(img + k * 64), 16, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint4 a = img[lane * 4], b = img[lane * 4 + 1], c = img[lane * 4 + 2], d = img[lane * 4 + 3];
        uint4 r;
        r.x = a.x ^ b.y ^ c.z ^ d.w;
        r.y = a.y ^ b.z ^ c.w ^ d.x;
        r.z = a.z ^ b.w ^ c.x ^ d.y;
        r.w = a.w ^ b.x ^ c.y ^ d.z;
        if (t * 64 + lane < n) out[t * 64 + lane] = r;
    }
}

// Read-only ceiling: the same 64 B/packet reads, no record stores (a store
// only if the data hits a sentinel, which synthetic frames never do).
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ in, uint4* __restrict__ out,
                                              uint64_t n) {
    const uint64_t ntiles = (n + 63) / 64;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t t = (uint64_t)blockIdx.x * 4 + wave; t < ntiles; t += (uint64_t)gridDim.x * 4) {
        const uint4* base = in + t * 256;
        uint4 a = base[lane], b = base[64 + lane], c = base[128 + lane], d = base[192 + lane];
        const uint32_t x = a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
        if (x == 0x9E3779B9u && a.y == 0x7F4A7C15u) out[t * 64 + lane] = a;
    }
}

extern "C" int stream_run(int which, const void* in, void* out, uint64_t n, uint32_t grid,
                          void* stream) {
    if (which == 2) {
        hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                           (const uint4*)in, (uint4*)out, n);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    if (which == 0)
        hipLaunchKernelGGL(k_reg, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                           (const uint4*)in, (uint4*)out, n);
    else
        hipLaunchKernelGGL(k_glds, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                           (const uint8_t*)in, (uint4*)out, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// --- gather ceiling for packed variable-length frames (config 3 pattern) ---
// Each packet: read its descriptor (u64 off + u16 len), then NCHUNK 16-B chunks
// from its 16-B-aligned frame start, write one 16-B record.
template <int NCHUNK>
__global__ __launch_bounds__(256) void k_gather_reg(const uint8_t* __restrict__ arena,
                                                    const uint64_t* __restrict__ off,
                                                    const uint16_t* __restrict__ len,
                                                    uint4* __restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint32_t l = len[i];
    const uint4* p = reinterpret_cast<const uint4*>(arena + (o & ~15ull));
    uint4 acc = make_uint4(l, 0, 0, 0);
#pragma unroll
    for (int c = 0; c < NCHUNK; ++c) {
        const uint4 v = p[c];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    out[i] = acc;
}

template <int NCH>
__global__ __launch_bounds__(256) void k_gather_glds(const uint8_t* __restrict__ arena,
                                                     const uint64_t* __restrict__ off,
                                                     const uint16_t* __restrict__ len,
                                                     uint4* __restrict__ out, uint64_t n) {
    __shared__ __attribute__((aligned(16))) uint4 s[4 * 64 * NCH];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint4* img = s + wave * 64 * NCH;
    const uint64_t t = (uint64_t)blockIdx.x * 4 + wave;
    const uint64_t i = t * 64 + lane;
    const uint64_t o = i < n ? off[i] : 0;
    const uint64_t base = o & ~15ull;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
        const uint32_t q = k * 64 + lane, pp = q / NCH, c = q - pp * NCH;
        const uint64_t bp = (uint64_t)__shfl((long long)base, (int)pp);
        if (t * 64 + pp < n)
            __builtin_amdgcn_global_load_lds((const void*)(arena + bp + 16 * c),
                                             (lds_void*)(img + k * 64), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 acc = img[lane * NCH];
    acc.x ^= len[i < n ? i : 0];
    if (i < n) out[i] = acc;
}

extern "C" int gather_run(int which, const void* arena, const void* off, const void* len,
                          void* out, uint64_t n, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t g1 = (uint32_t)((n + 255) / 256);
    const auto* a = (const uint8_t*)arena;
    const auto* o = (const uint64_t*)off;
    const auto* l = (const uint16_t*)len;
    auto* r = (uint4*)out;
    switch (which) {
    case 0: hipLaunchKernelGGL(k_gather_reg<5>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 1: hipLaunchKernelGGL(k_gather_reg<8>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 2: hipLaunchKernelGGL(k_gather_reg<9>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 3: hipLaunchKernelGGL(k_gather_glds<5>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 4: hipLaunchKernelGGL(k_gather_glds<9>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    default: hipLaunchKernelGGL(k_gather_reg<0>, dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// --- fetch-granularity probe (config-3 frames): per packet, NSEG aligned
// segments of SEG bytes starting at off & ~(SEG-1), read as 16-B register
// loads; one 16-B record per packet.  Tells whether HBM traffic follows the
// bytes requested (32/64-B sectors) or whole 128-B lines.
template <int SEG, int NSEG>
__global__ __launch_bounds__(256) void k_gather_seg(const uint8_t* __restrict__ arena,
                                                    const uint64_t* __restrict__ off,
                                                    const uint16_t* __restrict__ len,
                                                    uint4* __restrict__ out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t o = off[i];
    const uint4* p = reinterpret_cast<const uint4*>(arena + (o & ~(uint64_t)(SEG - 1)));
    uint4 acc = make_uint4(len[i], 0, 0, 0);
#pragma unroll
    for (int c = 0; c < SEG * NSEG / 16; ++c) {
        const uint4 v = p[c];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    out[i] = acc;
}

extern "C" int seg_run(int which, const void* arena, const void* off, const void* len, void* out,
                       uint64_t n, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    const uint32_t g1 = (uint32_t)((n + 255) / 256);
    const auto* a = (const uint8_t*)arena;
    const auto* o = (const uint64_t*)off;
    const auto* l = (const uint16_t*)len;
    auto* r = (uint4*)out;
    switch (which) {
    case 0: hipLaunchKernelGGL((k_gather_seg<32, 1>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 1: hipLaunchKernelGGL((k_gather_seg<64, 1>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 2: hipLaunchKernelGGL((k_gather_seg<64, 2>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 3: hipLaunchKernelGGL((k_gather_seg<128, 1>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    case 4: hipLaunchKernelGGL((k_gather_seg<128, 2>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    default: hipLaunchKernelGGL((k_gather_seg<32, 2>), dim3(g1), dim3(256), 0, s, a, o, l, r, n); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// --- histogram flush probe (config 5 flow ids): the packed 16-bit single
// pass with its per-block flush as global atomics (product k_flow_hist16) vs
// plain stores of the block's counters into a scratch row + a reduce pass.
__global__ __launch_bounds__(1024) void k_h16(const uint32_t* __restrict__ flow, uint64_t n,
                                              uint32_t* __restrict__ hist, uint32_t* rows,
                                              uint64_t slice, int mode) {
    __shared__ uint32_t cnt[32768];
    for (uint32_t b = threadIdx.x; b < 32768; b += 1024) cnt[b] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * slice;
    const uint64_t hi = lo + slice < n ? lo + slice : n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 1024) {
        const uint32_t d = flow[i];
        if (d < 65536u) atomicAdd(&cnt[d >> 1], 1u << ((d & 1u) * 16u));
    }
    __syncthreads();
    if (mode == 0) {
        for (uint32_t b = threadIdx.x; b < 32768; b += 1024) {
            const uint32_t c = cnt[b];
            if (c & 0xffffu) atomicAdd(hist + 2u * b, c & 0xffffu);
            if (c >> 16) atomicAdd(hist + 2u * b + 1u, c >> 16);
        }
    } else if (mode == 1) {
        for (uint32_t b = threadIdx.x; b < 32768; b += 1024) rows[blockIdx.x * 32768u + b] = cnt[b];
    } else {
        uint32_t acc = 0;  // no flush at all: counting only
        for (uint32_t b = threadIdx.x; b < 32768; b += 1024) acc ^= cnt[b];
        if (acc == 0x9E3779B9u) hist[0] = acc;
    }
}

__global__ __launch_bounds__(256) void k_h16_reduce(const uint32_t* __restrict__ rows, uint32_t g,
                                                    uint32_t* __restrict__ hist) {
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;  // word = 2 bins
    uint32_t a0 = 0, a1 = 0;
    for (uint32_t r = 0; r < g; ++r) {
        const uint32_t c = rows[r * 32768u + w];
        a0 += c & 0xffffu;
        a1 += c >> 16;
    }
    hist[2 * w] += a0;
    hist[2 * w + 1] += a1;
}

extern "C" int h16_run(int mode, const void* flow, uint64_t n, void* hist, void* rows,
                       uint32_t g, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    const uint64_t slice = (n + g - 1) / g;
    hipLaunchKernelGGL(k_h16, dim3(g), dim3(1024), 0, s, (const uint32_t*)flow, n,
                       (uint32_t*)hist, (uint32_t*)rows, slice, mode);
    if (mode == 1)
        hipLaunchKernelGGL(k_h16_reduce, dim3(128), dim3(256), 0, s, (const uint32_t*)rows, g,
                           (uint32_t*)hist);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
