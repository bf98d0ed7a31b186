// api.cpp — the C ABI (include/ingot_gpu.h) over the HIP kernels.
//
// Argument checking, context handling and the string tables that mirror
// ingot's error surface: ParseError::as_cstr (ingot-types/src/error.rs:49-60)
// and the per-layer labels a generated chain attaches to PacketParseError
// (ingot-macros/src/parse.rs:36-50, field names from
// ingot-examples/src/packets.rs:18-40, 54-60).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/ingot_gpu.h"
#include "kernels.h"

namespace {

// One ingot_gpu_host_map of [host, host + bytes) by a context.  `owned`:
// the bytes lie inside a registration this library made (g_regs below);
// otherwise the memory was pinned and mapped by someone else (hipHostMalloc,
// or the caller's own hipHostRegister) and unmapping it is a no-op.
struct HostMapping {
    uintptr_t host, bytes, dev;
    bool owned;
};

// Pageable host ranges this library page-locked (hipHostRegister, mapped).
// Registration state is per process, not per context, so the table is too.
// Each entry is the exact byte range registered; every ingot_gpu_host_map of
// bytes inside it (by any context) holds a reference, and the last
// ingot_gpu_host_unmap unregisters it.  Nothing else is ever unregistered.
struct Registration {
    uintptr_t host, bytes, dev;
    uint32_t refs;
};
std::mutex g_reg_mu;
std::vector<Registration> g_regs;

}  // namespace

struct ingot_gpu_ctx {
    int device = 0;
    ingot_gpu::Tuning tuning;
    uint32_t wall_khz = 0;  // the device's constant-rate wall clock (stream delays)
    size_t lds_bytes = 160u * 1024u;  // LDS per workgroup (the device's, at create)
    // live ingot_gpu_host_map mappings of this context (dropped on unmap)
    std::mutex mu;
    std::vector<HostMapping> host;
};

namespace {

const char* const kParseErrorNames[] = {
    "Ok",           "Unwanted",       "NeedsHint", "TooSmall",    "StraddledHeader",
    "NoRemainingChunks", "CannotAccept", "Reject",    "IllegalValue",
};

const char* const kUdpParserLabels[] = {"eth", "l3", "l4"};
const char* const kGenericUlpLabels[] = {"inner_eth", "inner_l3", "inner_ulp"};
const char* const kVlanUlpLabels[] = {"eth", "vlan", "l3", "l4"};
// ingot-examples/src/packets.rs:27-40
const char* const kGeneveLabels[] = {"outer_eth", "outer_v6",  "outer_udp", "outer_encap",
                                     "inner_eth", "inner_l3", "inner_ulp"};

int chain_ok(int chain) { return chain >= 0 && chain < INGOT_CHAIN_COUNT; }

int from_hip(hipError_t e) { return e == hipSuccess ? INGOT_GPU_SUCCESS : INGOT_GPU_EHIP; }

// Make the context's device current for the launch (callers may juggle
// devices on one thread).
int enter(const ingot_gpu_ctx* ctx) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return INGOT_GPU_EHIP;
    if (cur != ctx->device && hipSetDevice(ctx->device) != hipSuccess) return INGOT_GPU_EHIP;
    return INGOT_GPU_SUCCESS;
}

// The context's tuning for a call over `arena`: frames in mapped host memory
// get the host-arena window defaults (launch_parse).
ingot_gpu::Tuning tuning_for(ingot_gpu_ctx* ctx, const void* arena) {
    ingot_gpu::Tuning t = ctx->tuning;
    const uintptr_t a = (uintptr_t)arena;
    std::lock_guard<std::mutex> g(ctx->mu);
    for (const auto& m : ctx->host)
        if (a >= m.dev && a < m.dev + m.bytes) t.host_arena = true;
    return t;
}

// Drop one reference to the library's registration holding [h, h + n); the
// last one unregisters it.  Caller holds g_reg_mu.
void release_registration(uintptr_t h, uintptr_t n) {
    for (size_t i = 0; i < g_regs.size(); ++i) {
        Registration& r = g_regs[i];
        if (h < r.host || h + n > r.host + r.bytes) continue;
        if (--r.refs == 0) {
            if (hipHostUnregister(reinterpret_cast<void*>(r.host)) != hipSuccess)
                (void)hipGetLastError();
            g_regs.erase(g_regs.begin() + (long)i);
        }
        return;
    }
}

int stride_ok(const uint8_t* d_arena, uint32_t stride) {
    if (stride == 0 || stride % 16u != 0 || stride > 65535u) return INGOT_GPU_ERANGE;
    if (((uintptr_t)d_arena & 15u) != 0) return INGOT_GPU_EINVAL;
    return INGOT_GPU_SUCCESS;
}

int parse_indexed(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                  const uint16_t* d_len, uint64_t n, int chain, void* d_out, int mode,
                  void* stream) {
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_off || !d_len || !d_out) return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    ingot_gpu::ParseArgs a{d_arena, d_off, d_len, 0, n, d_out};
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_INDEXED, chain, mode,
                                            tuning_for(ctx, d_arena), (hipStream_t)stream));
}

int parse_strided(ingot_gpu_ctx* ctx, const uint8_t* d_arena, uint32_t stride,
                  const uint16_t* d_len, uint64_t n, int chain, void* d_out, int mode,
                  void* stream) {
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_out) return INGOT_GPU_EINVAL;
    if (int e = stride_ok(d_arena, stride)) return e;
    if (int e = enter(ctx)) return e;
    ingot_gpu::ParseArgs a{d_arena, nullptr, d_len, stride, n, d_out};
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_STRIDED, chain, mode,
                                            tuning_for(ctx, d_arena), (hipStream_t)stream));
}

// ingot_field -> (header kind, first bit, width): the setters' BE geometry
// (ethernet.rs:46-65, ip.rs:63-93 / 159-182, tcp.rs:9-30, udp.rs:8-15,
// icmp.rs:42-50, geneve.rs:16-44; layout rules packet/mod.rs:547-821).
struct FieldGeo {
    uint8_t kind;
    uint16_t bit;
    uint8_t bits;
};
constexpr FieldGeo kFieldGeo[INGOT_F_COUNT] = {
    {ingot_gpu::HK_ETH, 96, 16},
    {ingot_gpu::HK_VLAN, 0, 3},    {ingot_gpu::HK_VLAN, 3, 1},
    {ingot_gpu::HK_VLAN, 4, 12},   {ingot_gpu::HK_VLAN, 16, 16},
    {ingot_gpu::HK_V4, 0, 4},      {ingot_gpu::HK_V4, 4, 4},     {ingot_gpu::HK_V4, 8, 6},
    {ingot_gpu::HK_V4, 14, 2},     {ingot_gpu::HK_V4, 16, 16},   {ingot_gpu::HK_V4, 32, 16},
    {ingot_gpu::HK_V4, 48, 3},     {ingot_gpu::HK_V4, 51, 13},   {ingot_gpu::HK_V4, 64, 8},
    {ingot_gpu::HK_V4, 72, 8},     {ingot_gpu::HK_V4, 80, 16},   {ingot_gpu::HK_V4, 96, 32},
    {ingot_gpu::HK_V4, 128, 32},
    {ingot_gpu::HK_V6, 0, 4},      {ingot_gpu::HK_V6, 4, 6},     {ingot_gpu::HK_V6, 10, 2},
    {ingot_gpu::HK_V6, 12, 20},    {ingot_gpu::HK_V6, 32, 16},   {ingot_gpu::HK_V6, 48, 8},
    {ingot_gpu::HK_V6, 56, 8},
    {ingot_gpu::HK_TCP, 0, 16},    {ingot_gpu::HK_TCP, 16, 16},  {ingot_gpu::HK_TCP, 32, 32},
    {ingot_gpu::HK_TCP, 64, 32},   {ingot_gpu::HK_TCP, 96, 4},   {ingot_gpu::HK_TCP, 100, 4},
    {ingot_gpu::HK_TCP, 104, 8},   {ingot_gpu::HK_TCP, 112, 16}, {ingot_gpu::HK_TCP, 128, 16},
    {ingot_gpu::HK_TCP, 144, 16},
    {ingot_gpu::HK_UDP, 0, 16},    {ingot_gpu::HK_UDP, 16, 16},  {ingot_gpu::HK_UDP, 32, 16},
    {ingot_gpu::HK_UDP, 48, 16},
    {ingot_gpu::HK_ICMP, 0, 8},    {ingot_gpu::HK_ICMP, 8, 8},   {ingot_gpu::HK_ICMP, 16, 16},
    {ingot_gpu::HK_GENEVE, 0, 2},  {ingot_gpu::HK_GENEVE, 2, 6}, {ingot_gpu::HK_GENEVE, 8, 8},
    {ingot_gpu::HK_GENEVE, 16, 16}, {ingot_gpu::HK_GENEVE, 32, 24},
    {ingot_gpu::HK_GENEVE, 56, 8},
};

int parse_segmented(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_seg_off,
                    const uint16_t* d_seg_len, const uint32_t* d_pkt_seg, uint64_t n, int chain,
                    void* d_out, uint16_t* d_chunk, int mode, void* stream) {
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_seg_off || !d_seg_len || !d_pkt_seg || !d_out) return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    ingot_gpu::ParseArgs a{d_arena, d_seg_off, d_seg_len, 0, n, d_out, d_pkt_seg, d_chunk};
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_SEGMENTED, chain, mode,
                                            tuning_for(ctx, d_arena), (hipStream_t)stream));
}

}  // namespace

extern "C" {

int ingot_gpu_abi_version(void) { return INGOT_GPU_ABI_VERSION; }

const char* ingot_gpu_build_info(void) {
    return "ingot_gpu " __DATE__ " gfx950 (LDS-DMA staged wave-per-64-packet parse)";
}

int ingot_gpu_ctx_create(int device, ingot_gpu_ctx** out) {
    if (!out) return INGOT_GPU_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
        return INGOT_GPU_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return INGOT_GPU_EHIP;
    // Code objects are built for gfx950 only.
    if (prop.gcnArchName[0] && std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return INGOT_GPU_ENODEV;
    ingot_gpu_ctx* c = new (std::nothrow) ingot_gpu_ctx();  // value-initialised
    if (!c) return INGOT_GPU_ENOMEM;
    c->device = device;
    if (prop.multiProcessorCount > 0) c->tuning.cus = (uint32_t)prop.multiProcessorCount;
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) ==
            hipSuccess &&
        lds > 0)
        c->lds_bytes = (size_t)lds;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess &&
        khz > 0)
        c->wall_khz = (uint32_t)khz;
    *out = c;
    return INGOT_GPU_SUCCESS;
}

void ingot_gpu_ctx_destroy(ingot_gpu_ctx* ctx) {
    if (!ctx) return;
    {  // the context's mappings still open release their registrations
        std::lock_guard<std::mutex> g(g_reg_mu);
        std::lock_guard<std::mutex> c(ctx->mu);
        for (const HostMapping& m : ctx->host)
            if (m.owned) release_registration(m.host, m.bytes);
        ctx->host.clear();
    }
    delete ctx;
}

int ingot_gpu_ctx_device(const ingot_gpu_ctx* ctx) { return ctx ? ctx->device : -1; }

size_t ingot_gpu_packed_workspace_size(uint64_t n) { return ingot_gpu::packed_workspace(n); }

int ingot_gpu_parse_packed(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint16_t* d_len,
                           uint64_t n, int chain, ingot_rec* d_out, uint64_t* d_off_out,
                           void* d_work, size_t work_bytes, void* stream) {
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_len || !d_out || !d_work || ((uintptr_t)d_work & 7u)) return INGOT_GPU_EINVAL;
    if (work_bytes < ingot_gpu::packed_workspace(n)) return INGOT_GPU_ERANGE;
    if (int e = enter(ctx)) return e;
    const hipStream_t s = (hipStream_t)stream;
    if (int e = from_hip(ingot_gpu::launch_tile_bases(d_len, n, d_work, s))) return e;
    const uint64_t ngroups = ((n + 63) / 64 + ingot_gpu::PACKED_GROUP - 1) / ingot_gpu::PACKED_GROUP;
    ingot_gpu::ParseArgs a{d_arena, static_cast<const uint64_t*>(d_work), d_len, 0, n, d_out};
    a.tile_local = reinterpret_cast<const uint32_t*>(static_cast<const uint64_t*>(d_work) + ngroups);
    a.off_out = d_off_out;
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_PACKED, chain,
                                            ingot_gpu::OUT_REC16, tuning_for(ctx, d_arena), s));
}

int ingot_gpu_parse_header(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                           const uint16_t* d_len, uint32_t stride, uint64_t n, int kind,
                           const uint32_t* d_hint, uint32_t hint, ingot_hdr* d_out,
                           void* stream) {
    const bool kind_ok = (kind >= INGOT_HDR_ETHERNET && kind <= INGOT_HDR_GENEVE) ||
                         (kind >= INGOT_HDR_L3 && kind <= INGOT_HDR_ULP);
    if (!ctx || !kind_ok) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_out) return INGOT_GPU_EINVAL;
    if (d_off) {
        if (!d_len) return INGOT_GPU_EINVAL;
        stride = 0;
    } else if (stride == 0 || stride > 65535u) {
        return INGOT_GPU_ERANGE;
    }
    if (int e = enter(ctx)) return e;
    ingot_gpu::HeaderArgs a{d_arena, d_off, d_len, stride, n, kind, d_hint, hint, d_out};
    return from_hip(ingot_gpu::launch_header(a, (hipStream_t)stream));
}

int ingot_gpu_host_map(ingot_gpu_ctx* ctx, void* host, size_t bytes, void** d_ptr) {
    if (!ctx || !host || !d_ptr || bytes == 0) return INGOT_GPU_EINVAL;
    *d_ptr = nullptr;
    const uintptr_t h = (uintptr_t)host;
    if (h + bytes < h) return INGOT_GPU_ERANGE;
    if (int e = enter(ctx)) return e;
    std::lock_guard<std::mutex> g(g_reg_mu);
    HostMapping m{h, bytes, 0, false};
    // 1. inside one of our registrations: one more reference to it
    for (Registration& r : g_regs) {
        if (h >= r.host && h + bytes <= r.host + r.bytes) {
            ++r.refs;
            m.dev = r.dev + (h - r.host);
            m.owned = true;
            break;
        }
        // partly overlapping bytes we registered: the rest is not ours to
        // register, and a second registration of the same bytes is refused
        if (h < r.host + r.bytes && r.host < h + bytes) return INGOT_GPU_EINVAL;
    }
    if (!m.owned) {
        // 2. pinned and mapped by someone else (hipHostMalloc, the caller's
        //    own hipHostRegister): used as it is, never unregistered here
        hipPointerAttribute_t attr;
        void* d = nullptr;
        if (hipPointerGetAttributes(&attr, host) == hipSuccess &&
            attr.type == hipMemoryTypeHost && hipHostGetDevicePointer(&d, host, 0) == hipSuccess) {
            m.dev = (uintptr_t)d;
        } else {
            // 3. pageable: page-lock and map exactly these bytes (pages
            //    shared with neighbours stay usable by them)
            (void)hipGetLastError();  // clear the probe's error
            if (hipHostRegister(host, bytes, hipHostRegisterMapped) != hipSuccess) {
                (void)hipGetLastError();
                return INGOT_GPU_EHIP;
            }
            if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
                (void)hipHostUnregister(host);
                (void)hipGetLastError();
                return INGOT_GPU_EHIP;
            }
            m.dev = (uintptr_t)d;
            m.owned = true;
            g_regs.push_back(Registration{h, bytes, m.dev, 1u});
        }
    }
    {
        std::lock_guard<std::mutex> c(ctx->mu);
        ctx->host.push_back(m);
    }
    *d_ptr = reinterpret_cast<void*>(m.dev);
    return INGOT_GPU_SUCCESS;
}

int ingot_gpu_host_unmap(ingot_gpu_ctx* ctx, void* host) {
    if (!ctx || !host) return INGOT_GPU_EINVAL;
    const uintptr_t h = (uintptr_t)host;
    std::lock_guard<std::mutex> g(g_reg_mu);
    HostMapping m{};
    {
        std::lock_guard<std::mutex> c(ctx->mu);
        size_t i = ctx->host.size();
        while (i > 0 && ctx->host[i - 1].host != h) --i;  // the latest mapping of `host`
        if (i == 0) return INGOT_GPU_EINVAL;               // not mapped by this context
        m = ctx->host[i - 1];
        ctx->host.erase(ctx->host.begin() + (long)(i - 1));
    }
    if (m.owned) release_registration(m.host, m.bytes);  // registrations are per process
    return INGOT_GPU_SUCCESS;
}

// Doorbell: one pinned, coherent host word the command processor polls
// (hipStreamWaitValue32).  Host stores to coherent memory are seen by the
// device without a flush.
struct ingot_gpu_doorbell {
    int device = 0;
    uint32_t* word;
    uint32_t* dword = nullptr;  // the word's device address (ingot_gpu_parse_ring polls it)
};

int ingot_gpu_doorbell_create(ingot_gpu_ctx* ctx, ingot_gpu_doorbell** out,
                              volatile uint32_t** host_word) {
    if (!ctx || !out) return INGOT_GPU_EINVAL;
    *out = nullptr;
    if (host_word) *host_word = nullptr;
    if (int e = enter(ctx)) return e;
    int can = 0;
    if (hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, ctx->device) !=
            hipSuccess ||
        !can)
        return INGOT_GPU_ENODEV;
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        return INGOT_GPU_EHIP;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
        (void)hipHostFree(p);
        return INGOT_GPU_EHIP;
    }
    ingot_gpu_doorbell* d =
        new (std::nothrow) ingot_gpu_doorbell{ctx->device, (uint32_t*)p, (uint32_t*)dp};
    if (!d) {
        (void)hipHostFree(p);
        return INGOT_GPU_ENOMEM;
    }
    __atomic_store_n(d->word, 0u, __ATOMIC_SEQ_CST);
    *out = d;
    if (host_word) *host_word = d->word;
    return INGOT_GPU_SUCCESS;
}

int ingot_gpu_doorbell_wait(ingot_gpu_doorbell* db, uint32_t value, void* stream) {
    if (!db) return INGOT_GPU_EINVAL;
    return from_hip(hipStreamWaitValue32((hipStream_t)stream, db->word, value,
                                         hipStreamWaitValueGte, 0xffffffffu));
}

int ingot_gpu_doorbell_ring(ingot_gpu_doorbell* db, uint32_t value) {
    if (!db) return INGOT_GPU_EINVAL;
    __atomic_store_n(db->word, value, __ATOMIC_SEQ_CST);
    return INGOT_GPU_SUCCESS;
}

int ingot_gpu_stream_delay(ingot_gpu_ctx* ctx, uint32_t ns, void* stream) {
    if (!ctx) return INGOT_GPU_EINVAL;
    if (ns == 0) return INGOT_GPU_SUCCESS;
    if (!ctx->wall_khz) return INGOT_GPU_ENODEV;
    if (int e = enter(ctx)) return e;
    const uint64_t ticks = ((uint64_t)ns * ctx->wall_khz + 999999u) / 1000000u;
    return from_hip(ingot_gpu::launch_delay(ticks, (hipStream_t)stream));
}

void ingot_gpu_doorbell_destroy(ingot_gpu_doorbell* db) {
    if (!db) return;
    (void)hipHostFree(db->word);
    delete db;
}

int ingot_gpu_ctx_set_tuning(ingot_gpu_ctx* ctx, int key, int value) {
    if (!ctx || !ingot_gpu::tuning_valid(key, value)) return INGOT_GPU_EINVAL;
    switch (key) {
    case INGOT_TUNE_WINDOW_INDEXED: ctx->tuning.window_indexed = value; break;
    case INGOT_TUNE_WINDOW_STRIDED: ctx->tuning.window_strided = value; break;
    case INGOT_TUNE_PIPELINE: ctx->tuning.pipeline = value; break;
    case INGOT_TUNE_CACHE_POLICY: ctx->tuning.cache_policy = value; break;
    case INGOT_TUNE_PIPE_DEPTH: ctx->tuning.pipe_depth = value; break;
    case INGOT_TUNE_WRITEBACK: ctx->tuning.writeback = value; break;
    case INGOT_TUNE_FLOW_TABLE: ctx->tuning.flow_table = value; break;
    case INGOT_TUNE_SLOW_PATH: ctx->tuning.slow_path = value; break;
    case INGOT_TUNE_READ_PLAN: ctx->tuning.read_plan = value; break;
    case INGOT_TUNE_FLOW_KERNEL: ctx->tuning.flow_kernel = value; break;
    case INGOT_TUNE_RING_GRID: ctx->tuning.ring_grid = value; break;
    case INGOT_TUNE_RING_GROUPS: ctx->tuning.ring_groups = value; break;
    case INGOT_TUNE_XCD_REMAP: ctx->tuning.xcd_remap = value; break;
    default: ctx->tuning.max_blocks = (uint32_t)value; break;
    }
    return INGOT_GPU_SUCCESS;
}

int ingot_gpu_ctx_get_tuning(const ingot_gpu_ctx* ctx, int key) {
    if (!ctx) return INGOT_GPU_EINVAL;
    switch (key) {
    case INGOT_TUNE_WINDOW_INDEXED: return ctx->tuning.window_indexed;
    case INGOT_TUNE_WINDOW_STRIDED: return ctx->tuning.window_strided;
    case INGOT_TUNE_MAX_BLOCKS: return (int)ctx->tuning.max_blocks;
    case INGOT_TUNE_PIPELINE: return ctx->tuning.pipeline;
    case INGOT_TUNE_CACHE_POLICY: return ctx->tuning.cache_policy;
    case INGOT_TUNE_PIPE_DEPTH: return ctx->tuning.pipe_depth;
    case INGOT_TUNE_WRITEBACK: return ctx->tuning.writeback;
    case INGOT_TUNE_FLOW_TABLE: return ctx->tuning.flow_table;
    case INGOT_TUNE_SLOW_PATH: return ctx->tuning.slow_path;
    case INGOT_TUNE_READ_PLAN: return ctx->tuning.read_plan;
    case INGOT_TUNE_FLOW_KERNEL: return ctx->tuning.flow_kernel;
    case INGOT_TUNE_RING_GRID: return ctx->tuning.ring_grid;
    case INGOT_TUNE_RING_GROUPS: return ctx->tuning.ring_groups;
    case INGOT_TUNE_XCD_REMAP: return ctx->tuning.xcd_remap;
    default: return INGOT_GPU_EINVAL;
    }
}

int ingot_gpu_parse(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                    const uint16_t* d_len, uint64_t n, int chain, ingot_rec* d_out,
                    void* stream) {
    return parse_indexed(ctx, d_arena, d_off, d_len, n, chain, d_out, ingot_gpu::OUT_REC16,
                         stream);
}

int ingot_gpu_parse_strided(ingot_gpu_ctx* ctx, const uint8_t* d_arena, uint32_t stride,
                            const uint16_t* d_len, uint64_t n, int chain, ingot_rec* d_out,
                            void* stream) {
    return parse_strided(ctx, d_arena, stride, d_len, n, chain, d_out, ingot_gpu::OUT_REC16,
                         stream);
}

int ingot_gpu_parse_ring(ingot_gpu_ctx* ctx, const ingot_ring_batch* batches, uint32_t nbatches,
                         uint32_t stride, uint64_t n, int chain, uint32_t record_bytes,
                         const ingot_gpu_doorbell* db, uint32_t db_first, uint32_t timeout_ms,
                         uint32_t* d_status, void* stream) {
    if (!ctx || !chain_ok(chain) || chain == INGOT_CHAIN_GENEVE_OVER_V6) return INGOT_GPU_EINVAL;
    if (record_bytes != 16 && record_bytes != 8) return INGOT_GPU_EINVAL;
    if (nbatches > INGOT_RING_MAX_BATCHES) return INGOT_GPU_ERANGE;
    if (stride < 64u || stride % 16u != 0 || stride > 65535u) return INGOT_GPU_ERANGE;
    if (db && (timeout_ms == 0 || timeout_ms > 60000u)) return INGOT_GPU_ERANGE;
    // the kernel compares the word with db_first + b (b < nbatches) in 32
    // bits: the largest, db_first + nbatches - 1, must not wrap
    if (db && nbatches && (uint64_t)db_first + nbatches - 1u > 0xffffffffull)
        return INGOT_GPU_ERANGE;
    if (db && db->device != ctx->device) return INGOT_GPU_EINVAL;
    if (nbatches == 0 || n == 0) return INGOT_GPU_SUCCESS;
    if (!batches) return INGOT_GPU_EINVAL;
    // the kernel's tile cursors are 32-bit
    const uint64_t tiles = (n + 63u) / 64u;
    if (tiles * nbatches >= (1ull << 31)) return INGOT_GPU_ERANGE;
    ingot_gpu::RingArgs a{};
    for (uint32_t b = 0; b < nbatches; ++b) {
        const ingot_ring_batch& x = batches[b];
        if (!x.d_arena || !x.d_out || ((uintptr_t)x.d_arena & 15u)) return INGOT_GPU_EINVAL;
        a.b[b] = ingot_gpu::RingBatch{x.d_arena, x.d_out};
    }
    if (db && !ctx->wall_khz) return INGOT_GPU_ENODEV;
    if (int e = enter(ctx)) return e;
    a.n = n;
    a.stride = stride;
    a.nbatches = nbatches;
    a.tiles_per_batch = (uint32_t)tiles;
    a.published = db ? 0u : nbatches;
    a.doorbell = db ? db->dword : nullptr;
    a.db_first = db_first;
    a.timeout_ticks = (uint64_t)timeout_ms * ctx->wall_khz;
    a.status = d_status;
    return from_hip(ingot_gpu::launch_ring(a, chain,
                                           record_bytes == 8 ? ingot_gpu::OUT_REC8
                                                             : ingot_gpu::OUT_REC16,
                                           tuning_for(ctx, batches[0].d_arena),
                                           (hipStream_t)stream));
}

int ingot_gpu_parse_compact(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                            const uint16_t* d_len, uint64_t n, int chain, ingot_rec8* d_out,
                            void* stream) {
    if (chain == INGOT_CHAIN_GENEVE_OVER_V6) return INGOT_GPU_EINVAL;
    return parse_indexed(ctx, d_arena, d_off, d_len, n, chain, d_out, ingot_gpu::OUT_REC8,
                         stream);
}

int ingot_gpu_parse_strided_compact(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                                    uint32_t stride, const uint16_t* d_len, uint64_t n,
                                    int chain, ingot_rec8* d_out, void* stream) {
    if (chain == INGOT_CHAIN_GENEVE_OVER_V6) return INGOT_GPU_EINVAL;
    return parse_strided(ctx, d_arena, stride, d_len, n, chain, d_out, ingot_gpu::OUT_REC8,
                         stream);
}

int ingot_gpu_fields(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                     const uint16_t* d_len, uint32_t stride, uint64_t n, int chain,
                     ingot_fields* d_out, void* stream) {
    if (chain == INGOT_CHAIN_GENEVE_OVER_V6) return INGOT_GPU_EINVAL;  // 384-B blocks
    if (d_off)
        return parse_indexed(ctx, d_arena, d_off, d_len, n, chain, d_out, ingot_gpu::OUT_FIELDS,
                             stream);
    return parse_strided(ctx, d_arena, stride, d_len, n, chain, d_out, ingot_gpu::OUT_FIELDS,
                         stream);
}

int ingot_gpu_geneve_fields(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                            const uint16_t* d_len, uint32_t stride, uint64_t n,
                            ingot_geneve_fields* d_out, void* stream) {
    const int chain = INGOT_CHAIN_GENEVE_OVER_V6;
    if (d_off)
        return parse_indexed(ctx, d_arena, d_off, d_len, n, chain, d_out, ingot_gpu::OUT_FIELDS,
                             stream);
    return parse_strided(ctx, d_arena, stride, d_len, n, chain, d_out, ingot_gpu::OUT_FIELDS,
                         stream);
}

int ingot_gpu_parse_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_seg_off,
                         const uint16_t* d_seg_len, const uint32_t* d_pkt_seg, uint64_t n,
                         int chain, ingot_rec* d_out, uint16_t* d_chunk, void* stream) {
    return parse_segmented(ctx, d_arena, d_seg_off, d_seg_len, d_pkt_seg, n, chain, d_out,
                           d_chunk, ingot_gpu::OUT_REC16, stream);
}

int ingot_gpu_parse_read_first(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                               const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                               const uint32_t* d_pkt_seg, const uint64_t* d_first, uint64_t n,
                               int chain, ingot_rec* d_out, uint16_t* d_chunk, void* stream) {
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_seg_off || !d_seg_len || !d_pkt_seg || !d_first || !d_out)
        return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    ingot_gpu::ParseArgs a{d_arena, d_seg_off, d_seg_len, 0, n, d_out, d_pkt_seg, d_chunk};
    a.first = d_first;
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_SEGMENTED, chain,
                                            ingot_gpu::OUT_REC16, tuning_for(ctx, d_arena),
                                            (hipStream_t)stream));
}

int ingot_gpu_fields_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_seg_off,
                          const uint16_t* d_seg_len, const uint32_t* d_pkt_seg, uint64_t n,
                          int chain, ingot_fields* d_out, uint16_t* d_chunk, void* stream) {
    if (chain == INGOT_CHAIN_GENEVE_OVER_V6) return INGOT_GPU_EINVAL;  // 384-B blocks
    return parse_segmented(ctx, d_arena, d_seg_off, d_seg_len, d_pkt_seg, n, chain, d_out,
                           d_chunk, ingot_gpu::OUT_FIELDS, stream);
}

int ingot_gpu_geneve_fields_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                                 const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                                 const uint32_t* d_pkt_seg, uint64_t n,
                                 ingot_geneve_fields* d_out, uint16_t* d_chunk, void* stream) {
    return parse_segmented(ctx, d_arena, d_seg_off, d_seg_len, d_pkt_seg, n,
                           INGOT_CHAIN_GENEVE_OVER_V6, d_out, d_chunk, ingot_gpu::OUT_FIELDS,
                           stream);
}

int ingot_gpu_parse_read_dense(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_seg,
                               const uint32_t* d_pkt_seg, uint64_t n, int chain, int fields,
                               void* d_out, uint16_t* d_chunk, void* stream) {
    if (!ctx || !chain_ok(chain) || fields < 0 || fields > 2) return INGOT_GPU_EINVAL;
    if ((fields == 1 && chain == INGOT_CHAIN_GENEVE_OVER_V6) ||
        (fields == 2 && chain != INGOT_CHAIN_GENEVE_OVER_V6))
        return INGOT_GPU_EINVAL;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_seg || !d_pkt_seg || !d_out) return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    // len == NULL selects the dense table (launch_parse)
    ingot_gpu::ParseArgs a{d_arena, d_seg, nullptr, 0, n, d_out, d_pkt_seg, d_chunk};
    return from_hip(ingot_gpu::launch_parse(a, ingot_gpu::LAYOUT_SEGMENTED, chain,
                                            fields ? ingot_gpu::OUT_FIELDS : ingot_gpu::OUT_REC16,
                                            tuning_for(ctx, d_arena), (hipStream_t)stream));
}

int ingot_gpu_parse_modify(ingot_gpu_ctx* ctx, uint8_t* d_arena, const uint64_t* d_off,
                           const uint16_t* d_len, uint32_t stride, uint64_t n, int chain,
                           const ingot_edit* edits, uint32_t n_edits, ingot_rec* d_out,
                           void* stream) {
    if (!ctx || !chain_ok(chain) || n_edits > INGOT_MAX_EDITS || (n_edits && !edits))
        return INGOT_GPU_EINVAL;
    ingot_gpu::ModifyArgs a{};
    for (uint32_t k = 0; k < n_edits; ++k) {
        const ingot_edit& e = edits[k];
        if (e.field >= INGOT_F_COUNT || e.op > INGOT_OP_XOR ||
            (int)e.layer >= ingot_chain_layer_count(chain))
            return INGOT_GPU_EINVAL;
        const FieldGeo g = kFieldGeo[e.field];
        ingot_gpu::Edit& d = a.e[k];
        d.layer = e.layer;
        d.kind = g.kind;
        d.op = e.op;
        d.index = e.index;
        d.byte0 = (uint8_t)(g.bit / 8u);
        d.nbytes = (uint8_t)((g.bit % 8u + g.bits + 7u) / 8u);
        d.rshift = (uint8_t)((8u - ((g.bit + g.bits) % 8u)) % 8u);
        d.bits = g.bits;
        d.value = e.value;
    }
    a.n_edits = n_edits;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena) return INGOT_GPU_EINVAL;
    int layout = ingot_gpu::LAYOUT_INDEXED;
    if (!d_off) {
        if (int e = stride_ok(d_arena, stride)) return e;
        layout = ingot_gpu::LAYOUT_STRIDED;
    } else if (!d_len) {
        return INGOT_GPU_EINVAL;
    }
    if (int e = enter(ctx)) return e;
    a.p = ingot_gpu::ParseArgs{d_arena, d_off, d_len, stride, n, d_out};
    return from_hip(ingot_gpu::launch_modify(a, layout, chain, tuning_for(ctx, d_arena),
                                             (hipStream_t)stream));
}

}  // extern "C"

namespace {

// The header block and its setters -> EmitArgs (shared by both emit calls).
int emit_args(const uint8_t* hdr, uint32_t hdr_len, const ingot_emit_set* sets,
              uint32_t n_sets, ingot_gpu::EmitArgs& a) {
    if (hdr_len > INGOT_MAX_EMIT_HDR || (hdr_len && !hdr) || n_sets > INGOT_MAX_EMIT_SETS ||
        (n_sets && !sets))
        return INGOT_GPU_EINVAL;
    if (hdr_len) std::memcpy(a.hdr, hdr, hdr_len);  // the rest stays zero
    a.hdr_len = hdr_len;
    for (uint32_t k = 0; k < n_sets; ++k) {
        const ingot_emit_set& e = sets[k];
        if (e.field >= INGOT_F_COUNT || e.source > INGOT_EMIT_VALUE) return INGOT_GPU_EINVAL;
        if ((e.source == INGOT_EMIT_U16 || e.source == INGOT_EMIT_U32) && !e.d_values)
            return INGOT_GPU_EINVAL;
        const FieldGeo g = kFieldGeo[e.field];
        ingot_gpu::EmitSet& d = a.sets[k];
        const uint32_t pos = (uint32_t)e.at + g.bit / 8u;  // 32 bits: no wrap before the check
        d.nbytes = (uint8_t)((g.bit % 8u + g.bits + 7u) / 8u);
        if (pos + d.nbytes > hdr_len) return INGOT_GPU_EINVAL;  // field inside hdr
        d.pos = (uint16_t)pos;
        d.rshift = (uint8_t)((8u - ((g.bit + g.bits) % 8u)) % 8u);
        d.bits = g.bits;
        d.source = e.source;
        d.at = e.at;
        d.add = e.add;
        d.values = e.d_values;
    }
    a.n_sets = n_sets;
    return INGOT_GPU_SUCCESS;
}

// The device's LDS per workgroup must hold one emit block's (ERANGE if not).
int emit_fits(const ingot_gpu_ctx* ctx, const ingot_gpu::EmitArgs& a) {
    return ingot_gpu::emit_lds_bytes(a) <= ctx->lds_bytes ? INGOT_GPU_SUCCESS : INGOT_GPU_ERANGE;
}

}  // namespace

extern "C" {

int ingot_gpu_emit_packets(ingot_gpu_ctx* ctx, const uint8_t* hdr, uint32_t hdr_len,
                           const ingot_emit_set* sets, uint32_t n_sets, const uint8_t* d_src,
                           const uint64_t* d_off, const uint16_t* d_len, uint64_t n,
                           uint8_t* d_dst, const uint64_t* d_dst_off, void* stream) {
    if (!ctx) return INGOT_GPU_EINVAL;
    ingot_gpu::EmitArgs a{};
    if (int e = emit_args(hdr, hdr_len, sets, n_sets, a)) return e;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_src || !d_off || !d_len || !d_dst || !d_dst_off) return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    a.src = d_src;
    a.off = d_off;
    a.len = d_len;
    a.dst = d_dst;
    a.dst_off = d_dst_off;
    a.n = n;
    if (int e = emit_fits(ctx, a)) return e;
    return from_hip(ingot_gpu::launch_emit(a, (hipStream_t)stream));
}

int ingot_gpu_emit_headers(ingot_gpu_ctx* ctx, const uint8_t* hdr, uint32_t hdr_len,
                           const ingot_emit_set* sets, uint32_t n_sets, const uint16_t* d_len,
                           uint64_t n, uint8_t* d_out, const uint64_t* d_out_off,
                           uint32_t out_stride, void* stream) {
    if (!ctx) return INGOT_GPU_EINVAL;
    ingot_gpu::EmitArgs a{};
    if (int e = emit_args(hdr, hdr_len, sets, n_sets, a)) return e;
    if (!d_out_off && out_stride < hdr_len) return INGOT_GPU_ERANGE;  // blocks would overlap
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_len || !d_out || hdr_len == 0) return INGOT_GPU_EINVAL;
    if (int e = enter(ctx)) return e;
    a.len = d_len;
    a.dst = d_out;
    a.dst_off = d_out_off;
    a.stride = out_stride;
    a.n = n;
    if (int e = emit_fits(ctx, a)) return e;
    return from_hip(ingot_gpu::launch_emit(a, (hipStream_t)stream));
}

int ingot_gpu_flow_hist_ws(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                           const uint16_t* d_len, uint32_t stride, uint64_t n, int chain,
                           const uint8_t* key, uint32_t bins, uint32_t* d_flow, uint32_t* d_hash,
                           uint32_t* d_hist, void* d_work, size_t work_bytes, void* stream) {
    // The standard Microsoft RSS key (the one its published verification
    // vectors use; tests/test_flows.py).
    static const uint8_t kRssKey[INGOT_FLOW_KEY_BYTES] = {
        0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2, 0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3,
        0x8f, 0xb0, 0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4, 0x77, 0xcb, 0x2d, 0xa3,
        0x80, 0x30, 0xf2, 0x0c, 0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa};
    if (!ctx || !chain_ok(chain)) return INGOT_GPU_EINVAL;
    if (bins == 0 || (bins & (bins - 1)) != 0 || bins > (1u << 24)) return INGOT_GPU_ERANGE;
    if (n == 0) return INGOT_GPU_SUCCESS;
    if (!d_arena || !d_flow) return INGOT_GPU_EINVAL;
    int layout = ingot_gpu::LAYOUT_INDEXED;
    if (!d_off) {
        if (int e = stride_ok(d_arena, stride)) return e;
        layout = ingot_gpu::LAYOUT_STRIDED;
    } else if (!d_len) {
        return INGOT_GPU_EINVAL;
    }
    if (int e = enter(ctx)) return e;
    const uint8_t* k = key ? key : kRssKey;
    ingot_gpu::FlowArgs a{};
    a.p = ingot_gpu::ParseArgs{d_arena, d_off, d_len, stride, n, nullptr};
    a.flow = d_flow;
    a.bin_mask = bins - 1u;
    a.hash = d_hash;
    for (uint32_t b = 0; b < ingot_gpu::FLOW_INPUT_BITS; ++b) {
        uint32_t w = 0;
        for (uint32_t j = 0; j < 32; ++j) {
            const uint32_t bit = b + j;
            w = (w << 1) | ((k[bit >> 3] >> (7u - (bit & 7u))) & 1u);
        }
        a.w[b] = w;
    }
    // the 16-bit table: entry (p, v) = low 16 bits of the XOR of the windows
    // of v's set bits at nibble position p (bit 3 of v = input bit 4p)
    for (uint32_t e = 0; e < 2 * ingot_gpu::FLOW_TAB16_DW; ++e) {
        const uint32_t p = e / 16u, v = e & 15u;
        uint32_t acc = 0;
        for (uint32_t j = 0; j < 4; ++j)
            if ((v >> (3u - j)) & 1u) acc ^= a.w[4u * p + j];
        a.tab16[e / 2] |= (acc & 0xffffu) << (16u * (e & 1u));
    }
    const hipStream_t s = (hipStream_t)stream;
    if (int e = from_hip(ingot_gpu::launch_flows(a, layout, chain, tuning_for(ctx, d_arena), s)))
        return e;
    if (!d_hist) return INGOT_GPU_SUCCESS;
    return from_hip(ingot_gpu::launch_flow_hist(d_flow, n, d_hist, bins, d_work, work_bytes, s));
}

int ingot_gpu_flow_hist(ingot_gpu_ctx* ctx, const uint8_t* d_arena, const uint64_t* d_off,
                        const uint16_t* d_len, uint32_t stride, uint64_t n, int chain,
                        const uint8_t* key, uint32_t bins, uint32_t* d_flow, uint32_t* d_hash,
                        uint32_t* d_hist, void* stream) {
    return ingot_gpu_flow_hist_ws(ctx, d_arena, d_off, d_len, stride, n, chain, key, bins, d_flow,
                                  d_hash, d_hist, nullptr, 0, stream);
}

size_t ingot_gpu_flow_hist_workspace_size(uint64_t n, uint32_t bins) {
    if (bins == 0 || (bins & (bins - 1)) != 0 || bins > (1u << 24)) return 0;
    return ingot_gpu::flow_hist_workspace(n, bins);
}

const char* ingot_gpu_strerror(int code) {
    switch (code) {
    case INGOT_GPU_SUCCESS: return "success";
    case INGOT_GPU_EINVAL: return "invalid argument";
    case INGOT_GPU_EHIP: return "HIP runtime error";
    case INGOT_GPU_ENOMEM: return "out of host memory";
    case INGOT_GPU_ENODEV: return "no such gfx950 device";
    case INGOT_GPU_ERANGE: return "size outside the supported range";
    case INGOT_GPU_ECOMM: return "collective (RCCL) call failed";
    default: return "unknown error";
    }
}

const char* ingot_parse_error_name(int status) {
    if (status < 0 || status > INGOT_ERR_ILLEGAL_VALUE) return nullptr;
    return kParseErrorNames[status];
}

int ingot_chain_layer_count(int chain) {
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER: return 3;
    case INGOT_CHAIN_GENERIC_ULP: return 3;
    case INGOT_CHAIN_VLAN_ULP: return 4;
    case INGOT_CHAIN_GENEVE_OVER_V6: return 7;
    default: return -1;
    }
}

const char* ingot_chain_layer_label(int chain, int layer) {
    if (layer < 0 || layer >= ingot_chain_layer_count(chain)) return nullptr;
    switch (chain) {
    case INGOT_CHAIN_UDP_PARSER: return kUdpParserLabels[layer];
    case INGOT_CHAIN_GENERIC_ULP: return kGenericUlpLabels[layer];
    case INGOT_CHAIN_VLAN_ULP: return kVlanUlpLabels[layer];
    default: return kGeneveLabels[layer];
    }
}

}  // extern "C"
