// kernels.h — internal interface between the C ABI (api.cpp) and the HIP
// kernels (parse.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ingot_gpu.h"

namespace ingot_gpu {

// STRIDED: frame i at i*stride; INDEXED: (off[i], len[i]); SEGMENTED: packet i
// is the chunks pkt_seg[i] .. pkt_seg[i+1] of (off, len) = (seg_off, seg_len),
// walked with parse_read's chunk semantics (read.hip).
// PACKED: frames back to back with only a length array; `off` holds one u64
// base per group of tiles and `tile_local` each tile's prefix in its group
// (packed.hip); the frame offsets come from a wavefront prefix scan of the
// tile's lengths.
enum LayoutKind { LAYOUT_STRIDED = 0, LAYOUT_INDEXED = 1, LAYOUT_SEGMENTED = 2, LAYOUT_PACKED = 3 };

// Output mode: 16-B ingot_rec, 8-B ingot_rec8, 256-B ingot_fields, or the
// flow hash + histogram (OUT_FLOWS16: only the hash's low 16 bits, enough for
// <= 65,536 bins when the full hash is not requested — half the LDS table).
enum OutMode {
    OUT_REC16 = 0,
    OUT_REC8 = 1,
    OUT_FIELDS = 2,
    OUT_FLOWS = 3,
    OUT_MODIFY = 4,
    OUT_FLOWS16 = 5
};

// Toeplitz key windows: w[b] = the 32 key bits starting at input bit b, for
// every bit of the longest input (IPv6 src|dst|ports = 36 bytes).
constexpr uint32_t FLOW_INPUT_BITS = 36 * 8;
// The 16-bit nibble table (OUT_FLOWS16), in dwords: 72 positions x 16 values
// x 2 B.  Computed once per call on the host (api.cpp) and passed with the
// kernel arguments, so a block loads it instead of building it.
constexpr uint32_t FLOW_TAB16_DW = FLOW_INPUT_BITS / 4 * 16 / 2;

struct ParseArgs {
    const uint8_t* arena;
    const uint64_t* off;   // LAYOUT_INDEXED (LAYOUT_SEGMENTED: per chunk)
    const uint16_t* len;   // optional for LAYOUT_STRIDED (LAYOUT_SEGMENTED: per chunk)
    uint32_t stride;       // LAYOUT_STRIDED
    uint64_t n;
    void* out;             // n records of the OutMode's type
    const uint32_t* pkt_seg = nullptr;  // LAYOUT_SEGMENTED: n+1 chunk-index bounds
    uint16_t* chunk = nullptr;          // LAYOUT_SEGMENTED, optional: remainder's chunk
    uint64_t* off_out = nullptr;        // LAYOUT_PACKED, optional: the computed offsets
    const uint32_t* tile_local = nullptr;  // LAYOUT_PACKED: tile prefix within its group
    uint32_t policy = 0;                // INGOT_TUNE_CACHE_POLICY bits (launch_parse sets it)
    uint32_t linewin = 0;  // windows from byte 12: >= linewin chunks, then to the line end
    // LAYOUT_SEGMENTED, optional (ingot_gpu_parse_read_first): per packet,
    // chunk 0's (offset << 16) | length, indexed like pkt_seg
    const uint64_t* first = nullptr;
    uint32_t xcd_remap = 0;  // k_parse_pipe: logical block = XCD-major (INGOT_TUNE_XCD_REMAP)
};

struct FlowArgs {
    ParseArgs p;
    uint32_t* flow;  // per-packet bin or INGOT_FLOW_NONE
    uint32_t bin_mask;
    uint32_t* hash;  // optional
    uint32_t w[FLOW_INPUT_BITS];
    alignas(16) uint32_t tab16[FLOW_TAB16_DW];  // entry (p, v) at half-word 16p + v
};

// In-place rewrite (ingot_gpu_parse_modify): api.cpp resolves each ingot_edit's
// field to its header kind and BE bit geometry, so the kernel needs no tables.
enum HdrKind : uint8_t { HK_ETH, HK_VLAN, HK_V4, HK_V6, HK_TCP, HK_UDP, HK_ICMP, HK_GENEVE };
struct Edit {
    uint8_t layer, kind, op, index;
    uint8_t byte0, nbytes, rshift, bits;  // field bytes [byte0, byte0+nbytes) of the header
    uint32_t value;
};
struct ModifyArgs {
    ParseArgs p;
    uint32_t wb = 32;  // ring kernel: write-back unit in bytes (16, 32, 64)
    uint32_t n_edits;
    Edit e[INGOT_MAX_EDITS];
};
// 3,824 B today (ParseArgs + key windows + the 16-bit table): the kernarg
// segment is 4 KiB, and a larger FlowArgs would fail flow launches at run
// time, not here.
static_assert(sizeof(FlowArgs) <= 4096, "FlowArgs exceeds the 4 KiB kernel-argument limit");

// Persistent ring consumer (ingot_gpu_parse_ring): one launch parses up to
// INGOT_RING_MAX_BATCHES batches of n fixed slots, batch b from b.arena into
// b.out; tiles of batch b are staged only once b is published (b < published,
// or the doorbell word reaches db_first + b).
struct RingBatch {
    const uint8_t* arena;
    void* out;
};
struct RingArgs {
    uint64_t n;               // frames per batch
    uint32_t stride;          // slot bytes (>= 64, multiple of 16)
    uint32_t nbatches;
    uint32_t policy;          // INGOT_TUNE_CACHE_POLICY bits
    uint32_t published;       // batches known published at launch (no poll below)
    const uint32_t* doorbell; // device address of the doorbell word, or NULL
    uint32_t db_first;        // doorbell value that publishes batch 0
    uint32_t tiles_per_batch;
    uint64_t timeout_ticks;   // wall-clock ticks a wave waits for a batch
    uint32_t* status;         // optional: |= 1 when a wave gave up waiting
    uint32_t groups = 1;      // batch groups in flight at once (launch_ring)
    RingBatch b[INGOT_RING_MAX_BATCHES];
};
static_assert(sizeof(RingArgs) <= 4096, "RingArgs exceeds the 4 KiB kernel-argument limit");

// Histogram pass over flow bins (flow.hip).
hipError_t launch_flow_hist(const uint32_t* flow, uint64_t n, uint32_t* hist, uint32_t bins,
                            void* work, size_t work_bytes, hipStream_t s);
size_t flow_hist_workspace(uint64_t n, uint32_t bins);

// Single-header parse (ingot_gpu_parse_header, header.hip).
struct HeaderArgs {
    const uint8_t* arena;
    const uint64_t* off;  // NULL: slots of `stride`
    const uint16_t* len;
    uint32_t stride;
    uint64_t n;
    int kind;              // enum ingot_header_kind
    const uint32_t* hints;  // per-slice choice hints, or NULL: `hint`
    uint32_t hint;
    ingot_hdr* out;
};
hipError_t launch_header(const HeaderArgs& a, hipStream_t s);

// Batched Emit (ingot_gpu_emit_packets / _headers, emit.hip).  api.cpp
// resolves each ingot_emit_set to the covering bytes of its field in the
// header block, so the kernel needs no tables.
struct EmitSet {
    uint16_t pos;      // first covering byte of the field in the header block
    uint16_t at;       // INGOT_EMIT_LENGTH counts the packet's bytes from here
    uint8_t nbytes, rshift, bits, source;
    int32_t add;
    const void* values;  // U16 / U32 sources: n per-packet values
};
struct EmitArgs {
    const uint8_t* src;      // NULL: header blocks only
    const uint64_t* off;     // source offsets (whole packets)
    const uint16_t* len;     // payload bytes per packet
    uint8_t* dst;
    const uint64_t* dst_off; // NULL: i * stride
    uint32_t stride;
    uint32_t hdr_len;
    uint64_t n;
    uint32_t n_sets;
    EmitSet sets[INGOT_MAX_EMIT_SETS];
    uint32_t hdr[INGOT_MAX_EMIT_HDR / 4];  // the header block, zero-padded
};
static_assert(sizeof(EmitArgs) <= 4096, "EmitArgs exceeds the 4 KiB kernel-argument limit");
// bytes of dynamic LDS one emit block needs (checked against the device)
size_t emit_lds_bytes(const EmitArgs& a);
hipError_t launch_emit(const EmitArgs& a, hipStream_t s);

// Lengths-only packed frames (packed.hip): tile base = u64 base of its group
// of PACKED_GROUP tiles (at the start of `work`, >= packed_workspace(n)
// bytes) + the tile's u32 prefix within the group (after the group bases).
constexpr uint32_t PACKED_GROUP = 128;
size_t packed_workspace(uint64_t n);
hipError_t launch_tile_bases(const uint16_t* len, uint64_t n, void* work, hipStream_t s);

// One wave that holds its stream for `ticks` of the device's constant-rate
// wall clock (ingot_gpu_stream_delay, stream.hip).
hipError_t launch_delay(uint64_t ticks, hipStream_t s);

// Per-context tuning (0 = measured default); see INGOT_TUNE_* in ingot_gpu.h.
struct Tuning {
    int window_indexed = 0;
    int window_strided = 0;
    uint32_t max_blocks = 0;
    int pipeline = 0;  // ring kernel: 0 = auto (2 blocks per CU), 1 = off, k = k tiles per wave
    int pipe_depth = 0;    // ring kernel: tiles in flight per wave (0 = 2)
    int writeback = 0;     // ring rewrite kernel: write-back unit (0 = measured default)
    int cache_policy = 0;  // bit 0: nt staging loads; bit 1: nt record stores
    int flow_table = 0;    // flows: 0 = auto (16-bit table when it suffices), 32 = 32-bit
    int slow_path = 0;     // bytes past the window: per-lane loads (0, the only value left)
    int read_plan = 0;     // parse_read: 0 / 11 line-completing chunk-0 window, 1 = 4 pieces,
                           // 17 = chunk bounds loaded lazily (parse_read_first)
    int flow_kernel = 0;   // flows: 0 / 15 = the measured default (k_flows_bits when it applies)
    int ring_grid = 0;     // ring consumer: blocks per CU (0 = measured default)
    int ring_groups = 0;   // ring consumer: batches in flight at once (0 = measured default)
    int xcd_remap = 0;     // slot ring: 1 = each XCD's blocks take a contiguous share of tiles
    uint32_t cus = 256;  // compute units of the context's device (grid shaping)
    bool host_arena = false;  // per call: the arena is host memory (ingot_gpu_host_map)
};

hipError_t launch_parse(const ParseArgs& a, int layout_kind, int chain, int mode,
                        const Tuning& t, hipStream_t s);
hipError_t launch_flows(const FlowArgs& a, int layout_kind, int chain, const Tuning& t,
                        hipStream_t s);
hipError_t launch_ring(const RingArgs& a, int chain, int mode, const Tuning& t, hipStream_t s);
// Flow classification over the plain parse's window with the table-free
// Toeplitz hash (tuple.hip, k_flows_bits): offset-addressed device frames,
// 16-bit bins, not the tunnel chain.
hipError_t launch_flows_tuple(const FlowArgs& a, int chain, const Tuning& t, hipStream_t s);
// launch_parse's branches in their own files: parse_read over chunk lists
// (read.hip; `a` with its cache policy set, `g` the one-tile-per-wave grid)
// and the slot-ring kernels (ring.hip).
hipError_t launch_segmented(const ParseArgs& a, int chain, int mode, const Tuning& t, uint32_t g,
                            hipStream_t s);
hipError_t launch_slot_ring(const ParseArgs& a, int chain, int mode, const Tuning& t,
                            hipStream_t s);
hipError_t launch_modify_ring(const ModifyArgs& a, int chain, const Tuning& t, hipStream_t s);
hipError_t launch_modify(const ModifyArgs& a, int layout_kind, int chain, const Tuning& t,
                         hipStream_t s);
bool tuning_valid(int key, int value);

}  // namespace ingot_gpu
