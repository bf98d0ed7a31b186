/*
 * ingot_gpu.h — C ABI of the MI355X (gfx950) batched L2/L3/L4 header extractor.
 *
 * This is the drop-in boundary for ingot's per-packet parse path.  In ingot the
 * path sits behind Rust traits, not an FFI:
 *
 *   HeaderParse::parse / parse_choice      ingot-types/src/lib.rs:137-147
 *   Success<T, B> = (T, Option<Denom>, B)   ingot-types/src/lib.rs:208
 *   <Chain>::parse_slice(from)              ingot-macros/src/parse.rs:496-509
 *   PacketParseError { label, inner }       ingot-types/src/error.rs:119-171
 *   ParseError (8 kinds)                    ingot-types/src/error.rs:21-44
 *
 * and it is called once per packet by the caller's loop
 * (ingot-examples/benches/packet.rs:136-172).  The entry points below replace
 * that loop + the parse bodies for a whole batch at once: the caller owns a
 * packet arena in device memory (borrow semantics: nothing is copied, nothing
 * is allocated per call) and gets one fixed-size record per packet that says
 * what `parse_slice` would have returned — Ok with the layer views as
 * (offset, kind) pairs and the remainder offset, or the PacketParseError
 * (failing layer index == label, ParseError discriminant).
 *
 * Plain C, plain pointers and sizes; `stream` is a hipStream_t passed as void*
 * (NULL = the null stream).  Every call is asynchronous on `stream`.  API
 * errors are negative ints (see ingot_gpu_strerror); per-packet parse errors
 * live in the records and are never API errors — like ingot, malformed input
 * never fails the call.
 *
 * Threading: a context is bound to one device; calls on distinct contexts or
 * distinct streams may run concurrently.  The context holds no per-call state.
 */
#ifndef INGOT_GPU_H
#define INGOT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: ingot_gpu_comm_wrap (borrow the host's RCCL communicator).
 * 2: ingot_gpu_comm_* / ingot_gpu_flow_hist_allreduce (config 5's reduce);
 *    host mappings counted per map, ingot_gpu_host_unmap EINVAL for a pointer
 *    the context never mapped (1: any pointer, hipHostUnregister'd). */
#define INGOT_GPU_ABI_VERSION 3

/* ---------------------------------------------------------------------------
 * Per-packet status: 0 = Ok, else 1 + the ParseError discriminant in the
 * declaration order of ingot-types/src/error.rs:22-44.  Reachable: UNWANTED
 * and TOO_SMALL, STRADDLED_HEADER under ingot_gpu_parse_read;
 * the others are listed so the numbering is ingot's.
 * ------------------------------------------------------------------------- */
enum ingot_status {
    INGOT_OK = 0,
    INGOT_ERR_UNWANTED = 1,
    INGOT_ERR_NEEDS_HINT = 2,
    INGOT_ERR_TOO_SMALL = 3,
    INGOT_ERR_STRADDLED_HEADER = 4,
    INGOT_ERR_NO_REMAINING_CHUNKS = 5,
    INGOT_ERR_CANNOT_ACCEPT = 6,
    INGOT_ERR_REJECT = 7,
    INGOT_ERR_ILLEGAL_VALUE = 8
};

/* ---------------------------------------------------------------------------
 * Parse chains (the `#[derive(Parse)]` structs the batch is parsed as).
 *
 * UDP_PARSER   ingot-examples/src/packets.rs:18-24
 *              eth: Ethernet, l3: L3 (v4|v6), l4: from L4 (tcp|udp) -> Udp
 *              layer labels "eth", "l3", "l4"
 * GENERIC_ULP  ingot-examples/src/packets.rs:54-60  (control = exit_on_arp)
 *              inner_eth: Ethernet, inner_l3: Option<L3>, inner_ulp: Option<Ulp>
 *              layer labels "inner_eth", "inner_l3", "inner_ulp"
 * VLAN_ULP     build-defined (ingot declares VlanBody, ethernet.rs:57-65, but
 *              no chain uses it): eth, 0..2 x VlanBody while the ethertype is
 *              0x8100/0x9100, L3, Ulp; no control.  Labels "eth", "vlan",
 *              "l3", "l4".  Parity for this chain is unpinned by the reference.
 * GENEVE_OVER_V6  ingot-examples/src/packets.rs:27-40 (OPTE's inbound path)
 *              outer_eth: Ethernet, outer_v6: from L3 -> Ipv6 (+EHs),
 *              outer_udp: from L4 -> Udp, outer_encap: Geneve (+options,
 *              geneve.rs:16-44), then GenericUlp's three layers (control =
 *              exit_on_arp on inner_eth).  Labels "outer_eth", "outer_v6",
 *              "outer_udp", "outer_encap", "inner_eth", "inner_l3", "inner_ulp".
 * ------------------------------------------------------------------------- */
enum ingot_chain {
    INGOT_CHAIN_UDP_PARSER = 0,
    INGOT_CHAIN_GENERIC_ULP = 1,
    INGOT_CHAIN_VLAN_ULP = 2,
    INGOT_CHAIN_GENEVE_OVER_V6 = 3,
    INGOT_CHAIN_COUNT = 4
};

enum ingot_l3_kind { INGOT_L3_NONE = 0, INGOT_L3_IPV4 = 1, INGOT_L3_IPV6 = 2 };
enum ingot_l4_kind {
    INGOT_L4_NONE = 0,
    INGOT_L4_TCP = 1,
    INGOT_L4_UDP = 2,
    INGOT_L4_ICMPV4 = 3,
    INGOT_L4_ICMPV6 = 4
};

/* rec.flags */
#define INGOT_REC_ACCEPTED 0x01u /* a parse control accepted early (parse.rs:221-254) */
#define INGOT_REC_INNER 0x02u    /* tunnel chain: the walk reached inner_eth */

/* ---------------------------------------------------------------------------
 * ingot_rec — the 16-byte per-packet result.
 *
 * Fields are filled as the chain walks, so an error record still shows how
 * far the walk got:
 *   status/err_layer  Ok, or (1+ParseError, index of the failing layer label)
 *                     err_layer = 0xff when Ok.
 *   l3_kind/l4_kind   set when the L3 / L4 choice selects a variant (before
 *                     that variant is parsed).
 *   l3_off/l4_off     frame offset where the L3 / L4 layer starts (0 = never
 *                     reached).
 *   payload_off       offset of the remainder: bytes consumed by the headers
 *                     that parsed successfully (== remainder start on Ok).
 *   ethertype         the Ethertype hint handed to the L3 choice (after VLAN
 *                     tags); 0 if Ethernet did not parse.
 *   l4_proto          the IpProtocol hint handed to the L4 choice (IPv6: the
 *                     last extension header's next_header, ip.rs:180-181,
 *                     util.rs:189-228).
 *   n_vlan/n_v6ext    VLAN tags / IPv6 extension headers fully parsed.
 *
 * GENEVE_OVER_V6: the fields describe the innermost layers reached.  While
 * the walk is in the outer layers they describe outer_v6 / outer_udp; once
 * inner_eth parses, flags |= INGOT_REC_INNER and l3/l4 kind, offsets,
 * n_v6ext, l4_proto restart for the inner frame (ethertype = the inner one).
 * The inner frame then starts at l3_off - 14 (inner L3 reached) or
 * payload_off - 14 (walk ended at inner_eth); ingot_gpu_geneve_fields gives
 * every outer offset and getter.
 * ------------------------------------------------------------------------- */
typedef struct ingot_rec {
    uint8_t status;
    uint8_t err_layer;
    uint8_t l3_kind;
    uint8_t l4_kind;
    uint8_t n_vlan;
    uint8_t n_v6ext;
    uint8_t l4_proto;
    uint8_t flags;
    uint16_t l3_off;
    uint16_t l4_off;
    uint16_t payload_off;
    uint16_t ethertype;
} ingot_rec;

/* ---------------------------------------------------------------------------
 * ingot_rec8 — the same result in 8 bytes (for record-bandwidth-bound
 * callers).  Everything a caller needs to rebuild the layer views is kept;
 * the dropped rec16 fields are derivable from it and the frame:
 *   l3_off    = 14 + 4*n_vlan            (when l3_kind != NONE)
 *   ethertype = be16(frame, 12 + 4*n_vlan)
 *   err_layer = 0xff when status == Ok
 *
 *   b0: status (bits 0-3) | err_layer (bits 4-5, 0 when Ok) | l3_kind (bits 6-7)
 *   b1: l4_kind (bits 0-2) | n_vlan (bits 3-4) | accepted (bit 5)
 * ------------------------------------------------------------------------- */
typedef struct ingot_rec8 {
    uint8_t status_layer_l3;
    uint8_t l4_vlan_flags;
    uint8_t n_v6ext;
    uint8_t l4_proto;
    uint16_t l4_off;
    uint16_t payload_off;
} ingot_rec8;

/* One IPv6 extension header as ingot's getters see it
 * (IpV6ExtFragment ip.rs:190-200, IpV6Ext6564 ip.rs:202-211). */
#define INGOT_EH_FRAGMENT 1
#define INGOT_EH_RFC6564 2
#define INGOT_MAX_EH_FIELDS 4 /* first 4 EHs are materialised; count is exact */

typedef struct ingot_v6eh {
    uint32_t ident;         /* fragment: ident (u32be) */
    uint16_t frag_offset;   /* fragment: fragment_offset (u13be) */
    uint16_t off;           /* frame offset of this EH */
    uint8_t kind;           /* INGOT_EH_FRAGMENT / INGOT_EH_RFC6564 */
    uint8_t next_header;    /* both */
    uint8_t ext_len;        /* 6564: ext_len; fragment: reserved */
    uint8_t frag_res_more;  /* fragment: res << 1 | more_frags */
} ingot_v6eh;

/* ---------------------------------------------------------------------------
 * ingot_fields — every getter of every header on the chain, materialised
 * (parity mode).  Values are exactly what ingot's generated XRef getters
 * return (bitfield.rs:40-315 BE bit order; NetworkRepr conversions applied:
 * `*_ecn` is Ecn::from_network (3 -> Capable0 == 1, ip.rs:111-119), flags are
 * bitflags from_bits_truncate (identity on the stored bits)).  Variable-length
 * fields (options, EH data) are given as (offset, length) into the frame.
 * Headers that were not reached are all-zero.
 * ------------------------------------------------------------------------- */
typedef struct ingot_fields {
    ingot_rec rec;                      /*   0 */
    /* 32-bit */
    uint32_t v6_flow_label;             /*  16 */
    uint32_t tcp_sequence;              /*  20 */
    uint32_t tcp_acknowledgement;       /*  24 */
    /* 16-bit */
    uint16_t eth_ethertype;             /*  28 */
    uint16_t vlan_vid[2];               /*  30 */
    uint16_t vlan_ethertype[2];         /*  34 */
    uint16_t v4_total_len;              /*  38 */
    uint16_t v4_identification;         /*  40 */
    uint16_t v4_fragment_offset;        /*  42 */
    uint16_t v4_checksum;               /*  44 */
    uint16_t v4_options_off;            /*  46 */
    uint16_t v4_options_len;            /*  48 */
    uint16_t v6_payload_len;            /*  50 */
    uint16_t v6_ext_off;                /*  52  RepeatedView span start */
    uint16_t v6_ext_len;                /*  54  RepeatedView span bytes */
    uint16_t l4_source;                 /*  56  tcp/udp source */
    uint16_t l4_destination;            /*  58  tcp/udp destination */
    uint16_t tcp_window_size;           /*  60 */
    uint16_t tcp_checksum;              /*  62 */
    uint16_t tcp_urgent_ptr;            /*  64 */
    uint16_t tcp_options_off;           /*  66 */
    uint16_t tcp_options_len;           /*  68 */
    uint16_t udp_length;                /*  70 */
    uint16_t udp_checksum;              /*  72 */
    uint16_t icmp_checksum;             /*  74 */
    /* 8-bit */
    uint8_t eth_destination[6];         /*  76 */
    uint8_t eth_source[6];              /*  82 */
    uint8_t vlan_priority[2];           /*  88 */
    uint8_t vlan_dei[2];                /*  90 */
    uint8_t v4_version;                 /*  92 */
    uint8_t v4_ihl;                     /*  93 */
    uint8_t v4_dscp;                    /*  94 */
    uint8_t v4_ecn_raw;                 /*  95 */
    uint8_t v4_ecn;                     /*  96 */
    uint8_t v4_flags;                   /*  97 */
    uint8_t v4_hop_limit;               /*  98 */
    uint8_t v4_protocol;                /*  99 */
    uint8_t v4_source[4];               /* 100 */
    uint8_t v4_destination[4];          /* 104 */
    uint8_t v6_version;                 /* 108 */
    uint8_t v6_dscp;                    /* 109 */
    uint8_t v6_ecn_raw;                 /* 110 */
    uint8_t v6_ecn;                     /* 111 */
    uint8_t v6_next_header;             /* 112 */
    uint8_t v6_hop_limit;               /* 113 */
    uint8_t v6_source[16];              /* 114 */
    uint8_t v6_destination[16];         /* 130 */
    uint8_t tcp_data_offset;            /* 146 */
    uint8_t tcp_reserved;               /* 147 */
    uint8_t tcp_flags;                  /* 148 */
    uint8_t icmp_ty;                    /* 149 */
    uint8_t icmp_code;                  /* 150 */
    uint8_t icmp_rest_of_hdr[4];        /* 151 */
    uint8_t _pad0;                      /* 155 */
    ingot_v6eh v6_eh[INGOT_MAX_EH_FIELDS]; /* 156 (4 x 12) */
    uint8_t _pad1[52];                  /* 204 -> 256 */
} ingot_fields;

/* ---------------------------------------------------------------------------
 * GENEVE_OVER_V6 parity mode: the outer layers' getters (128 B) after the
 * inner frame's ingot_fields (whose eth_* / v4_* / v6_* / l4 fields are
 * inner_eth / inner_l3 / inner_ulp).  Geneve getters follow geneve.rs:16-44:
 * version u2, opt_len u6, flags = GeneveFlags::from_bits_truncate (bits 0xC0
 * kept), protocol_type u16be, vni [u8;3] as a 24-bit BE integer, reserved
 * u8.  Options (Repeated<GeneveOpt>, geneve.rs:80-102) are listed in order;
 * the first INGOT_MAX_GENEVE_OPT_FIELDS are materialised, the count is exact.
 * ------------------------------------------------------------------------- */
#define INGOT_MAX_GENEVE_OPT_FIELDS 4

typedef struct ingot_geneve_opt {
    uint16_t opt_class;     /* class (u16be) */
    uint16_t data_off;      /* frame offset of data (length*4 bytes) */
    uint8_t option_type;    /* GeneveOptionType (is_critical = bit 7) */
    uint8_t reserved;       /* u3 */
    uint8_t length;         /* u5, in 4-byte words */
    uint8_t _pad;
} ingot_geneve_opt;

typedef struct ingot_tunnel_fields {
    uint8_t outer_eth_destination[6];   /*   0 */
    uint8_t outer_eth_source[6];        /*   6 */
    uint16_t outer_eth_ethertype;       /*  12 */
    uint16_t outer_udp_off;             /*  14  frame offset of outer_udp */
    uint8_t outer_v6_source[16];        /*  16 */
    uint8_t outer_v6_destination[16];   /*  32 */
    uint32_t outer_v6_flow_label;       /*  48 */
    uint16_t outer_v6_payload_len;      /*  52 */
    uint16_t outer_v6_ext_len;          /*  54  EH span bytes (from offset 54) */
    uint8_t outer_v6_version;           /*  56 */
    uint8_t outer_v6_dscp;              /*  57 */
    uint8_t outer_v6_ecn_raw;           /*  58 */
    uint8_t outer_v6_ecn;               /*  59 */
    uint8_t outer_v6_next_header;       /*  60 */
    uint8_t outer_v6_hop_limit;         /*  61 */
    uint8_t outer_v6_n_ext;             /*  62 */
    uint8_t outer_l4_proto;             /*  63  hint handed to the outer L4 choice */
    uint16_t outer_udp_source;          /*  64 */
    uint16_t outer_udp_destination;     /*  66 */
    uint16_t outer_udp_length;          /*  68 */
    uint16_t outer_udp_checksum;        /*  70 */
    uint16_t geneve_off;                /*  72 */
    uint16_t inner_eth_off;             /*  74 */
    uint32_t geneve_vni;                /*  76 */
    uint16_t geneve_protocol_type;      /*  80 */
    uint8_t geneve_version;             /*  82 */
    uint8_t geneve_opt_len;             /*  83 */
    uint8_t geneve_flags;               /*  84 */
    uint8_t geneve_reserved;            /*  85 */
    uint8_t geneve_n_opts;              /*  86  (saturates at 255) */
    uint8_t geneve_critical;            /*  87  any option_type.is_critical() */
    ingot_geneve_opt geneve_opt[INGOT_MAX_GENEVE_OPT_FIELDS]; /* 88 (4 x 8) */
    uint8_t _pad[8];                    /* 120 -> 128 */
} ingot_tunnel_fields;

typedef struct ingot_geneve_fields {
    ingot_fields inner;                 /*   0  rec + inner layers */
    ingot_tunnel_fields outer;          /* 256 */
} ingot_geneve_fields;

#ifdef __cplusplus
static_assert(sizeof(ingot_rec) == 16, "ingot_rec is 16 bytes");
static_assert(sizeof(ingot_rec8) == 8, "ingot_rec8 is 8 bytes");
static_assert(sizeof(ingot_v6eh) == 12, "ingot_v6eh is 12 bytes");
static_assert(sizeof(ingot_fields) == 256, "ingot_fields is 256 bytes");
static_assert(sizeof(ingot_geneve_opt) == 8, "ingot_geneve_opt is 8 bytes");
static_assert(sizeof(ingot_tunnel_fields) == 128, "ingot_tunnel_fields is 128 bytes");
static_assert(sizeof(ingot_geneve_fields) == 384, "ingot_geneve_fields is 384 bytes");
#endif

/* API return codes (negative). */
#define INGOT_GPU_SUCCESS 0
#define INGOT_GPU_EINVAL (-1)   /* bad argument (null pointer, bad chain ...) */
#define INGOT_GPU_EHIP (-2)     /* a HIP runtime call failed */
#define INGOT_GPU_ENOMEM (-3)   /* context allocation failed */
#define INGOT_GPU_ENODEV (-4)   /* no such device / no gfx950 code object */
#define INGOT_GPU_ERANGE (-5)   /* size outside what the ABI supports */

typedef struct ingot_gpu_ctx ingot_gpu_ctx;

/* Library / ABI identification. */
int ingot_gpu_abi_version(void);
const char* ingot_gpu_build_info(void);

/* Context: binds a device.  Cheap; owns no per-call buffers. */
int ingot_gpu_ctx_create(int device, ingot_gpu_ctx** out);
void ingot_gpu_ctx_destroy(ingot_gpu_ctx* ctx);
int ingot_gpu_ctx_device(const ingot_gpu_ctx* ctx);

/*
 * Zero-copy host rings.  The path often starts and ends in host memory (a NIC
 * or loopback ring).  ingot_gpu_host_map makes host memory [host, host+bytes)
 * device-addressable — memory already pinned by hipHostMalloc is used as it
 * is, pageable memory is page-locked and mapped (hipHostRegister, mapped) —
 * and returns the device address of `host` in *d_ptr.  That address may be
 * passed as any device pointer of the calls below (d_arena, descriptors,
 * d_out ...): the kernels then read only the header bytes they touch across
 * PCIe (LDS-DMA staging from host memory) instead of a whole-frame
 * hipMemcpy, and can write records straight into host memory.  Results are
 * identical to a device-resident arena.
 *
 * Mappings are counted.  Every successful ingot_gpu_host_map is paired with
 * one ingot_gpu_host_unmap(ctx, host) by the same context and the same
 * `host` (INGOT_GPU_EINVAL if this context holds no mapping starting there).
 * The library unregisters only what it registered itself: pageable ranges it
 * page-locked, once the last mapping inside them is unmapped (by any context)
 * or its context is destroyed.  Memory pinned by someone else (hipHostMalloc,
 * the caller's own hipHostRegister) is never unregistered: unmapping it only
 * forgets the mapping.  A range inside one registered by an earlier map
 * shares that registration (e.g. a record buffer carved out of a mapped
 * ring); a range that partly overlaps one is refused (INGOT_GPU_EINVAL).
 * Two buffers whose bytes are disjoint but share a page are registered
 * separately and may be mapped at the same time.  The caller keeps the bytes
 * stable while a call that reads them runs, unmaps only after the calls that
 * use a mapping have completed, and frees (or munmaps) pageable memory only
 * after unmapping it: a registration whose pages were freed leaves a stale
 * device mapping behind.
 */
int ingot_gpu_host_map(ingot_gpu_ctx* ctx, void* host, size_t bytes, void** d_ptr);
int ingot_gpu_host_unmap(ingot_gpu_ctx* ctx, void* host);

/*
 * Doorbells.  A ring consumer that knows its next batches in advance (a NIC
 * or loopback ring: slot k of the ring is batch k) can enqueue their parse
 * launches before the frames arrive, each behind a doorbell wait; the
 * producer publishes batch k by writing k (or more) into the doorbell from
 * the host, and the GPU starts the queued launch with no host round trip
 * (no launch latency on the critical path).  The doorbell is one 32-bit word
 * of pinned host memory polled by the GPU's command processor
 * (hipStreamWaitValue32, compare >=).  *host_word may be written directly by
 * the producer (e.g. another thread) or through ingot_gpu_doorbell_ring.
 *   ingot_gpu_doorbell_wait: everything enqueued on `stream` after this call
 *     runs only once *doorbell >= value.  The caller must make sure the
 *     doorbell is eventually rung: a stream left waiting never drains.
 *   ingot_gpu_doorbell_destroy: only after every wait on it has been passed.
 * ENODEV when the device cannot wait on memory values.
 *
 * A doorbell wait holds a whole HARDWARE queue, not just its stream: HIP
 * maps streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by
 * default), and the command processor stops at the wait packet, so every
 * other stream mapped to that queue (a producer's copy stream, RCCL's
 * stream, torch's current stream) stalls behind it until the ring.  A
 * producer must therefore publish frames from the host, or from a stream
 * known to sit on another hardware queue; publishing with GPU work that
 * shares the held queue and ringing only after that work completes
 * deadlocks (tests/test_doorbell.py::test_held_queue_blocks_its_streams).
 * ingot_gpu_parse_ring's in-kernel doorbell has no such constraint.
 */
typedef struct ingot_gpu_doorbell ingot_gpu_doorbell;
int ingot_gpu_doorbell_create(ingot_gpu_ctx* ctx, ingot_gpu_doorbell** out,
                              volatile uint32_t** host_word);
int ingot_gpu_doorbell_wait(ingot_gpu_doorbell* db, uint32_t value, void* stream);
int ingot_gpu_doorbell_ring(ingot_gpu_doorbell* db, uint32_t value);
void ingot_gpu_doorbell_destroy(ingot_gpu_doorbell* db);

/*
 * Persistent ring consumer.  One launch parses `nbatches` (<=
 * INGOT_RING_MAX_BATCHES) batches of `n` frames in fixed slots of `stride`
 * bytes (>= 64, a multiple of 16; no length array, like
 * ingot_gpu_parse_strided with d_len NULL): batch b from batches[b].d_arena
 * into batches[b].d_out (n ingot_rec when record_bytes is 16, n ingot_rec8
 * when 8; not GENEVE_OVER_V6).  The records are exactly those of
 * ingot_gpu_parse_strided over each batch.  Instead of one launch per batch
 * (each paying a grid ramp-up and drain), every wave walks its share of all
 * the batches' tiles in order, keeping the next tile's LDS-DMA in flight
 * across batch boundaries.
 *
 *   db == NULL: every batch is resident when the launch starts.
 *   db != NULL: a wave stages tiles of batch b only once the doorbell word
 *     is >= db_first + b (the producer rings db_first + b after batch b's
 *     frames are in memory; rings may cover several batches at once).  The
 *     wave polls the word (one lane, with sleeps) only when it reaches a batch
 *     not yet known published, then invalidates its caches (system-scope
 *     acquire), so frames written by the host, a copy engine or another
 *     kernel after the launch started are seen.  A wave that waits more than
 *     `timeout_ms` (1..60000) for a batch stops, and *d_status (optional,
 *     device memory, caller-zeroed) gets bit 0 set.  Waves give up one by
 *     one: a wave that reaches the ring later may still see a batch published
 *     and parse its tiles.  So when bit 0 is set, the record buffers of
 *     EVERY batch from the first one not published at launch onward are
 *     undefined (some tiles written, some not); batches published before the
 *     launch are complete.  Every launch ends, rung or not.  Doorbell values
 *     must increase monotonically across ring launches, the last batch's
 *     value db_first + nbatches - 1 must fit in 32 bits (else
 *     INGOT_GPU_ERANGE), and `db` must belong to
 *     ctx's device (else INGOT_GPU_EINVAL).
 * The arenas are read-only for the launch; a batch buffer must not be
 * rewritten while the launch may still read it (a ring reuses a slot only
 * after the launch that consumes it has completed).  Unlike a
 * doorbell_wait, the polling kernel holds no hardware queue: other streams
 * (a producer's copies included) keep running beside it.
 */
#define INGOT_RING_MAX_BATCHES 64
typedef struct ingot_ring_batch {
    const uint8_t* d_arena; /* n slots of `stride` bytes, 16-B aligned */
    void* d_out;            /* n records */
} ingot_ring_batch;
int ingot_gpu_parse_ring(ingot_gpu_ctx* ctx, const ingot_ring_batch* batches,
                         uint32_t nbatches, uint32_t stride, uint64_t n, int chain,
                         uint32_t record_bytes, const ingot_gpu_doorbell* db,
                         uint32_t db_first, uint32_t timeout_ms, uint32_t* d_status,
                         void* stream);

/*
 * Staggered streams.  A consumer that alternates its batches over two (or
 * more) streams keeps one launch ramping up while another drains; started
 * together, the streams' launches ramp and drain in lockstep and that
 * overlap is lost until they drift apart.  ingot_gpu_stream_delay enqueues
 * on `stream` a one-wave wait of `ns` nanoseconds of the device's wall clock
 * (everything enqueued after it starts that much later); enqueued right after
 * a doorbell wait, it starts a second stream behind the first.
 * ENODEV when the device reports no wall-clock rate.
 */
int ingot_gpu_stream_delay(ingot_gpu_ctx* ctx, uint32_t ns, void* stream);

/*
 * Tuning knobs (results never depend on them).  Defaults are the measured
 * best on MI355X; value 0 restores the default.
 *   INGOT_TUNE_WINDOW_INDEXED  16-B chunks staged in LDS per packed frame:
 *                              2,3,4,5,6,8,9, or 100 = no staging; 20 + k:
 *                              record / flow modes, a window from byte 12's
 *                              chunk to the end of the 128-B line its second
 *                              chunk lies in, at most k chunks (packed
 *                              frames: k = 2, 3, 5 or 8); 1000 + 10 m + k:
 *                              the same from at least m chunks.  Defaults:
 *                              records 25 (the tunnel chain 1069; packed
 *                              tunnel frames 8), fields / rewrites 3 (tunnel
 *                              8), mapped host memory 5.  Flows: offset-
 *                              addressed device frames with 16-bit bins use
 *                              k_flows_bits over a 4-to-5-chunk window; any
 *                              explicit value here turns that kernel off and
 *                              runs the k_parse flows mode with the value
 *                              (its own default, for the full 32-bit hash,
 *                              the tunnel chain and host memory: 1056)
 *   INGOT_TUNE_WINDOW_STRIDED  16-B chunks staged per slot: 2,3,4,5,8 or 100
 *                              (default 4 for slots <= 64 B, else 3)
 *   INGOT_TUNE_MAX_BLOCKS      grid cap in 256-thread blocks (0 = one
 *                              64-packet tile per wave)
 *   INGOT_TUNE_PIPELINE        strided rings (slots >= 64 B) without a length
 *                              array, 16- or 8-B records: the multi-tile kernel
 *                              that stages the next tile while parsing one
 *                              (double-buffered LDS).  0 = on, 2 blocks per CU
 *                              (default); 1 = off; k >= 2 = k tiles per wave
 *   INGOT_TUNE_CACHE_POLICY    0 = measured default (non-temporal record
 *                              stores; the ring kernel: non-temporal staging
 *                              loads and, for 16-B records, device-scope
 *                              record stores); else bit 0: stage frame
 *                              bytes with non-temporal loads, bit 1:
 *                              non-temporal record stores (4 = neither);
 *                              bits 3-5, when non-zero, set the record
 *                              stores' cache bits instead of bit 1: 1 sc1,
 *                              2 sc1 nt, 3 sc0 sc1, 4 sc0 sc1 nt, 5 sc0;
 *                              bits 6-8, when non-zero, the staging loads'
 *                              instead of bit 0 (same codes, 6 sc0 nt)
 *   INGOT_TUNE_PIPE_DEPTH      the multi-tile ring kernel's tiles in flight
 *                              per wave (LDS images): 2 (default), 3 or 4
 *                              (the rewrite ring kernel: 2 or 3)
 *   INGOT_TUNE_WRITEBACK       ingot_gpu_parse_modify on slot rings: bytes
 *                              written back per edited unit, 16, 32 or 64
 *                              (0 = measured default)
 *   INGOT_TUNE_FLOW_TABLE      ingot_gpu_flow_hist's Toeplitz lookup table:
 *                              0 / 16 = 16-bit entries when bins <= 65,536
 *                              and no full hash is requested (default), 32 =
 *                              always 32-bit entries (same flow bins)
 *   INGOT_TUNE_SLOW_PATH       bytes past the staged window: 0 = read per
 *                              lane from L2/HBM (the only value; the
 *                              compacted re-stage and resume-style variants
 *                              lost and were removed: EINVAL)
 *   INGOT_TUNE_READ_PLAN       ingot_gpu_parse_read / _read_first (16-B
 *                              records): 0 / 11 = chunk 0 staged in a
 *                              line-completing window of 3 to 5 16-B pieces
 *                              (to the end of the 128-B line its third piece
 *                              lies in; default); 1 = 4 pieces (the default
 *                              for chunk pools in mapped host memory,
 *                              ingot_gpu_host_map); 17 = the default window
 *                              with the chunk bounds loaded lazily, per lane,
 *                              only by a walk that leaves chunk 0 or fails
 *                              in it (ingot_gpu_parse_read_first only: one
 *                              descriptor stream for header-split packets;
 *                              elsewhere it means 0).  Field blocks stage 4
 *                              pieces, and ingot_gpu_parse_read_dense always
 *                              stages 4 pieces (the knob is ignored there).
 *                              Other values: EINVAL
 *   INGOT_TUNE_FLOW_KERNEL     ingot_gpu_flow_hist: 0 / 15 = the measured
 *                              default (the only values; EINVAL otherwise):
 *                              offset-addressed device frames with bins <=
 *                              65,536, no full hash, no explicit window and
 *                              not the tunnel chain run k_flows_bits (the
 *                              plain parse's 4-to-5-chunk window, the
 *                              Toeplitz hash bit by bit from the key windows,
 *                              no LDS table); everything else runs k_parse's
 *                              flows mode (LDS table: 16-bit entries one tile
 *                              per wave, 32-bit entries on a persistent grid)
 *   INGOT_TUNE_RING_GRID       ingot_gpu_parse_ring: 256-thread blocks per
 *                              CU (1..8; 0 = measured default).  The ring's
 *                              tiles in flight per wave follow
 *                              INGOT_TUNE_PIPE_DEPTH
 *   INGOT_TUNE_XCD_REMAP       slot-ring kernels (parse, rewrite) tile order:
 *                              0 = measured default (= 1); 1 = blocks
 *                              renumbered XCD-major (block b runs on XCD b % 8;
 *                              logical block (b % 8) * G/8 + b / 8), so each
 *                              XCD walks a contiguous eighth of every round of
 *                              tiles; 2 = each wave walks a contiguous run of
 *                              tiles instead of striding by the grid; 3 = both;
 *                              4 = hardware order, grid stride; 5 = the batch
 *                              in 8 contiguous regions, one per XCD (parse ring
 *                              only; the rewrite ring takes 0/1/4)
 *   INGOT_TUNE_RING_GROUPS     ingot_gpu_parse_ring: batches in flight at
 *                              once (1, 2 or 4; 0 = measured default): the
 *                              grid is cut into that many block groups, group
 *                              q consuming batches q, q+G, ...
 */
#define INGOT_TUNE_WINDOW_INDEXED 1
#define INGOT_TUNE_WINDOW_STRIDED 2
#define INGOT_TUNE_MAX_BLOCKS 3
#define INGOT_TUNE_PIPELINE 4
#define INGOT_TUNE_CACHE_POLICY 5
#define INGOT_TUNE_PIPE_DEPTH 6
#define INGOT_TUNE_WRITEBACK 7
#define INGOT_TUNE_FLOW_TABLE 8
#define INGOT_TUNE_SLOW_PATH 9
#define INGOT_TUNE_READ_PLAN 10
#define INGOT_TUNE_FLOW_KERNEL 11
#define INGOT_TUNE_RING_GRID 12
#define INGOT_TUNE_RING_GROUPS 13
#define INGOT_TUNE_XCD_REMAP 14
int ingot_gpu_ctx_set_tuning(ingot_gpu_ctx* ctx, int key, int value);
int ingot_gpu_ctx_get_tuning(const ingot_gpu_ctx* ctx, int key);

/*
 * Batched `<Chain>::parse_slice` over frames in a device arena.
 *
 *   d_arena   device pointer to the packet bytes, any alignment (the
 *             kernels align the absolute addresses they stage; they may read
 *             up to 15 bytes before d_arena + d_off[i] and after a frame's
 *             end, never outside that frame's 16-byte blocks)
 *   d_off     per-packet byte offset into d_arena (u64)
 *   d_len     per-packet length in bytes (u16); the caller guarantees every
 *             [d_off[i], d_off[i] + d_len[i]) lies inside its allocation
 *             (ingot's borrowed-slice contract: the kernels read no byte of
 *             a frame past d_len[i] except within its last 16-byte block)
 *   n         number of packets
 *   chain     enum ingot_chain
 *   d_out     n records (device memory, 16 B each)
 *
 * Replaces the caller's per-packet loop over `parse_slice`
 * (ingot-examples/benches/packet.rs:136-172) for the whole batch.
 */
int ingot_gpu_parse(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                    const uint64_t* d_off, const uint16_t* d_len, uint64_t n,
                    int chain, ingot_rec* d_out, void* stream);

/*
 * Same, for fixed-stride arenas (ring buffers with one frame per slot):
 * frame i starts at d_arena + i*stride; its length is d_len[i], or `stride`
 * when d_len is NULL.  stride must be a multiple of 16 and <= 65535 and
 * d_arena 16-byte aligned.  No descriptor bytes are read when d_len is NULL.
 */
int ingot_gpu_parse_strided(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                            uint32_t stride, const uint16_t* d_len, uint64_t n,
                            int chain, ingot_rec* d_out, void* stream);

/* The two batch calls above with 8-byte ingot_rec8 records.  Not for
 * GENEVE_OVER_V6 (EINVAL): the inner offsets do not fit its derivation rules. */
int ingot_gpu_parse_compact(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                            const uint64_t* d_off, const uint16_t* d_len,
                            uint64_t n, int chain, ingot_rec8* d_out,
                            void* stream);
int ingot_gpu_parse_strided_compact(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                                    uint32_t stride, const uint16_t* d_len,
                                    uint64_t n, int chain, ingot_rec8* d_out,
                                    void* stream);

/*
 * Parity mode: every getter of every parsed header (ingot_fields, 256 B per
 * packet).  Same inputs as ingot_gpu_parse; d_off may be NULL to select the
 * strided layout with `stride` (ignored otherwise).
 */
int ingot_gpu_fields(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                     const uint64_t* d_off, const uint16_t* d_len,
                     uint32_t stride, uint64_t n, int chain,
                     ingot_fields* d_out, void* stream);
/* (chain GENEVE_OVER_V6 is EINVAL here: use ingot_gpu_geneve_fields.) */

/*
 * Parity mode for GeneveOverV6Tunnel (384 B per packet): the inner frame's
 * ingot_fields + the outer layers' ingot_tunnel_fields.  Same inputs as
 * ingot_gpu_fields, chain implied.
 */
int ingot_gpu_geneve_fields(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                            const uint64_t* d_off, const uint16_t* d_len,
                            uint32_t stride, uint64_t n,
                            ingot_geneve_fields* d_out, void* stream);

/*
 * Batched `<Chain>::parse_read` (ingot-macros/src/parse.rs:511-537) over
 * multi-chunk packets (mblk_t-style chains) — the `Read` input of
 * ingot-types/src/lib.rs:151-166 as a chunk list:
 *   d_seg_off / d_seg_len  every chunk's device offset into d_arena and length;
 *   d_pkt_seg              n+1 u32 bounds: packet i is chunks
 *                          [d_pkt_seg[i], d_pkt_seg[i+1]) in order.
 * Semantics are parse_read's: a header must lie inside one chunk; a layer
 * that ends its chunk makes the next chunk the slice (none left: TooSmall at
 * that layer, even if the rest was accepted); a header cut by its chunk's end
 * is StraddledHeader when another chunk follows, else TooSmall
 * (error.rs:65-72); no chunks at all is TooSmall at the first label.
 * Record offsets are logical (into the chunks concatenated; a packet's
 * chunks should total <= 65535 B: later bytes are not seen).  d_chunk
 * (optional, n x u16) = index within the packet of the chunk holding the
 * remainder: Parsed::last_chunk is that chunk from payload_off (None when
 * empty), Parsed::data the chunks after it.  No 8-B records or flow mode.
 */
int ingot_gpu_parse_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                         const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                         const uint32_t* d_pkt_seg, uint64_t n, int chain,
                         ingot_rec* d_out, uint16_t* d_chunk, void* stream);
/* Parity mode of the same (GENEVE_OVER_V6: EINVAL, use the geneve form). */
int ingot_gpu_fields_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                          const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                          const uint32_t* d_pkt_seg, uint64_t n, int chain,
                          ingot_fields* d_out, uint16_t* d_chunk, void* stream);
int ingot_gpu_geneve_fields_read(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                                 const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                                 const uint32_t* d_pkt_seg, uint64_t n,
                                 ingot_geneve_fields* d_out, uint16_t* d_chunk,
                                 void* stream);
/*
 * ingot_gpu_parse_read with a dense chunk table: one 8-byte entry per chunk,
 * d_seg[k] = (offset << 16) | length (offset < 2^48), instead of the u64 and
 * u16 arrays — one load per chunk descriptor and no padding between them.
 * fields = 0: d_out holds ingot_rec records; 1: ingot_fields blocks (EINVAL
 * for GENEVE_OVER_V6); 2: ingot_geneve_fields blocks (GENEVE_OVER_V6 only).
 * Staging: chunk 0 in a fixed 4-piece (64-B) window, whatever
 * INGOT_TUNE_READ_PLAN says.
 */
int ingot_gpu_parse_read_dense(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                               const uint64_t* d_seg, const uint32_t* d_pkt_seg,
                               uint64_t n, int chain, int fields, void* d_out,
                               uint16_t* d_chunk, void* stream);

/*
 * ingot_gpu_parse_read with chunk 0 of every packet also given per packet:
 * d_first[i] = (seg_off[pkt_seg[i]] << 16) | seg_len[pkt_seg[i]] (0 for a
 * packet without chunks; offsets < 2^48).  An mblk chain's packet pointer is
 * its first chunk, so a ring of packets naturally carries this; the kernel
 * then loads chunk 0's descriptor beside the packet's chunk bounds instead of
 * after them (one HBM round trip before the staging, not two).  The chunk
 * table is still read for chunks >= 1.  Records and chunk indices are those
 * of ingot_gpu_parse_read over the same chunks (the caller keeps d_first
 * consistent with the table).  16-B records; chunk 0 in the default
 * line-completing 3-5-piece window (INGOT_TUNE_READ_PLAN 1: 4 pieces; 17:
 * the chunk bounds loaded only by walks that leave chunk 0 or fail in it —
 * set it for header-split producers).
 */
int ingot_gpu_parse_read_first(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                               const uint64_t* d_seg_off, const uint16_t* d_seg_len,
                               const uint32_t* d_pkt_seg, const uint64_t* d_first, uint64_t n,
                               int chain, ingot_rec* d_out, uint16_t* d_chunk, void* stream);

/* ---------------------------------------------------------------------------
 * In-place header rewrite: ingot's generated setters (packet/mod.rs:2097-2255;
 * BE bitfield set paths, bitfield.rs:188-315) after the parse, e.g. the
 * reference's `parse-and-decr-v4` bench (ingot-examples/benches/packet.rs:
 * 139-145: l4.set_destination(l4.destination() - 1)).
 *
 * Every packet is parsed as `chain`; for packets that parse Ok the edits are
 * applied in order, each to the header at chain layer `layer` (the label
 * index: UdpParser 0 eth, 1 l3, 2 l4; GenericUlp 0-2; VlanUlp 0 eth, 1 vlan
 * (tag `index`), 2 l3, 3 l4; GeneveOverV6Tunnel 0-6) when that layer holds
 * the header kind the field belongs to (an IPv4 field on an IPv6 layer, or
 * on a layer skipped by an accepting control, is not applied).  Values are
 * the raw wire bits (NetworkRepr::to_network already applied, e.g. Ecn
 * Capable1 = 2); ADD/SUB wrap modulo 2^width; the neighbouring bits of a
 * bitfield are preserved.  Offsets come from the one parse: an edit never
 * re-parses (as in ingot, setting ihl does not move the L4 view).
 * ------------------------------------------------------------------------- */
enum ingot_field {
    INGOT_F_ETH_ETHERTYPE = 0,
    INGOT_F_VLAN_PRIORITY, INGOT_F_VLAN_DEI, INGOT_F_VLAN_VID, INGOT_F_VLAN_ETHERTYPE,
    INGOT_F_V4_VERSION, INGOT_F_V4_IHL, INGOT_F_V4_DSCP, INGOT_F_V4_ECN, INGOT_F_V4_TOTAL_LEN,
    INGOT_F_V4_IDENTIFICATION, INGOT_F_V4_FLAGS, INGOT_F_V4_FRAGMENT_OFFSET,
    INGOT_F_V4_HOP_LIMIT, INGOT_F_V4_PROTOCOL, INGOT_F_V4_CHECKSUM, INGOT_F_V4_SOURCE,
    INGOT_F_V4_DESTINATION,
    INGOT_F_V6_VERSION, INGOT_F_V6_DSCP, INGOT_F_V6_ECN, INGOT_F_V6_FLOW_LABEL,
    INGOT_F_V6_PAYLOAD_LEN, INGOT_F_V6_NEXT_HEADER, INGOT_F_V6_HOP_LIMIT,
    INGOT_F_TCP_SOURCE, INGOT_F_TCP_DESTINATION, INGOT_F_TCP_SEQUENCE,
    INGOT_F_TCP_ACKNOWLEDGEMENT, INGOT_F_TCP_DATA_OFFSET, INGOT_F_TCP_RESERVED,
    INGOT_F_TCP_FLAGS, INGOT_F_TCP_WINDOW_SIZE, INGOT_F_TCP_CHECKSUM, INGOT_F_TCP_URGENT_PTR,
    INGOT_F_UDP_SOURCE, INGOT_F_UDP_DESTINATION, INGOT_F_UDP_LENGTH, INGOT_F_UDP_CHECKSUM,
    INGOT_F_ICMP_TY, INGOT_F_ICMP_CODE, INGOT_F_ICMP_CHECKSUM,
    INGOT_F_GENEVE_VERSION, INGOT_F_GENEVE_OPT_LEN, INGOT_F_GENEVE_FLAGS,
    INGOT_F_GENEVE_PROTOCOL_TYPE, INGOT_F_GENEVE_VNI, INGOT_F_GENEVE_RESERVED,
    INGOT_F_COUNT
};
enum ingot_edit_op {
    INGOT_OP_SET = 0, INGOT_OP_ADD = 1, INGOT_OP_SUB = 2, INGOT_OP_AND = 3, INGOT_OP_OR = 4,
    INGOT_OP_XOR = 5
};
#define INGOT_MAX_EDITS 16

typedef struct ingot_edit {
    uint8_t layer;   /* chain layer index (label) */
    uint8_t field;   /* enum ingot_field */
    uint8_t op;      /* enum ingot_edit_op */
    uint8_t index;   /* VLAN tag (VLAN_ULP's vlan layer), else 0 */
    uint32_t value;  /* raw wire bits */
} ingot_edit;

#ifdef __cplusplus
static_assert(sizeof(ingot_edit) == 8, "ingot_edit is 8 bytes");
#endif

/* Parse + rewrite in place.  `edits` is host memory (<= INGOT_MAX_EDITS);
 * d_out (optional) receives the parse records.  d_off == NULL selects the
 * strided layout (as ingot_gpu_fields). */
int ingot_gpu_parse_modify(ingot_gpu_ctx* ctx, uint8_t* d_arena,
                           const uint64_t* d_off, const uint16_t* d_len,
                           uint32_t stride, uint64_t n, int chain,
                           const ingot_edit* edits, uint32_t n_edits,
                           ingot_rec* d_out, void* stream);

/* ---------------------------------------------------------------------------
 * Batched Emit: ingot's `Emit` (ingot-types/src/emit.rs:8-120; the generated
 * owned `emit_raw`, ingot-macros/src/packet/mod.rs:2097-2255) of one owned
 * header stack per packet, followed by the packet's own bytes — the tuple
 * `(headers, &payload[..])` emitted for every packet of a batch, e.g. OPTE's
 * outbound Geneve encapsulation (outer Ethernet / IPv6 / UDP / Geneve + options
 * in front of the inner frame, ingot-examples/src/packets.rs:27-40).
 *
 * The owned headers are serialised ONCE, on the host, by the caller (ingot's
 * own `(eth, v6, udp, geneve).emit_vec()`, or ingot_amd.emit_headers in the
 * Python mirror): `hdr`, hdr_len <= INGOT_MAX_EMIT_HDR bytes of host memory.
 * The device then writes them in front of every packet and applies the
 * per-packet setters `sets` (<= INGOT_MAX_EMIT_SETS; host memory) to that
 * packet's copy, in order: the field `field` (enum ingot_field) of the header
 * that starts at byte `at` of `hdr` is set (bitfield.rs:188-315 set paths,
 * neighbouring bits kept, big-endian) to
 *   INGOT_EMIT_LENGTH  the packet's emitted bytes from `at` to its end, + add
 *                      (IPv6 payload_len: at = the IPv6 header, add = -40;
 *                      UDP / IPv4 length: add = 0);
 *   INGOT_EMIT_U16     ((const uint16_t*)d_values)[i] + add  (device array);
 *   INGOT_EMIT_U32     ((const uint32_t*)d_values)[i] + add  (device array);
 *   INGOT_EMIT_VALUE   add (the same value for every packet);
 * wrapping modulo 2^width.  The field must lie inside hdr (EINVAL).
 *
 * ingot_gpu_emit_packets: packet i (hdr_len + d_len[i] bytes) is written at
 * d_dst + d_dst_off[i]: the headers, then d_src[d_off[i] .. + d_len[i]).
 * hdr_len 0 is a plain gather-copy (decapsulation: the inner frames at their
 * parsed offsets).  Sources are read in aligned 16-B blocks (the arena must be
 * readable to the 16-B boundary past each packet); destinations are written
 * exactly (packets may be packed back to back); source and destination must
 * not overlap.
 *
 * ingot_gpu_emit_headers: only the header blocks, packet i's at d_out +
 * (d_out_off ? d_out_off[i] : i * out_stride); LENGTH counts hdr_len +
 * d_len[i] (the payload that will follow).  With d_out_off[i] = off[i] -
 * hdr_len into the frames' own arena this is `emit_suffix` into headroom (the
 * packet becomes contiguous in place); into separate slots it is the header
 * chunk of a two-chunk packet that ingot_gpu_parse_read parses as is.
 * hdr_len must be >= 1 here (EINVAL); slots narrower than the block
 * (d_out_off NULL, out_stride < hdr_len) are ERANGE.  Header blocks are
 * written exactly (neighbouring bytes untouched); destinations at any
 * alignment.
 * ------------------------------------------------------------------------- */
enum ingot_emit_source {
    INGOT_EMIT_LENGTH = 0,
    INGOT_EMIT_U16 = 1,
    INGOT_EMIT_U32 = 2,
    INGOT_EMIT_VALUE = 3
};
#define INGOT_MAX_EMIT_SETS 8
#define INGOT_MAX_EMIT_HDR 256

typedef struct ingot_emit_set {
    uint16_t at;           /* byte offset in hdr of the header holding the field */
    uint8_t field;         /* enum ingot_field */
    uint8_t source;        /* enum ingot_emit_source */
    int32_t add;           /* added to the value (VALUE: the value) */
    const void* d_values;  /* U16 / U32: n per-packet values (device memory) */
} ingot_emit_set;

#ifdef __cplusplus
static_assert(sizeof(ingot_emit_set) == 16, "ingot_emit_set is 16 bytes");
#endif

int ingot_gpu_emit_packets(ingot_gpu_ctx* ctx, const uint8_t* hdr, uint32_t hdr_len,
                           const ingot_emit_set* sets, uint32_t n_sets,
                           const uint8_t* d_src, const uint64_t* d_off,
                           const uint16_t* d_len, uint64_t n, uint8_t* d_dst,
                           const uint64_t* d_dst_off, void* stream);
int ingot_gpu_emit_headers(ingot_gpu_ctx* ctx, const uint8_t* hdr, uint32_t hdr_len,
                           const ingot_emit_set* sets, uint32_t n_sets,
                           const uint16_t* d_len, uint64_t n, uint8_t* d_out,
                           const uint64_t* d_out_off, uint32_t out_stride, void* stream);

/*
 * Flow classification + per-flow histogram (config 5; build-defined, ingot
 * has no flow hash).  For every packet that parses Ok as `chain` with an
 * IPv4/IPv6 layer, the RSS Toeplitz hash of
 *     source addr | destination addr | (source port | destination port)
 * (ports only when the L4 layer is TCP or UDP; network byte order, the
 * Microsoft RSS input order) with the 40-byte `key` (host memory; NULL =
 * the standard Microsoft RSS key).  Outputs:
 *   d_flow  (required, n x u32)  the packet's flow bin hash & (bins - 1), or
 *           INGOT_FLOW_NONE for packets that are not counted;
 *   d_hash  (optional, n x u32)  the full hash, 0 when not counted;
 *   d_hist  (optional, bins x u32) d_hist[bin] += 1 per counted packet —
 *           accumulated into (zero it to start a new histogram).
 * bins is a power of two <= 2^24.  d_off == NULL selects the strided layout
 * (as ingot_gpu_fields).  Two launches: parse + hash, then a contention-free
 * histogram pass over d_flow (LDS-privatised counters).
 *
 * ingot_gpu_flow_hist_ws: the same with a caller-owned device workspace
 * (d_work, work_bytes >= ingot_gpu_flow_hist_workspace_size(n, bins), e.g.
 * 16 MiB for 8 M packets x 65,536 bins): the histogram pass then stores
 * per-block counters there and reduces them without atomics (faster; see
 * DESIGN.md).  Size 0 = no workspace is used for (n, bins); a smaller or NULL
 * workspace falls back to the atomic pass.  Like the arena, the workspace is
 * borrowed for the call: calls that run concurrently need their own.
 */
#define INGOT_FLOW_KEY_BYTES 40
#define INGOT_FLOW_NONE 0xffffffffu
int ingot_gpu_flow_hist(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                        const uint64_t* d_off, const uint16_t* d_len,
                        uint32_t stride, uint64_t n, int chain,
                        const uint8_t* key, uint32_t bins, uint32_t* d_flow,
                        uint32_t* d_hash, uint32_t* d_hist, void* stream);
int ingot_gpu_flow_hist_ws(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                           const uint64_t* d_off, const uint16_t* d_len,
                           uint32_t stride, uint64_t n, int chain,
                           const uint8_t* key, uint32_t bins, uint32_t* d_flow,
                           uint32_t* d_hash, uint32_t* d_hist, void* d_work,
                           size_t work_bytes, void* stream);
size_t ingot_gpu_flow_hist_workspace_size(uint64_t n, uint32_t bins);

/*
 * The multi-GPU reduce of config 5 (the only collective of the design).
 * Packets shard across GPUs by contiguous index ranges with no exchange;
 * each rank's ingot_gpu_flow_hist leaves a per-rank histogram, and the job's
 * histogram is their element-wise sum: RCCL all-reduce (sum, uint32) over
 * xGMI, 65,536 x u32 = 256 KiB at the default bins.
 *
 * One process (or thread) per GPU.  Rank 0 makes a communicator id with
 * ingot_gpu_comm_unique_id and the host sends its INGOT_COMM_ID_BYTES bytes to
 * every rank over its own control channel; every rank then calls
 * ingot_gpu_comm_create with the same id, nranks and its own rank (this
 * blocks until all ranks have joined).  The communicator is bound to ctx's
 * device.  RCCL is loaded at the first call of these functions (librccl.so.1,
 * the one already in the process if there is one); INGOT_GPU_ENODEV if it
 * cannot be loaded, INGOT_GPU_ECOMM if an RCCL call fails.
 *
 * ingot_gpu_flow_hist_allreduce enqueues the in-place sum of d_hist (bins x
 * u32, device memory of the communicator's device) across all ranks on
 * `stream`, ordered after the work already enqueued there (e.g. the
 * ingot_gpu_flow_hist that filled it) and before what follows; every rank
 * must enqueue the same sequence of reduces.  The counts wrap modulo 2^32.
 *
 * Release: ingot_gpu_comm_destroy on every rank flushes the reduces issued,
 * waits until the communicator is quiescent on all ranks (ncclCommFinalize)
 * and frees it; ingot_gpu_comm_abort frees it at once, locally, aborting any
 * reduce still in flight (error paths, or a process that is exiting after its
 * streams have drained).  Either way the handle is gone afterwards.
 *
 * A host that already holds an RCCL communicator over the same ranks (its
 * own, or PyTorch's ProcessGroupNCCL) hands it over with ingot_gpu_comm_wrap
 * instead of creating a second one: one RCCL communicator per process is the
 * layout that ran clean (with two per process the world-2
 * rehearsal stalled).  `nccl_comm` is an ncclComm_t of the process's
 * librccl.so.1; the handle borrows it: size and rank are the communicator's,
 * its device must be ctx's (else INGOT_GPU_EINVAL), and
 * ingot_gpu_comm_destroy / _abort free only the handle — the borrowed
 * communicator stays the host's and must outlive the handle.
 */
#define INGOT_GPU_ECOMM (-6)    /* a collective (RCCL) call failed */
#define INGOT_COMM_ID_BYTES 128
typedef struct ingot_gpu_comm ingot_gpu_comm;
int ingot_gpu_comm_unique_id(uint8_t id[INGOT_COMM_ID_BYTES]);
int ingot_gpu_comm_create(ingot_gpu_ctx* ctx, int nranks, int rank,
                          const uint8_t id[INGOT_COMM_ID_BYTES], ingot_gpu_comm** out);
int ingot_gpu_comm_wrap(ingot_gpu_ctx* ctx, void* nccl_comm, ingot_gpu_comm** out);
int ingot_gpu_comm_destroy(ingot_gpu_comm* comm);
int ingot_gpu_comm_abort(ingot_gpu_comm* comm);
int ingot_gpu_comm_size(const ingot_gpu_comm* comm);
int ingot_gpu_comm_rank(const ingot_gpu_comm* comm);
int ingot_gpu_flow_hist_allreduce(ingot_gpu_comm* comm, uint32_t* d_hist, uint32_t bins,
                                  void* stream);

/* ---------------------------------------------------------------------------
 * Frames stored back to back with only a length array (a capture buffer, a
 * ring without a descriptor table): frame i starts at d_arena + the sum of
 * d_len[0..i).  The offsets are derived on the device — a base per
 * 64-packet tile from a scan of tile sums (two small passes over the lengths,
 * into the caller's workspace d_work of >= ingot_gpu_packed_workspace_size(n)
 * bytes, 8-B aligned), then a wavefront prefix scan of each tile's lengths
 * inside the parse — and the batch is parsed as by ingot_gpu_parse.  2 B of
 * descriptor per packet instead of 10.  d_off_out (optional, n x u64)
 * receives the offsets.
 * ------------------------------------------------------------------------- */
size_t ingot_gpu_packed_workspace_size(uint64_t n);
int ingot_gpu_parse_packed(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                           const uint16_t* d_len, uint64_t n, int chain,
                           ingot_rec* d_out, uint64_t* d_off_out, void* d_work,
                           size_t work_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * Single-header parse, batched: `HeaderParse::parse(slice)` of one header kind
 * at the start of every slice (ingot-types/src/lib.rs:137-147; the generated
 * bodies, packet/mod.rs:1831-2005) — ValidEthernet::parse, ValidIpv4::parse
 * ... as the reference's `ingot/benches/modify.rs:79-104` parse benches — or
 * a choice's `parse_choice(slice, hint)` (ingot-macros/src/choice.rs:231-246:
 * no hint -> NeedsHint, a hint no variant takes -> Unwanted), as
 * `ValidL3::parse_choice` in `ingot-examples/benches/choice.rs`.
 *
 * Per slice one 8-B ingot_hdr: status (0 Ok, else 1 + ParseError), the header
 * parsed (for a choice: the variant taken), `used` = its HeaderLen (the
 * remainder starts there) and `hint` = its NextLayer hint (ethertype /
 * IpProtocol; INGOT_HINT_NONE = None: TCP, UDP, ICMP, Geneve).  Choices take
 * d_hint[i] when d_hint is non-NULL, else `hint` for every slice
 * (INGOT_HINT_NONE = None).  Slices: (d_off[i], d_len[i]) or fixed slots of
 * `stride` bytes (d_off NULL; d_len optional).
 * ------------------------------------------------------------------------- */
enum ingot_header_kind {
    INGOT_HDR_ETHERNET = 0,  /* ethernet.rs:46-55 */
    INGOT_HDR_VLAN = 1,      /* ethernet.rs:57-65 (VlanBody) */
    INGOT_HDR_IPV4 = 2,      /* ip.rs:63-93 */
    INGOT_HDR_IPV6 = 3,      /* ip.rs:159-182, with its extension-header chain */
    INGOT_HDR_TCP = 4,       /* tcp.rs:9-30 */
    INGOT_HDR_UDP = 5,       /* udp.rs:8-15 */
    INGOT_HDR_ICMP = 6,      /* icmp.rs:42-50 (v4 and v6 share the layout) */
    INGOT_HDR_REPEATED_UDP = 7, /* Repeated<Udp> over the whole slice (util.rs:189-228) */
    INGOT_HDR_GENEVE = 8,    /* geneve.rs:16-44, options subparsed */
    INGOT_HDR_L3 = 16,       /* choice L3 (ingot-examples/src/choices.rs:17-21) */
    INGOT_HDR_L4 = 17,       /* choice L4 (choices.rs:25-29) */
    INGOT_HDR_ULP = 18       /* choice Ulp (choices.rs:32-38) */
};
#define INGOT_HINT_NONE 0xffffffffu

typedef struct ingot_hdr {
    uint8_t status;  /* 0 = Ok, else 1 + ParseError */
    uint8_t kind;    /* enum ingot_header_kind parsed (a choice's variant) */
    uint16_t used;   /* HeaderLen: bytes consumed from the slice start */
    uint32_t hint;   /* NextLayer hint, INGOT_HINT_NONE = None */
} ingot_hdr;

#ifdef __cplusplus
static_assert(sizeof(ingot_hdr) == 8, "ingot_hdr is 8 bytes");
#endif

int ingot_gpu_parse_header(ingot_gpu_ctx* ctx, const uint8_t* d_arena,
                           const uint64_t* d_off, const uint16_t* d_len,
                           uint32_t stride, uint64_t n, int kind,
                           const uint32_t* d_hint, uint32_t hint,
                           ingot_hdr* d_out, void* stream);

/* Error strings. */
const char* ingot_gpu_strerror(int api_code);
/* ParseError name as ingot prints it (error.rs:49-60): "Unwanted", ... ;
 * "Ok" for 0, NULL if out of range. */
const char* ingot_parse_error_name(int status);
/* Layer label of a chain (the PacketParseError label, parse.rs:36-50). */
const char* ingot_chain_layer_label(int chain, int layer);
int ingot_chain_layer_count(int chain);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* INGOT_GPU_H */
