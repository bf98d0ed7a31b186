/*
 * ingot_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A scalar CPU restatement of ingot's single-slice parse path, used as the
 * parity checker for the HIP kernels and as the CPU baseline in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product library (ingot_amd/) never links or calls it.
 *
 * The reference (Rust, toolchain 1.81.0) cannot be built or run here: there is
 * no cargo/rustc in this image.  This restatement is pinned by
 * the reference's own known-answer tests, transcribed as fixtures under
 * tests/golden/ (see tests/golden/make_golden.py).
 *
 * Records and field blocks use the product ABI layouts (include/ingot_gpu.h)
 * so results can be compared byte-for-byte.
 */
#ifndef INGOT_ORACLE_H
#define INGOT_ORACLE_H

#include <stdint.h>
#include "../include/ingot_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parse one frame as `chain`; fills *rec (required) and *fields (optional). */
void oracle_parse_one(const uint8_t* frame, uint32_t len, int chain,
                      ingot_rec* rec, ingot_fields* fields);

/* GeneveOverV6Tunnel with the outer layers' getters (inner.rec is the record);
 * batch form single-threaded (layouts as oracle_parse_batch). */
void oracle_parse_geneve(const uint8_t* frame, uint32_t len, ingot_geneve_fields* out);
int oracle_geneve_fields_batch(const uint8_t* arena, const uint64_t* off,
                               const uint16_t* len, uint32_t stride, uint64_t n,
                               ingot_geneve_fields* out);

/* parse_read (ingot-macros/src/parse.rs:511-537) over multi-segment packets:
 * packet i is the chunks seg[pkt_seg[i] .. pkt_seg[i+1]) of (seg_off, seg_len)
 * in `arena`; record offsets are logical (the chunks concatenated).  chunk[i]
 * (optional) = index of the chunk holding the remainder.  fields (ingot_fields)
 * or gfields (GENEVE_OVER_V6's ingot_geneve_fields) optional, not both. */
int oracle_parse_read_batch(const uint8_t* arena, const uint64_t* seg_off,
                            const uint16_t* seg_len, const uint32_t* pkt_seg, uint64_t n,
                            int chain, ingot_rec* rec, ingot_fields* fields,
                            ingot_geneve_fields* gfields, uint16_t* chunk, int nthreads);

/* Batch form.  off == NULL selects the strided layout (frame i at i*stride);
 * len == NULL means every frame is `stride` bytes long.  fields may be NULL.
 * nthreads <= 1 runs on the calling thread; otherwise a static contiguous
 * partition over nthreads pthreads.  Returns 0, or -1 on bad arguments. */
int oracle_parse_batch(const uint8_t* arena, const uint64_t* off,
                       const uint16_t* len, uint32_t stride, uint64_t n,
                       int chain, ingot_rec* rec, ingot_fields* fields,
                       int nthreads);

/* Throughput measurement only: every batch worker repeats its range `passes`
 * times per call (thread start-up amortised over more work). */
void oracle_set_passes(int passes);
/* Pin batch worker t to cpus[t % n] (NULL / 0: unpinned); bench.py's CPU baseline. */
void oracle_set_affinity(const int* cpus, int n);

/* Generic big-endian bitfield getter (ingot-macros/src/packet/bitfield.rs
 * BE get paths): the n_bits (<= 64) starting at bit first_bit, MSB first. */
uint64_t oracle_be_bits(const uint8_t* hdr, uint32_t first_bit, uint32_t n_bits);

/* BE setter (bitfield.rs set paths): n_bits of value at first_bit, other bits
 * of the covering bytes unchanged. */
void oracle_be_set_bits(uint8_t* hdr, uint32_t first_bit, uint32_t n_bits, uint64_t value);

/* ingot_gpu_parse_modify semantics on one frame / a batch (in place). */
int oracle_parse_modify(uint8_t* frame, uint32_t len, int chain, const ingot_edit* edits,
                        uint32_t n_edits, ingot_rec* rec);
int oracle_parse_modify_batch(uint8_t* arena, const uint64_t* off, const uint16_t* len,
                              uint32_t stride, uint64_t n, int chain, const ingot_edit* edits,
                              uint32_t n_edits, ingot_rec* rec, int nthreads);

/* ingot_gpu_emit_packets (copy = 1) / ingot_gpu_emit_headers (copy = 0)
 * semantics on the host; U16 / U32 set sources are host arrays.  Packets
 * written by different threads must not share destination bytes. */
int oracle_emit_batch(const uint8_t* hdr, uint32_t hdr_len, const ingot_emit_set* sets,
                      uint32_t n_sets, const uint8_t* src, const uint64_t* off,
                      const uint16_t* len, uint64_t n, uint8_t* dst, const uint64_t* dst_off,
                      uint32_t stride, int copy, int nthreads);

/* IpProtocol::class (ingot/src/ip.rs:40-54): 0 = None, 1 = FragmentHeader,
 * 2 = Rfc6564. */
int oracle_v6eh_class(uint8_t proto);

/* Header-level parse (ValidX::parse); see ingot_oracle.c. */
int oracle_parse_header(int kind, const uint8_t* s, uint32_t n, uint32_t* used,
                        uint32_t* hint_out);
/* A choice's parse_choice(slice, hint) (choice.rs:231-246): kind 16 = L3,
 * 17 = L4, 18 = Ulp (choices.rs:17-38); hint 0xffffffff = None.  *variant =
 * the header kind taken (0-8 numbering of oracle_parse_header). */
int oracle_parse_choice(int kind, uint32_t hint, const uint8_t* s, uint32_t n, uint32_t* used,
                        uint32_t* hint_out, uint32_t* variant);
/* ingot_gpu_parse_header semantics over a batch of slices ((off, len) or
 * slots of `stride`), one ingot_hdr each. */
int oracle_parse_header_batch(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                              uint32_t stride, uint64_t n, int kind, const uint32_t* hints,
                              uint32_t hint, ingot_hdr* out);

/* Toeplitz (RSS) hash of `n` input bytes with a key of >= n+4 bytes. */
uint32_t oracle_toeplitz(const uint8_t* key, uint32_t key_len,
                         const uint8_t* data, uint32_t n);

/* Flow classification (ingot_gpu_flow_hist semantics): returns 1 and the
 * Toeplitz hash when the frame is counted, else 0 (*hash = 0). */
int oracle_flow_hash(const uint8_t* frame, uint32_t len, int chain, const uint8_t* key,
                     uint32_t* hash);
/* Batch: hist[hash & (bins-1)] += 1 for counted frames (accumulates);
 * hash_out / flow_out (bin or INGOT_FLOW_NONE) optional. */
int oracle_flow_hist(const uint8_t* arena, const uint64_t* off, const uint16_t* len,
                     uint32_t stride, uint64_t n, int chain, const uint8_t* key, uint32_t* hist,
                     uint32_t bins, uint32_t* hash_out, uint32_t* flow_out);

#ifdef __cplusplus
}
#endif

#endif
