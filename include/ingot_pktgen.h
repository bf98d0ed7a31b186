/*
 * ingot_pktgen.h — synthetic traffic for benches and parity tests (C ABI).
 *
 * Not part of the parse path: a device-side frame generator whose output is a
 * pure function of (profile, seed, frame index), so any shard of any size can
 * be regenerated on any GPU and sampled frames can be re-checked on the host.
 * Profiles follow SURVEY.md §8d (seed 20250808 by convention):
 *
 *   INGOT_GEN_ADVERSARIAL  0..160-B frames, random/truncated header chains,
 *                          random ihl/data_offset 0-15, unknown ethertypes and
 *                          protocols, IPv6 EH chains of random type/length —
 *                          the parity fuzz set (every error path).
 *   INGOT_GEN_V4UDP64      C1/C2: 64-B Eth/IPv4/UDP, modelled on
 *                          ingot-examples/benches/packet.rs:15-34 (dst 00:..,
 *                          src ff:.., ihl 5, ttl 0xf0, proto 17), random
 *                          addresses/ports, zero padding.
 *   INGOT_GEN_MIXED        C3: len ~ U[64,1500]; v4:v6 1:1; TCP:UDP 1:1;
 *                          ihl 5 (p .9) else U[6,15]; data_offset 5 (p .7) else
 *                          U[6,15]; v6 EH count 0 (p .8) else U[1,3] drawn from
 *                          {0,60,43,44}, ext_len U[0,3]; length raised to fit.
 *   INGOT_GEN_VLAN_V6EH    C4: as MIXED but VLAN p .5 (QinQ 0x9100+0x8100 p .2
 *                          of those), IPv6 p .5 with EHs p .5.
 *   INGOT_GEN_FLOWS        C5: C4 framing; the 5-tuple is drawn from 65,536
 *                          flows with Zipf(1.1) popularity.
 *   INGOT_GEN_GENEVE       C6 (GeneveOverV6Tunnel, OPTE inbound): outer Eth /
 *                          IPv6 (HBH p .05) / UDP 6081 / Geneve with 0, 1
 *                          (class 0x0129, p .8) or 2 options; inner Eth with
 *                          ARP p .02, IPv4 p .68, IPv6 p .30; TCP p .75, UDP
 *                          p .22, ICMP p .03; inner length U[64,1500].
 *   INGOT_GEN_GENEVE_ADVERSARIAL  tunnel-shaped fuzz: outer ethertype / EHs /
 *                          L4 / Geneve option spans perturbed, adversarial
 *                          inner chain, lengths clustered at the chain's end.
 */
#ifndef INGOT_PKTGEN_H
#define INGOT_PKTGEN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ingot_gen_profile {
    INGOT_GEN_ADVERSARIAL = 0,
    INGOT_GEN_V4UDP64 = 2,
    INGOT_GEN_MIXED = 3,
    INGOT_GEN_VLAN_V6EH = 4,
    INGOT_GEN_FLOWS = 5,
    INGOT_GEN_GENEVE = 6,
    INGOT_GEN_GENEVE_ADVERSARIAL = 7
};

#define INGOT_GEN_SEED 20250808ull
#define INGOT_GEN_FLOWS_N 65536u

/* Frame lengths of frames [first, first+n) into d_len (device, u16). */
int ingot_pktgen_lengths(int profile, uint64_t seed, uint64_t first, uint64_t n,
                         uint16_t* d_len, void* stream);

/*
 * Write frames [first, first+n) into d_arena.  d_off == NULL selects the
 * strided layout (frame i at i*stride).  d_len must hold the lengths produced
 * by ingot_pktgen_lengths (or, strided, NULL = stride).  `arena_bytes` bounds
 * every write.  Bytes between/after frames are filled with a pattern too.
 */
int ingot_pktgen_fill(int profile, uint64_t seed, uint64_t first, uint64_t n,
                      const uint64_t* d_off, uint32_t stride, const uint16_t* d_len,
                      uint8_t* d_arena, uint64_t arena_bytes, void* stream);

/*
 * The same generator on the host (libingot_pktgen_host.so, no HIP): the
 * same bytes as the device calls for the same arguments, into host memory
 * (h_arena 16-B aligned); `threads` > 1 splits the work.  bench.py builds its
 * CPU baseline's sample with these before the process touches the GPU.
 */
int ingot_pktgen_lengths_host(int profile, uint64_t seed, uint64_t first, uint64_t n,
                              uint16_t* h_len, int threads);
int ingot_pktgen_fill_host(int profile, uint64_t seed, uint64_t first, uint64_t n,
                           const uint64_t* h_off, uint32_t stride, const uint16_t* h_len,
                           uint8_t* h_arena, uint64_t arena_bytes, int threads);

#ifdef __cplusplus
}
#endif

#endif
