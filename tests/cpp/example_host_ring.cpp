// example_host_ring.cpp — an OPTE-style consumer of the C ABI with frames that
// never leave host memory: a pageable ring of 256-B slots and its length table
// are mapped once (ingot_gpu_host_map); each batch is parsed in place over
// PCIe (only header chunks cross) with the records written straight into a
// mapped host array; results are checked against what UdpParser::parse /
// GenericUlp::parse_slice return for the same frames (ingot-examples/src/
// packets.rs:18-24, 54-60).  Run on the GPU by tests/test_cpp_mirror.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "ingot_gpu.h"

static int fail(const char* what) {
    std::printf("FAIL %s\n", what);
    return 1;
}

int main() {
    const uint32_t slot = 256, n = 100000;
    std::vector<uint8_t> ring((size_t)slot * n + 4096, 0);
    std::vector<uint16_t> lens(n);
    std::vector<ingot_rec> recs(n);
    // ingot-examples/benches/packet.rs:15-35 pkt_body_v4, UDP ports varied per
    // slot; every 7th slot an ARP frame, every 11th a truncated UDP header.
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* f = ring.data() + (size_t)i * slot;
        std::memset(f + 6, 0xff, 6);
        const bool arp = i % 7 == 3;
        f[12] = 0x08;
        f[13] = arp ? 0x06 : 0x00;
        const uint8_t v4[20] = {0x45, 0, 0, 28 + 8, 0, 0, 0, 0, 0xf0, 0x11, 0, 0,
                                192, 168, 0, 1, 192, 168, 0, 255};
        std::memcpy(f + 14, v4, 20);
        f[34] = (uint8_t)(i >> 8);
        f[35] = (uint8_t)i;
        f[36] = 0x17;
        f[37] = 0xc1;
        f[39] = 8;
        lens[i] = (uint16_t)(i % 11 == 5 ? 40 : 50);
    }
    ingot_gpu_ctx* ctx = nullptr;
    if (ingot_gpu_ctx_create(0, &ctx)) return fail("ctx_create");
    void *d_ring = nullptr, *d_len = nullptr, *d_rec = nullptr;
    if (ingot_gpu_host_map(ctx, ring.data(), ring.size(), &d_ring) ||
        ingot_gpu_host_map(ctx, lens.data(), lens.size() * 2, &d_len) ||
        ingot_gpu_host_map(ctx, recs.data(), recs.size() * sizeof(ingot_rec), &d_rec))
        return fail("host_map");
    int bad = 0;
    for (int chain : {INGOT_CHAIN_UDP_PARSER, INGOT_CHAIN_GENERIC_ULP}) {
        std::memset(recs.data(), 0xee, recs.size() * sizeof(ingot_rec));
        if (ingot_gpu_parse_strided(ctx, (const uint8_t*)d_ring, slot, (const uint16_t*)d_len, n,
                                    chain, (ingot_rec*)d_rec, nullptr))
            return fail("parse_strided");
        if (hipDeviceSynchronize() != hipSuccess) return fail("sync");
        for (uint32_t i = 0; i < n; ++i) {
            const ingot_rec& r = recs[i];
            const bool arp = i % 7 == 3, cut = i % 11 == 5;
            if (arp && chain == INGOT_CHAIN_UDP_PARSER) {
                // L3 choice: ARP is Unwanted at "l3"
                bad += r.status != INGOT_ERR_UNWANTED || r.err_layer != 1;
            } else if (arp) {
                // exit_on_arp accepts at inner_eth: Ok, remainder after 14 B
                bad += r.status != INGOT_OK || !(r.flags & INGOT_REC_ACCEPTED) ||
                       r.payload_off != 14;
            } else if (cut) {
                bad += r.status != INGOT_ERR_TOO_SMALL || r.err_layer != 2;
            } else {
                const uint8_t* f = ring.data() + (size_t)i * slot + r.l4_off;
                const uint16_t src = (uint16_t)(f[0] << 8 | f[1]);
                bad += r.status != INGOT_OK || r.l3_off != 14 || r.l4_off != 34 ||
                       r.payload_off != 42 || r.l4_kind != INGOT_L4_UDP ||
                       src != (uint16_t)i;
            }
        }
        std::printf("%s %s: %u frames parsed from host memory\n", bad ? "FAIL" : "ok  ",
                    ingot_chain_layer_label(chain, 0), n);
    }
    ingot_gpu_host_unmap(ctx, recs.data());
    ingot_gpu_host_unmap(ctx, lens.data());
    ingot_gpu_host_unmap(ctx, ring.data());
    ingot_gpu_ctx_destroy(ctx);
    std::printf("%d mismatches\n", bad);
    return bad ? 1 : 0;
}
