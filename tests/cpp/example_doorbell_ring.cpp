// example_doorbell_ring.cpp — a NIC-ring consumer of the C ABI that never
// launches on the critical path: the parses of the next BATCHES ring slots
// are enqueued up front, each behind ingot_gpu_doorbell_wait(db, k + 1); a
// producer thread fills slot k (frames copied into the device ring) and
// publishes it with ingot_gpu_doorbell_ring(db, k + 1); the GPU then starts
// that parse with no host round trip.  Checks: the first parse is still held
// before its doorbell rings, and every record equals what UdpParser::parse
// returns for the frame (ingot-examples/src/packets.rs:18-24: IPv4/UDP Ok,
// ARP Unwanted at l3).  Run on the GPU by tests/test_cpp_mirror.py.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "ingot_gpu.h"

static int fail(const char* what) {
    std::printf("FAIL %s\n", what);
    return 1;
}

#define HIP_OK(x)                                     \
    do {                                              \
        if ((x) != hipSuccess) return fail(#x);       \
    } while (0)

int main() {
    constexpr uint32_t kSlot = 64, kN = 65536, kBatches = 8;
    ingot_gpu_ctx* ctx = nullptr;
    if (ingot_gpu_ctx_create(0, &ctx) != 0) return fail("ctx_create");
    ingot_gpu_doorbell* db = nullptr;
    volatile uint32_t* word = nullptr;
    if (ingot_gpu_doorbell_create(ctx, &db, &word) != 0 || !word) return fail("doorbell_create");

    // the device ring (one batch per slot group) and the records
    uint8_t* d_ring = nullptr;
    ingot_rec* d_rec = nullptr;
    HIP_OK(hipMalloc(&d_ring, (size_t)kSlot * kN * kBatches));
    HIP_OK(hipMalloc(&d_rec, sizeof(ingot_rec) * kN * kBatches));
    HIP_OK(hipMemset(d_rec, 0xee, sizeof(ingot_rec) * kN * kBatches));
    hipStream_t cs, ps;
    HIP_OK(hipStreamCreate(&cs));
    HIP_OK(hipStreamCreate(&ps));

    // consumer: every batch's parse enqueued before any frame exists
    std::vector<hipEvent_t> done(kBatches);
    for (uint32_t k = 0; k < kBatches; ++k) {
        HIP_OK(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
        if (ingot_gpu_doorbell_wait(db, k + 1, cs) != 0) return fail("doorbell_wait");
        if (ingot_gpu_parse_strided(ctx, d_ring + (size_t)k * kSlot * kN, kSlot, nullptr, kN,
                                    INGOT_CHAIN_UDP_PARSER, d_rec + (size_t)k * kN, cs) != 0)
            return fail("parse_strided");
        HIP_OK(hipEventRecord(done[k], cs));
    }

    // producer: pkt_body_v4 (ingot-examples/benches/packet.rs:15-35) with the
    // UDP source port = the frame's index; every 5th frame of odd batches ARP
    std::vector<uint8_t> host((size_t)kSlot * kN);
    bool held = false, copy_stuck = false;
    std::thread producer([&] {
        for (uint32_t k = 0; k < kBatches; ++k) {
            std::memset(host.data(), 0, host.size());
            for (uint32_t i = 0; i < kN; ++i) {
                uint8_t* f = host.data() + (size_t)i * kSlot;
                std::memset(f + 6, 0xff, 6);
                const bool arp = (k & 1u) && i % 5 == 0;
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
            }
            (void)hipMemcpyAsync(d_ring + (size_t)k * kSlot * kN, host.data(), host.size(),
                                 hipMemcpyHostToDevice, ps);
            // the copy stream must not share a hardware queue with the held
            // consumer stream: poll with a deadline instead of blocking
            const auto t0 = std::chrono::steady_clock::now();
            while (hipStreamQuery(ps) == hipErrorNotReady) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                    copy_stuck = true;
                    ingot_gpu_doorbell_ring(db, kBatches);
                    (void)hipStreamSynchronize(ps);
                    return;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            if (k == 0) {
                // the first parse must still be waiting on its doorbell
                std::this_thread::sleep_for(std::chrono::milliseconds(50));
                held = hipEventQuery(done[0]) == hipErrorNotReady;
            }
            ingot_gpu_doorbell_ring(db, k + 1);  // publish slot k
        }
    });
    producer.join();
    ingot_gpu_doorbell_ring(db, kBatches);  // (a consumer never waits past the last slot)
    HIP_OK(hipStreamSynchronize(cs));
    if (copy_stuck) return fail("the producer's copy waited behind the held stream");
    if (!held) return fail("the first parse ran before its doorbell");
    if (*word != kBatches) return fail("doorbell word");

    std::vector<ingot_rec> recs((size_t)kN * kBatches);
    HIP_OK(hipMemcpy(recs.data(), d_rec, sizeof(ingot_rec) * recs.size(),
                     hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < kBatches; ++k) {
        for (uint32_t i = 0; i < kN; ++i) {
            const ingot_rec& r = recs[(size_t)k * kN + i];
            const bool arp = (k & 1u) && i % 5 == 0;
            if (arp) {  // UdpParser: L3 choice has no ARP variant -> Unwanted at "l3"
                if (r.status != INGOT_ERR_UNWANTED || r.err_layer != 1) return fail("arp record");
            } else if (r.status != INGOT_OK || r.l3_kind != INGOT_L3_IPV4 ||
                       r.l4_kind != INGOT_L4_UDP || r.l4_off != 34 || r.payload_off != 42) {
                std::printf("batch %u frame %u: status %u\n", k, i, r.status);
                return fail("udp record");
            }
        }
    }
    for (auto e : done) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(cs);
    (void)hipStreamDestroy(ps);
    (void)hipFree(d_ring);
    (void)hipFree(d_rec);
    ingot_gpu_doorbell_destroy(db);
    ingot_gpu_ctx_destroy(ctx);
    std::printf("doorbell ring: %u batches x %u frames parsed as published, first held: ok\n",
                kBatches, kN);
    return 0;
}
