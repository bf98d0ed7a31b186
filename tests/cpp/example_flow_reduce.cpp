// example_flow_reduce.cpp — config 5's step from a host that binds only the C
// ABI (no Python, no PyTorch: RCCL is the system librccl.so.1 the library
// opens itself).  One rank of the job: generate this rank's C5 frames, parse +
// hash + count them (ingot_gpu_flow_hist_ws), then sum the histogram across
// the job's ranks (ingot_gpu_flow_hist_allreduce over a communicator made
// from rank 0's id).  On the one-GPU test box the job has one rank; checks:
// the reduced histogram equals a host bincount of the per-packet flow bins,
// its total equals the packets that parsed Ok with an L3 layer (ingot_gpu_parse
// records of the same frames), the ABI's argument errors, and the same
// reduce over a communicator the host made itself and lent to the library
// (ingot_gpu_comm_wrap).
//
// example_flow_reduce NRANKS RANK DIR: rank RANK of an NRANKS-rank job over
// contiguous shards of 262,144 frames.  Rank 0 writes the communicator id to
// DIR/id (the host's control channel here is a file), the others wait for it;
// every rank writes its reduced histogram to DIR/hist.RANK and its own
// bincount of its flow bins to DIR/local.RANK, which the test sums.
// Run on the GPU by tests/test_cpp_mirror.py.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ingot_amd.hpp"
#include "ingot_gpu.h"
#include "ingot_pktgen.h"

static int fail(const char* what, int rc = 0) {
    std::printf("FAIL %s (%d: %s)\n", what, rc, ingot_gpu_strerror(rc));
    return 1;
}

static bool write_file(const std::string& path, const void* p, size_t bytes) {
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(p, 1, bytes, f) == bytes;
    return (std::fclose(f) == 0) && ok && std::rename(tmp.c_str(), path.c_str()) == 0;
}

static bool read_file(const std::string& path, void* p, size_t bytes, double wait_s) {
    const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(wait_s);
    for (;;) {
        if (FILE* f = std::fopen(path.c_str(), "rb")) {
            const bool ok = std::fread(p, 1, bytes, f) == bytes;
            std::fclose(f);
            return ok;
        }
        if (std::chrono::steady_clock::now() > end) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

int main(int argc, char** argv) {
    const int nranks = argc > 3 ? std::atoi(argv[1]) : 1;
    const int rank = argc > 3 ? std::atoi(argv[2]) : 0;
    const std::string dir = argc > 3 ? argv[3] : "";
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail("arguments", INGOT_GPU_EINVAL);
    const bool job = nranks > 1;
    const uint64_t n = job ? (1u << 18) : (1u << 20);
    const uint64_t first = (uint64_t)rank * n;
    const uint32_t bins = 1u << 16;
    ingot_gpu_ctx* ctx = nullptr;
    if (int rc = ingot_gpu_ctx_create(0, &ctx)) return fail("ctx_create", rc);
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return fail("stream");

    // this rank's frames: lengths on the device, offsets by a host prefix sum
    uint16_t* d_len;
    uint64_t* d_off;
    if (hipMalloc(&d_len, n * 2) != hipSuccess || hipMalloc(&d_off, n * 8) != hipSuccess)
        return fail("alloc");
    if (int rc = ingot_pktgen_lengths(INGOT_GEN_FLOWS, INGOT_GEN_SEED, first, n, d_len, s))
        return fail("pktgen_lengths", rc);
    std::vector<uint16_t> len(n);
    std::vector<uint64_t> off(n);
    if (hipMemcpyAsync(len.data(), d_len, n * 2, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail("lengths D2H");
    uint64_t bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        off[i] = bytes;
        bytes += len[i];
    }
    bytes += 64;
    uint8_t* d_arena;
    if (hipMalloc(&d_arena, bytes) != hipSuccess) return fail("arena");
    if (hipMemcpyAsync(d_off, off.data(), n * 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return fail("offsets H2D");
    if (int rc = ingot_pktgen_fill(INGOT_GEN_FLOWS, INGOT_GEN_SEED, first, n, d_off, 0, d_len,
                                   d_arena, bytes, s))
        return fail("pktgen_fill", rc);

    // the step: parse + hash + histogram, then the reduce, one stream
    uint32_t *d_flow, *d_hist;
    ingot_rec* d_rec;
    const size_t wb = ingot_gpu_flow_hist_workspace_size(n, bins);
    void* d_work = nullptr;
    if (hipMalloc(&d_flow, n * 4) != hipSuccess || hipMalloc(&d_hist, bins * 4) != hipSuccess ||
        hipMalloc(&d_rec, n * sizeof(ingot_rec)) != hipSuccess ||
        (wb && hipMalloc(&d_work, wb) != hipSuccess))
        return fail("step buffers");
    uint8_t id[INGOT_COMM_ID_BYTES];
    if (rank == 0) {
        if (int rc = ingot_gpu_comm_unique_id(id)) return fail("comm_unique_id", rc);
        if (job && !write_file(dir + "/id", id, sizeof id)) return fail("write id");
    } else if (!read_file(dir + "/id", id, sizeof id, 60.0)) {
        return fail("read id");
    }
    ingot_gpu_comm* comm = nullptr;
    if (int rc = ingot_gpu_comm_create(ctx, nranks, rank, id, &comm))
        return fail("comm_create", rc);
    if (ingot_gpu_comm_size(comm) != nranks || ingot_gpu_comm_rank(comm) != rank)
        return fail("comm size");
    if (hipMemsetAsync(d_hist, 0, bins * 4, s) != hipSuccess) return fail("memset");
    const int chain = INGOT_CHAIN_VLAN_ULP;
    if (int rc = ingot_gpu_flow_hist_ws(ctx, d_arena, d_off, d_len, 0, n, chain, nullptr, bins,
                                        d_flow, nullptr, d_hist, d_work, wb, s))
        return fail("flow_hist_ws", rc);
    if (int rc = ingot_gpu_flow_hist_allreduce(comm, d_hist, bins, s))
        return fail("flow_hist_allreduce", rc);
    if (int rc = ingot_gpu_parse(ctx, d_arena, d_off, d_len, n, chain, d_rec, s))
        return fail("parse", rc);
    std::vector<uint32_t> flow(n), hist(bins);
    std::vector<ingot_rec> rec(n);
    if (hipMemcpyAsync(flow.data(), d_flow, n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(hist.data(), d_hist, bins * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(rec.data(), d_rec, n * sizeof(ingot_rec), hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return fail("results D2H");

    std::vector<uint32_t> want(bins, 0);
    uint64_t counted = 0, ok_l3 = 0, total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (flow[i] != INGOT_FLOW_NONE) {
            ++want[flow[i]];
            ++counted;
        }
        ok_l3 += rec[i].status == INGOT_OK && rec[i].l3_kind != INGOT_L3_NONE;
    }
    if (job) {  // the sums over the ranks are the test's to check
        const std::string r = std::to_string(rank);
        if (!write_file(dir + "/hist." + r, hist.data(), bins * 4) ||
            !write_file(dir + "/local." + r, want.data(), bins * 4))
            return fail("write results");
        std::printf("rank %d of %d: %llu packets counted, %llu Ok with an L3 layer\n", rank,
                    nranks, (unsigned long long)counted, (unsigned long long)ok_l3);
        const int rc = ingot_gpu_comm_destroy(comm);  // every rank: graceful
        ingot_gpu_ctx_destroy(ctx);
        return rc ? fail("comm_destroy", rc) : 0;
    }
    uint64_t bad = 0;
    for (uint32_t b = 0; b < bins; ++b) {
        bad += hist[b] != want[b];
        total += hist[b];
    }
    bad += total != counted || counted != ok_l3 || counted == 0;
    // argument errors: bins not a power of two, no histogram, no communicator
    bad += ingot_gpu_flow_hist_allreduce(comm, d_hist, 1000, s) != INGOT_GPU_ERANGE;
    bad += ingot_gpu_flow_hist_allreduce(comm, nullptr, bins, s) != INGOT_GPU_EINVAL;
    bad += ingot_gpu_flow_hist_allreduce(nullptr, d_hist, bins, s) != INGOT_GPU_EINVAL;
    std::printf("rccl reduce over %d rank(s): %llu packets counted, %llu Ok with an L3 layer, "
                "histogram total %llu\n",
                ingot_gpu_comm_size(comm), (unsigned long long)counted,
                (unsigned long long)ok_l3, (unsigned long long)total);
    bad += ingot_gpu_comm_destroy(comm) != INGOT_GPU_SUCCESS;
    {  // the same reduce through the C++ mirror (include/ingot_amd.hpp)
        ingot::gpu::Context cctx(0);
        ingot::gpu::Comm c(cctx, 1, 0, ingot::gpu::Comm::unique_id());
        c.allreduce_hist(d_hist, bins, s);
        std::vector<uint32_t> again(bins);
        if (hipMemcpyAsync(again.data(), d_hist, bins * 4, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return fail("mirror D2H");
        bad += c.size() != 1 || again != hist;
    }
    {  // a communicator the host made itself, lent to the library
        ncclComm_t own = nullptr;
        int dev = 0;
        if (ncclCommInitAll(&own, 1, &dev) != ncclSuccess) return fail("ncclCommInitAll");
        ingot_gpu_comm* w = nullptr;
        if (int rc = ingot_gpu_comm_wrap(ctx, own, &w)) return fail("comm_wrap", rc);
        bad += ingot_gpu_comm_size(w) != 1 || ingot_gpu_comm_rank(w) != 0;
        bad += ingot_gpu_comm_wrap(ctx, nullptr, &w) != INGOT_GPU_EINVAL;
        std::vector<uint32_t> again(bins);
        if (int rc = ingot_gpu_flow_hist_allreduce(w, d_hist, bins, s))
            return fail("allreduce over the lent communicator", rc);
        bad += ingot_gpu_comm_destroy(w) != INGOT_GPU_SUCCESS;  // the handle only
        // the host's communicator outlives the handle and still reduces
        if (ncclAllReduce(d_hist, d_hist, bins, ncclUint32, ncclSum, own, s) != ncclSuccess)
            return fail("ncclAllReduce after the handle");
        if (hipMemcpyAsync(again.data(), d_hist, bins * 4, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return fail("lent D2H");
        bad += again != hist;
        bad += ncclCommDestroy(own) != ncclSuccess;
        std::printf("lent communicator: reduce ok\n");
    }
    (void)hipFree(d_work);
    (void)hipFree(d_rec);
    (void)hipFree(d_hist);
    (void)hipFree(d_flow);
    (void)hipFree(d_arena);
    (void)hipFree(d_off);
    (void)hipFree(d_len);
    (void)hipStreamDestroy(s);
    ingot_gpu_ctx_destroy(ctx);
    std::printf("%llu mismatches\n", (unsigned long long)bad);
    return bad ? 1 : 0;
}
