// comm.cpp — config 5's per-flow histogram reduce behind the C ABI
// (include/ingot_gpu.h: ingot_gpu_comm_*, ingot_gpu_flow_hist_allreduce).
//
// The reference has no collective at all: packets are
// independent and shard by index range; the one exchange of the GPU design is
// the element-wise sum of the per-rank flow histograms, an RCCL all-reduce
// (ncclSum over ncclUint32) over xGMI.  RCCL is opened with dlopen at first
// use, so the parse library loads and runs without it; in a process that
// already holds librccl.so.1 (PyTorch's ProcessGroupNCCL) the same copy is
// shared, never a second one.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <new>

#include "../../include/ingot_gpu.h"

static_assert(NCCL_UNIQUE_ID_BYTES == INGOT_COMM_ID_BYTES, "communicator id size");

struct ingot_gpu_comm {
    ncclComm_t nccl;
    int device, nranks, rank;
    bool owned;  // false: borrowed by ingot_gpu_comm_wrap, never finalized here
};

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommFinalize) finalize = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommCount) count = nullptr;
    decltype(&ncclCommUserRank) user_rank = nullptr;
    decltype(&ncclCommCuDevice) cu_device = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
        r.finalize = (decltype(r.finalize))dlsym(h, "ncclCommFinalize");
        r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
        r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.count = (decltype(r.count))dlsym(h, "ncclCommCount");
        r.user_rank = (decltype(r.user_rank))dlsym(h, "ncclCommUserRank");
        r.cu_device = (decltype(r.cu_device))dlsym(h, "ncclCommCuDevice");
        r.ok = r.get_unique_id && r.init_rank && r.finalize && r.destroy && r.abort &&
               r.all_reduce && r.count && r.user_rank && r.cu_device;
    });
    return r;
}

int set_device(int device) {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return INGOT_GPU_EHIP;
    if (cur != device && hipSetDevice(device) != hipSuccess) return INGOT_GPU_EHIP;
    return INGOT_GPU_SUCCESS;
}

}  // namespace

extern "C" {

int ingot_gpu_comm_unique_id(uint8_t id[INGOT_COMM_ID_BYTES]) {
    if (!id) return INGOT_GPU_EINVAL;
    const Rccl& r = rccl();
    if (!r.ok) return INGOT_GPU_ENODEV;
    ncclUniqueId u;
    if (r.get_unique_id(&u) != ncclSuccess) return INGOT_GPU_ECOMM;
    std::memcpy(id, u.internal, INGOT_COMM_ID_BYTES);
    return INGOT_GPU_SUCCESS;
}

int ingot_gpu_comm_create(ingot_gpu_ctx* ctx, int nranks, int rank,
                          const uint8_t id[INGOT_COMM_ID_BYTES], ingot_gpu_comm** out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return INGOT_GPU_EINVAL;
    *out = nullptr;
    const Rccl& r = rccl();
    if (!r.ok) return INGOT_GPU_ENODEV;
    const int device = ingot_gpu_ctx_device(ctx);
    if (int e = set_device(device)) return e;
    ncclUniqueId u;
    std::memcpy(u.internal, id, INGOT_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    if (r.init_rank(&c, nranks, u, rank) != ncclSuccess) return INGOT_GPU_ECOMM;
    ingot_gpu_comm* comm = new (std::nothrow) ingot_gpu_comm{c, device, nranks, rank, true};
    if (!comm) {
        (void)r.destroy(c);
        return INGOT_GPU_ENOMEM;
    }
    *out = comm;
    return INGOT_GPU_SUCCESS;
}

// The host's own communicator, borrowed: its size, rank and device are
// asked of RCCL, and the device must be the context's.
int ingot_gpu_comm_wrap(ingot_gpu_ctx* ctx, void* nccl_comm, ingot_gpu_comm** out) {
    if (!ctx || !nccl_comm || !out) return INGOT_GPU_EINVAL;
    *out = nullptr;
    const Rccl& r = rccl();
    if (!r.ok) return INGOT_GPU_ENODEV;
    ncclComm_t c = (ncclComm_t)nccl_comm;
    int nranks = 0, rank = -1, device = -1;
    if (r.count(c, &nranks) != ncclSuccess || r.user_rank(c, &rank) != ncclSuccess ||
        r.cu_device(c, &device) != ncclSuccess)
        return INGOT_GPU_ECOMM;
    if (device != ingot_gpu_ctx_device(ctx) || nranks < 1 || rank < 0 || rank >= nranks)
        return INGOT_GPU_EINVAL;
    ingot_gpu_comm* comm = new (std::nothrow) ingot_gpu_comm{c, device, nranks, rank, false};
    if (!comm) return INGOT_GPU_ENOMEM;
    *out = comm;
    return INGOT_GPU_SUCCESS;
}

// Graceful: flush every reduce issued and wait until the communicator is
// quiescent on all ranks (ncclCommFinalize), then free it locally.  A
// borrowed communicator is left to its owner.
int ingot_gpu_comm_destroy(ingot_gpu_comm* comm) {
    if (!comm) return INGOT_GPU_EINVAL;
    if (!comm->owned) {
        delete comm;
        return INGOT_GPU_SUCCESS;
    }
    (void)set_device(comm->device);
    const Rccl& r = rccl();
    const bool ok = r.finalize(comm->nccl) == ncclSuccess;
    const bool freed = r.destroy(comm->nccl) == ncclSuccess;
    delete comm;
    return ok && freed ? INGOT_GPU_SUCCESS : INGOT_GPU_ECOMM;
}

// Local and immediate: reduces still in flight are aborted.
int ingot_gpu_comm_abort(ingot_gpu_comm* comm) {
    if (!comm) return INGOT_GPU_EINVAL;
    if (!comm->owned) {
        delete comm;
        return INGOT_GPU_SUCCESS;
    }
    (void)set_device(comm->device);
    const bool ok = rccl().abort(comm->nccl) == ncclSuccess;
    delete comm;
    return ok ? INGOT_GPU_SUCCESS : INGOT_GPU_ECOMM;
}

int ingot_gpu_comm_size(const ingot_gpu_comm* comm) { return comm ? comm->nranks : INGOT_GPU_EINVAL; }

int ingot_gpu_comm_rank(const ingot_gpu_comm* comm) { return comm ? comm->rank : INGOT_GPU_EINVAL; }

int ingot_gpu_flow_hist_allreduce(ingot_gpu_comm* comm, uint32_t* d_hist, uint32_t bins,
                                  void* stream) {
    if (!comm || !d_hist) return INGOT_GPU_EINVAL;
    if (bins == 0 || (bins & (bins - 1)) != 0 || bins > (1u << 24)) return INGOT_GPU_ERANGE;
    if (int e = set_device(comm->device)) return e;
    return rccl().all_reduce(d_hist, d_hist, bins, ncclUint32, ncclSum, comm->nccl,
                             (hipStream_t)stream) == ncclSuccess
               ? INGOT_GPU_SUCCESS
               : INGOT_GPU_ECOMM;
}

}  // extern "C"
