// comm.cpp -- the multi-GPU film exchange of libnori_gpu: an RCCL
// communicator per process (one process per GPU) and the film sum over it.
//
// The reference renders one frame on one host: every 32x32 block's
// ImageBlock is merged into the full image under a mutex
// (ImageBlock::put(block), block.cpp:124-133).  Across GPUs the same merge is
// a sum of RGBW films -- neighbouring blocks' borders overlap, so it is a
// reduction, not a gather -- done with one ncclReduce / ncclAllReduce over
// xGMI on the render context's stream.
//
// RCCL is opened at run time (dlopen), from the directory of the HIP runtime
// already mapped into the process: a process that also runs PyTorch-ROCm
// (which ships its own libamdhip64 / librccl) must not load a second copy of
// either.  The library itself loads and runs single-GPU renders without RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>

#include "comm.h"

namespace nori {
namespace {

struct RcclApi {
    void *handle = nullptr;
    std::string path, error;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
    ncclResult_t (*async_error)(ncclComm_t, ncclResult_t *) = nullptr;
    ncclResult_t (*reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                           hipStream_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

// Directory of the libamdhip64 this process uses (where hipGetDeviceCount resolved).
std::string hip_runtime_dir() {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void *>(static_cast<hipError_t (*)(int *)>(&hipGetDeviceCount)), &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t s = p.find_last_of('/');
        if (s != std::string::npos) return p.substr(0, s);
    }
    return {};
}

RcclApi &rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        const std::string dir = hip_runtime_dir();
        const std::string candidates[] = {dir.empty() ? "" : dir + "/librccl.so.1", dir.empty() ? "" : dir + "/librccl.so",
                                          "librccl.so.1"};
        for (const std::string &c : candidates) {
            if (c.empty()) continue;
            api.handle = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (api.handle) {
                api.path = c;
                break;
            }
        }
        if (!api.handle) {
            api.error = std::string("RCCL not found next to the HIP runtime (") + dir + ") nor as librccl.so.1: " + dlerror();
            return;
        }
        auto sym = [&](const char *name) {
            void *f = dlsym(api.handle, name);
            if (!f && api.error.empty()) api.error = std::string("RCCL symbol missing: ") + name;
            return f;
        };
        api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(sym("ncclGetUniqueId"));
        api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(sym("ncclCommInitRank"));
        api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(sym("ncclCommDestroy"));
        api.comm_abort = reinterpret_cast<decltype(api.comm_abort)>(sym("ncclCommAbort"));
        api.async_error = reinterpret_cast<decltype(api.async_error)>(sym("ncclCommGetAsyncError"));
        api.reduce = reinterpret_cast<decltype(api.reduce)>(sym("ncclReduce"));
        api.all_reduce = reinterpret_cast<decltype(api.all_reduce)>(sym("ncclAllReduce"));
        api.error_string = reinterpret_cast<decltype(api.error_string)>(sym("ncclGetErrorString"));
    });
    if (!api.error.empty()) throw NoriException(NORI_ERR_UNSUPPORTED, api.error);
    return api;
}

void check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) {
        const char *s = rccl().error_string ? rccl().error_string(r) : "?";
        throw NoriException(NORI_ERR_HIP, std::string(what) + ": " + s);
    }
}

}  // namespace

void comm_unique_id(unsigned char *id) {
    static_assert(sizeof(ncclUniqueId) == NORI_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    check(rccl().get_unique_id(&u), "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
}

void *comm_create(const unsigned char *id, int nranks, int rank, int device) {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw NoriException(NORI_ERR_INVALID, "comm: rank out of range");
    if (hipSetDevice(device) != hipSuccess) throw NoriException(NORI_ERR_HIP, "comm: hipSetDevice failed");
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    check(rccl().comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank");
    return c;
}

void comm_destroy(void *c) {
    if (c) (void)rccl().comm_destroy(static_cast<ncclComm_t>(c));
}

void comm_abort(void *c) {
    if (c) (void)rccl().comm_abort(static_cast<ncclComm_t>(c));
}

// hipStreamSynchronize with a watchdog: a peer that died (or never reaches
// the collective) would leave this rank blocked forever in the RCCL kernel.
// Poll the stream; an asynchronous RCCL error or `timeout_s` without
// completion aborts the communicator (ncclCommAbort also releases the kernel
// waiting on the peer) and throws.
void comm_wait(void *c, hipStream_t stream, double timeout_s, bool &aborted) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int spin = 0;; ++spin) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) {
            comm_abort(c);
            aborted = true;
            throw NoriException(NORI_ERR_HIP, std::string("film exchange: ") + hipGetErrorString(e));
        }
        ncclResult_t ae = ncclSuccess;
        if (rccl().async_error(static_cast<ncclComm_t>(c), &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress) {
            comm_abort(c);
            aborted = true;
            throw NoriException(NORI_ERR_HIP, std::string("film exchange: RCCL error ") + rccl().error_string(ae));
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > timeout_s) {
            comm_abort(c);
            aborted = true;
            throw NoriException(NORI_ERR_HIP, "film exchange: no completion within " + std::to_string(timeout_s) +
                                                  " s (a peer rank failed or never joined); communicator aborted");
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

int comm_max_int(void *c, int *dev, int *pinned, int value, hipStream_t stream, double timeout_s, bool &aborted) {
    *pinned = value;
    if (hipMemcpyAsync(dev, pinned, sizeof(int), hipMemcpyHostToDevice, stream) != hipSuccess)
        throw NoriException(NORI_ERR_HIP, "status exchange: copy failed");
    check(rccl().all_reduce(dev, dev, 1, ncclInt32, ncclMax, static_cast<ncclComm_t>(c), stream), "ncclAllReduce");
    if (hipMemcpyAsync(pinned, dev, sizeof(int), hipMemcpyDeviceToHost, stream) != hipSuccess)
        throw NoriException(NORI_ERR_HIP, "status exchange: copy failed");
    comm_wait(c, stream, timeout_s, aborted);
    return *pinned;
}

void comm_sum(void *c, float *buf, size_t count, int root, hipStream_t stream) {
    if (root < 0)
        check(rccl().all_reduce(buf, buf, count, ncclFloat32, ncclSum, static_cast<ncclComm_t>(c), stream),
              "ncclAllReduce");
    else
        check(rccl().reduce(buf, buf, count, ncclFloat32, ncclSum, root, static_cast<ncclComm_t>(c), stream),
              "ncclReduce");
}

const char *comm_library_path() {
    try {
        return rccl().path.c_str();
    } catch (const NoriException &) {
        return nullptr;
    }
}

}  // namespace nori
