// comm.h -- internal interface of comm.cpp (RCCL film exchange), used by
// runtime.hip's nori_gpu_comm_* / nori_gpu_render_sharded entry points.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "host_scene.h"

namespace nori {

void comm_unique_id(unsigned char *id);                              // ncclGetUniqueId
void *comm_create(const unsigned char *id, int nranks, int rank, int device);  // ncclCommInitRank
void comm_destroy(void *comm);
void comm_abort(void *comm);  // ncclCommAbort: peers' pending collectives fail instead of hanging
// Wait for `stream` (its RCCL work included) with a watchdog: an asynchronous
// RCCL error or no completion within timeout_s aborts the communicator
// (aborted = true) and throws NoriException(NORI_ERR_HIP).
void comm_wait(void *comm, hipStream_t stream, double timeout_s, bool &aborted);
// Max of `value` over the ranks (ncclAllReduce of one int through the device
// word `dev` and the pinned host word `pinned`), waited for with comm_wait.
int comm_max_int(void *comm, int *dev, int *pinned, int value, hipStream_t stream, double timeout_s, bool &aborted);
// Sum `count` floats in place over the communicator on `stream`: into
// rank `root`'s buffer (ncclReduce) or every rank's (root < 0, ncclAllReduce).
void comm_sum(void *comm, float *buf, size_t count, int root, hipStream_t stream);
const char *comm_library_path();  // the librccl that was opened, NULL if none

}  // namespace nori
