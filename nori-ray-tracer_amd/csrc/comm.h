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
// Sum `count` floats in place over the communicator on `stream`: into
// rank `root`'s buffer (ncclReduce) or every rank's (root < 0, ncclAllReduce).
void comm_sum(void *comm, float *buf, size_t count, int root, hipStream_t stream);
const char *comm_library_path();  // the librccl that was opened, NULL if none

}  // namespace nori
