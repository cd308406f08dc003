// glx_comm.h — RCCL communicator used for row-sharded A (one process per GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct glx_comm;

namespace glx {
// in-place sum all-reduce on `st`; throws glx::Error on failure
void comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st);
}  // namespace glx
