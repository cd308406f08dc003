// glx_comm.h — RCCL communicator used for row-sharded A (one process per GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct glx_comm;

namespace glx {
// in-place sum all-reduce on `st`; throws glx::Error on failure
void comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st);
// in place over nranks chunks of `count` elements (comm.cpp)
void comm_reduce_scatter(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st);
void comm_all_gather(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st);
void comm_group_begin(glx_comm* c);
void comm_group_end(glx_comm* c);
int comm_rank(const glx_comm* c);
int comm_size(const glx_comm* c);
}  // namespace glx
