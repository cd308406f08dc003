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
// Round 6 (diagnosable multi-rank runs): RCCL's asynchronous error state (ncclCommGetAsyncError;
// 0 = none, the host transport always 0), aborting the communicator (ncclCommAbort: RCCL kernels
// blocked on a peer return, so the stream drains), and whether this is the RCCL transport
int comm_async_error(glx_comm* c);
void comm_abort(glx_comm* c);
bool comm_is_rccl(const glx_comm* c);
// collectives issued / completed by the host transport so far (a progress record for watchdogs)
int64_t comm_issued(const glx_comm* c);
}  // namespace glx
