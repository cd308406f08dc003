// comm.cpp — RCCL (over xGMI) for the multi-GPU path.
//
// The reference has no distribution. Row-sharding A and b across G ranks makes the per-rank
// work A_g x - b_g and A_g^T r_g; the only exchange per gradient is one sum all-reduce of the
// n x l gradient (4 MiB at the north-star size) plus 8-byte all-reduces of the squared
// residual norms the objective and the line-search tests need. x and every row-wise step are
// replicated, and RCCL hands every rank identical sums, so all ranks take identical branches.
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "glx.h"
#include "glx_comm.h"
#include "glx_internal.h"

struct glx_comm {
  ncclComm_t comm;
  int nranks, rank;
};

namespace glx {
void comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st) {
  const ncclDataType_t t = dtype == GLX_F64 ? ncclFloat64 : ncclFloat32;
  const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, t, ncclSum, c->comm, st);
  if (r != ncclSuccess) throw Error{GLX_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r)};
}
}  // namespace glx

extern "C" {

int glx_comm_unique_id(uint8_t id[GLX_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == GLX_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    glx::g_last_error = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return GLX_E_RCCL;
  }
  std::memcpy(id, &u, sizeof(u));
  return GLX_OK;
}

int glx_comm_create(glx_comm** out, const uint8_t id[GLX_COMM_ID_BYTES], int nranks, int rank) {
  if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) {
    glx::g_last_error = "glx_comm_create: bad arguments";
    return GLX_E_INVALID;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
  if (r != ncclSuccess) {
    glx::g_last_error = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    return GLX_E_RCCL;
  }
  *out = new glx_comm{c, nranks, rank};
  return GLX_OK;
}

int glx_comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, void* stream) {
  try {
    glx::comm_allreduce(c, buf, count, dtype, static_cast<hipStream_t>(stream));
    return GLX_OK;
  } catch (const glx::Error& e) {
    glx::g_last_error = e.msg;
    return e.code;
  }
}

void glx_comm_destroy(glx_comm* c) {
  if (!c) return;
  ncclCommDestroy(c->comm);
  delete c;
}

}  // extern "C"
