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

// Two transports behind one handle. RCCL is the product path (one GPU per rank, xGMI). The
// host transport stages each all-reduce through pinned host memory and hands it to a caller
// callback (e.g. torch.distributed over gloo): it exists so that several ranks can share ONE
// GPU and exercise the whole sharded solver on a one-GPU box or in a test, which RCCL refuses
// (one rank per device).
struct glx_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  glx_host_allreduce_fn host_fn = nullptr;
  void* host_user = nullptr;
  void* stage = nullptr;     // pinned staging buffer (host transport)
  size_t stage_bytes = 0;
};

namespace glx {
void comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st) {
  if (c->host_fn == nullptr) {
    const ncclDataType_t t = dtype == GLX_F64 ? ncclFloat64 : ncclFloat32;
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, t, ncclSum, c->comm, st);
    if (r != ncclSuccess) throw Error{GLX_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r)};
    return;
  }
  const size_t bytes = (size_t)count * (dtype == GLX_F64 ? 8 : 4);
  if (bytes > c->stage_bytes) {
    if (c->stage) (void)hipHostFree(c->stage);
    c->stage = nullptr;
    c->stage_bytes = 0;
    if (hipHostMalloc(&c->stage, bytes, hipHostMallocDefault) != hipSuccess)
      throw Error{GLX_E_HIP, "host comm: hipHostMalloc failed"};
    c->stage_bytes = bytes;
  }
  if (hipMemcpyAsync(c->stage, buf, bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    throw Error{GLX_E_HIP, "host comm: device-to-host staging failed"};
  const int rc = c->host_fn(c->stage, count, dtype, c->host_user);
  if (rc != 0) throw Error{GLX_E_RCCL, "host comm: all-reduce callback returned " + std::to_string(rc)};
  if (hipMemcpyAsync(buf, c->stage, bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)   // the staging buffer is reused by the next call
    throw Error{GLX_E_HIP, "host comm: host-to-device staging failed"};
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
  glx_comm* h = new glx_comm;
  h->comm = c;
  h->nranks = nranks;
  h->rank = rank;
  *out = h;
  return GLX_OK;
}

int glx_comm_create_host(glx_comm** out, int nranks, int rank, glx_host_allreduce_fn fn, void* user) {
  if (!out || !fn || nranks < 1 || rank < 0 || rank >= nranks) {
    glx::g_last_error = "glx_comm_create_host: bad arguments";
    return GLX_E_INVALID;
  }
  glx_comm* h = new glx_comm;
  h->nranks = nranks;
  h->rank = rank;
  h->host_fn = fn;
  h->host_user = user;
  *out = h;
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
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->stage) (void)hipHostFree(c->stage);
  delete c;
}

}  // extern "C"
