// comm.cpp — RCCL (over xGMI) for the multi-GPU path.
//
// The reference has no distribution. Row-sharding A and b across G ranks makes the per-rank
// work A_g x - b_g and A_g^T r_g. Two schedules (solver.cpp): the all-reduce schedule sums the
// n x l gradient on every rank (4 MiB at the north-star size) and replicates the row-wise step;
// the row-sharded schedule (round 5) reduce-scatters the gradient, runs the prox / trial on this
// rank's n / G rows and all-gathers the new iterate's rows with every rank's partial sums, which
// each rank then combines in rank order. Either way every rank holds identical values, so all
// ranks take identical branches.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
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
  // progress record (round 6): collectives issued on the stream, collectives the host transport
  // completed, the kind of the last one issued (1 all-reduce, 2 reduce-scatter, 3 all-gather), and
  // whether the communicator was aborted. Atomics: a watchdog thread reads them
  // (glx_comm_progress) while the solver thread issues.
  std::atomic<int64_t> issued{0}, host_done{0};
  std::atomic<int> last_kind{0};
  std::atomic<int> aborted{0};
};

namespace glx {
static void stage_reserve(glx_comm* c, size_t bytes) {
  if (bytes > c->stage_bytes) {
    if (c->stage) (void)hipHostFree(c->stage);
    c->stage = nullptr;
    c->stage_bytes = 0;
    if (hipHostMalloc(&c->stage, bytes, hipHostMallocDefault) != hipSuccess)
      throw Error{GLX_E_HIP, "host comm: hipHostMalloc failed"};
    c->stage_bytes = bytes;
  }
}
static void rccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw Error{GLX_E_RCCL, std::string(what) + ": " + ncclGetErrorString(r)};
}
static ncclDataType_t rccl_type(int dtype) { return dtype == GLX_F64 ? ncclFloat64 : ncclFloat32; }

void comm_allreduce(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st) {
  c->issued.fetch_add(1);
  c->last_kind.store(1);
  if (c->host_fn == nullptr) {
    rccl_check(ncclAllReduce(buf, buf, (size_t)count, rccl_type(dtype), ncclSum, c->comm, st), "ncclAllReduce");
    return;
  }
  const size_t bytes = (size_t)count * (dtype == GLX_F64 ? 8 : 4);
  stage_reserve(c, bytes);
  if (hipMemcpyAsync(c->stage, buf, bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    throw Error{GLX_E_HIP, "host comm: device-to-host staging failed"};
  const int rc = c->host_fn(c->stage, count, dtype, c->host_user);
  if (rc != 0) throw Error{GLX_E_RCCL, "host comm: all-reduce callback returned " + std::to_string(rc)};
  if (hipMemcpyAsync(buf, c->stage, bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)   // the staging buffer is reused by the next call
    throw Error{GLX_E_HIP, "host comm: host-to-device staging failed"};
  c->host_done.fetch_add(1);
}

// In place: buf holds nranks chunks of `count` elements; chunk `rank` receives the sum of every
// rank's chunk `rank` (the others are left undefined). Host transport: a full all-reduce.
void comm_reduce_scatter(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st) {
  if (c->host_fn == nullptr) {
    c->issued.fetch_add(1);
    c->last_kind.store(2);
    const size_t es = dtype == GLX_F64 ? 8 : 4;
    void* own = static_cast<char*>(buf) + (size_t)c->rank * (size_t)count * es;
    rccl_check(ncclReduceScatter(buf, own, (size_t)count, rccl_type(dtype), ncclSum, c->comm, st),
               "ncclReduceScatter");
    return;
  }
  comm_allreduce(c, buf, count * c->nranks, dtype, st);
}

// In place: chunk `rank` of buf (count elements) is sent, every chunk is received. Host
// transport: the other chunks are filled with -0.0 and summed, which is exact (x + (-0) = x for
// every x, +0 and -0 included), so the gathered bits are the senders' bits.
void comm_all_gather(glx_comm* c, void* buf, int64_t count, int dtype, hipStream_t st) {
  const size_t es = dtype == GLX_F64 ? 8 : 4;
  char* own = static_cast<char*>(buf) + (size_t)c->rank * (size_t)count * es;
  c->issued.fetch_add(1);
  c->last_kind.store(3);
  if (c->host_fn == nullptr) {
    rccl_check(ncclAllGather(own, buf, (size_t)count, rccl_type(dtype), c->comm, st), "ncclAllGather");
    return;
  }
  const size_t chunk = (size_t)count * es, bytes = chunk * (size_t)c->nranks;
  stage_reserve(c, bytes);
  if (hipMemcpyAsync(static_cast<char*>(c->stage) + (size_t)c->rank * chunk, own, chunk,
                     hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    throw Error{GLX_E_HIP, "host comm: device-to-host staging failed"};
  for (int r = 0; r < c->nranks; ++r) {
    if (r == c->rank) continue;
    char* p = static_cast<char*>(c->stage) + (size_t)r * chunk;
    if (dtype == GLX_F64) std::fill_n(reinterpret_cast<double*>(p), count, -0.0);
    else std::fill_n(reinterpret_cast<float*>(p), count, -0.0f);
  }
  const int rc = c->host_fn(c->stage, count * c->nranks, dtype, c->host_user);
  if (rc != 0) throw Error{GLX_E_RCCL, "host comm: all-gather callback returned " + std::to_string(rc)};
  if (hipMemcpyAsync(buf, c->stage, bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    throw Error{GLX_E_HIP, "host comm: host-to-device staging failed"};
  c->host_done.fetch_add(1);
}

// RCCL group: the collectives issued in between go out as one launch (no-op for the host
// transport, whose calls complete one by one)
void comm_group_begin(glx_comm* c) {
  if (c->host_fn == nullptr) rccl_check(ncclGroupStart(), "ncclGroupStart");
}
void comm_group_end(glx_comm* c) {
  if (c->host_fn == nullptr) rccl_check(ncclGroupEnd(), "ncclGroupEnd");
}
int comm_rank(const glx_comm* c) { return c->rank; }
int comm_size(const glx_comm* c) { return c->nranks; }
int comm_async_error(glx_comm* c) {
  if (c->host_fn != nullptr || c->comm == nullptr || c->aborted.load()) return 0;
  ncclResult_t a = ncclSuccess;
  if (ncclCommGetAsyncError(c->comm, &a) != ncclSuccess) return (int)ncclInternalError;
  return a == ncclInProgress ? 0 : (int)a;
}
void comm_abort(glx_comm* c) {
  if (c->host_fn == nullptr && c->comm != nullptr && c->aborted.exchange(1) == 0) (void)ncclCommAbort(c->comm);
}
bool comm_is_rccl(const glx_comm* c) { return c->host_fn == nullptr; }
int64_t comm_issued(const glx_comm* c) { return c->issued.load(); }
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

int glx_comm_reduce_scatter(glx_comm* c, void* buf, int64_t count, int dtype, void* stream) {
  try {
    glx::comm_reduce_scatter(c, buf, count, dtype, static_cast<hipStream_t>(stream));
    return GLX_OK;
  } catch (const glx::Error& e) {
    glx::g_last_error = e.msg;
    return e.code;
  }
}

int glx_comm_all_gather(glx_comm* c, void* buf, int64_t count, int dtype, void* stream) {
  try {
    glx::comm_all_gather(c, buf, count, dtype, static_cast<hipStream_t>(stream));
    return GLX_OK;
  } catch (const glx::Error& e) {
    glx::g_last_error = e.msg;
    return e.code;
  }
}

int glx_comm_progress(glx_comm* c, int64_t out[4]) {
  if (!c || !out) {
    glx::g_last_error = "glx_comm_progress: null argument";
    return GLX_E_INVALID;
  }
  out[0] = c->issued.load();
  out[1] = c->host_fn != nullptr ? c->host_done.load() : -1;
  out[2] = c->last_kind.load();
  out[3] = c->aborted.load() ? -1 : glx::comm_async_error(c);
  return GLX_OK;
}

void glx_comm_destroy(glx_comm* c) {
  if (!c) return;
  if (c->comm) {
    if (c->aborted.load() == 0) ncclCommDestroy(c->comm);   // an aborted one is already freed
  }
  if (c->stage) (void)hipHostFree(c->stage);
  delete c;
}

}  // extern "C"
