// RCCL (over xGMI on one MI355X node) for the per-pair / per-shard result exchange of
// one all-gather of fixed-size records at the end of a sharded run and a
// max-all-reduce of c* when one pair's hypotheses are split across GPUs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstring>

#include "common.h"
#include "ctx.h"

using rs::fail;

static int nccl_fail(ncclResult_t r, const char *what) {
  rs::set_error("%s: %s", what, ncclGetErrorString(r));
  return RS_ECOMM;
}

extern "C" int rs_comm_unique_id(uint8_t *id_out) {
  if (!id_out) return fail(RS_EINVAL, "null pointer");
  static_assert(sizeof(ncclUniqueId) <= RS_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
  std::memset(id_out, 0, RS_COMM_ID_BYTES);
  std::memcpy(id_out, &id, sizeof(id));
  return RS_OK;
}

extern "C" int rs_comm_init(rs_ctx *c, int32_t nranks, int32_t rank, const uint8_t *id) {
  if (!c || !id) return fail(RS_EINVAL, "null pointer");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(RS_EINVAL, "bad rank / nranks");
  if (c->comm) return fail(RS_EINVAL, "communicator already initialised");
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return rs::hip_fail(e, "hipSetDevice");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm;
  ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitRank");
  c->comm = comm;
  return RS_OK;
}

extern "C" int rs_comm_destroy(rs_ctx *c) {
  if (!c) return fail(RS_EINVAL, "null context");
  if (c->comm_buf) (void)hipFree(c->comm_buf);
  c->comm_buf = nullptr;
  c->comm_buf_bytes = 0;
  if (c->comm) {
    (void)ncclCommDestroy(static_cast<ncclComm_t>(c->comm));
    c->comm = nullptr;
  }
  return RS_OK;
}

static int comm_buffer(rs_ctx *c, size_t bytes) {
  if (c->comm_buf_bytes >= bytes) return RS_OK;
  if (c->comm_buf) (void)hipFree(c->comm_buf);
  c->comm_buf = nullptr;
  hipError_t e = hipMalloc(&c->comm_buf, bytes);
  if (e != hipSuccess) return rs::hip_fail(e, "hipMalloc(comm)");
  c->comm_buf_bytes = bytes;
  return RS_OK;
}

extern "C" int rs_comm_allgather(rs_ctx *c, const void *send, void *recv, int64_t bytes) {
  if (!c || !send || !recv) return fail(RS_EINVAL, "null pointer");
  if (!c->comm) return fail(RS_EINVAL, "communicator not initialised");
  if (bytes < 0) return fail(RS_EINVAL, "negative size");
  auto comm = static_cast<ncclComm_t>(c->comm);
  int nranks = 0;
  ncclResult_t r = ncclCommCount(comm, &nranks);
  if (r != ncclSuccess) return nccl_fail(r, "ncclCommCount");
  const size_t b = static_cast<size_t>(bytes);
  int st = comm_buffer(c, b * (static_cast<size_t>(nranks) + 1) + 16);
  if (st) return st;
  char *d_send = static_cast<char *>(c->comm_buf);
  char *d_recv = d_send + b;
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipMemcpyAsync(d_send, send, b, hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) return rs::hip_fail(e, "hipMemcpyAsync");
  r = ncclAllGather(d_send, d_recv, b, ncclChar, comm, c->stream);
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllGather");
  e = hipMemcpyAsync(recv, d_recv, b * nranks, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return rs::hip_fail(e, "allgather D2H");
  return RS_OK;
}

extern "C" int rs_comm_allreduce_max_i64(rs_ctx *c, int64_t *value) {
  if (!c || !value) return fail(RS_EINVAL, "null pointer");
  if (!c->comm) return fail(RS_EINVAL, "communicator not initialised");
  int st = comm_buffer(c, 64);
  if (st) return st;
  auto *d = static_cast<int64_t *>(c->comm_buf);
  hipError_t e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipMemcpyAsync(d, value, 8, hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) return rs::hip_fail(e, "hipMemcpyAsync");
  ncclResult_t r = ncclAllReduce(d, d, 1, ncclInt64, ncclMax, static_cast<ncclComm_t>(c->comm),
                                 c->stream);
  if (r != ncclSuccess) return nccl_fail(r, "ncclAllReduce");
  e = hipMemcpyAsync(value, d, 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return rs::hip_fail(e, "allreduce D2H");
  return RS_OK;
}

// Which RCCL this process runs: ncclGetVersion and the path of the shared object that holds it
// (dladdr).  A process that loaded another librccl.so first (torch's bundled copy, through
// `import torch.distributed`) binds the soname to that one; bench.py reports both.
extern "C" int rs_comm_library(int32_t *version, char *path, int64_t cap) {
  if (!version) return fail(RS_EINVAL, "null pointer");
  int v = 0;
  ncclResult_t r = ncclGetVersion(&v);
  if (r != ncclSuccess) return nccl_fail(r, "ncclGetVersion");
  *version = v;
  if (path && cap > 0) {
    Dl_info info{};
    const char *p = dladdr(reinterpret_cast<void *>(&ncclGetVersion), &info) && info.dli_fname
                        ? info.dli_fname
                        : "";
    std::strncpy(path, p, static_cast<size_t>(cap - 1));
    path[cap - 1] = '\0';
  }
  return RS_OK;
}
