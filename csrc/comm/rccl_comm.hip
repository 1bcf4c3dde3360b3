// Native RCCL communicator: the C API (rccl.h) on explicit HIP streams.
//
// the reference's collectives run through ProcessGroupNCCL
// (models/comm_ops.py:26,39,59,74, layers.py:38,83,116); here a communicator is created
// directly from an ncclUniqueId (exchanged over the c10d store by the Python side,
// parallel/rccl.py) and every collective is enqueued on the HIP stream the caller names —
// no work objects, no watchdog thread, capturable in a HIP graph.
//
// Linked against the librccl.so that PyTorch itself loads (torch/lib, build_ext.py), so the
// process holds one RCCL instance whichever path opens a communicator.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

namespace {
thread_local char g_err[512] = {0};

int fail(const char* what, ncclResult_t r) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, ncclGetErrorString(r));
  return (int)r;
}
}  // namespace

extern "C" const char* dpfs_rccl_last_error() { return g_err; }

extern "C" int dpfs_rccl_id_bytes() { return (int)sizeof(ncclUniqueId); }

extern "C" int dpfs_rccl_unique_id(void* out) {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail("ncclGetUniqueId", r);
  memcpy(out, &id, sizeof(id));
  return 0;
}

// Blocks until all `nranks` ranks have called it with the same id (on their own devices).
extern "C" int dpfs_rccl_init(const void* id_bytes, int nranks, int rank, void** comm_out) {
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  ncclComm_t c = nullptr;
  ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  if (r != ncclSuccess) return fail("ncclCommInitRank", r);
  *comm_out = (void*)c;
  return 0;
}

extern "C" int dpfs_rccl_destroy(void* comm) {
  ncclResult_t r = ncclCommDestroy((ncclComm_t)comm);
  return r == ncclSuccess ? 0 : fail("ncclCommDestroy", r);
}

extern "C" int dpfs_rccl_async_error(void* comm) {
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &e);
  if (r != ncclSuccess) return fail("ncclCommGetAsyncError", r);
  return e == ncclSuccess ? 0 : fail("async", e);
}

// op: 0 sum, 1 prod, 2 max, 3 min, 4 avg; dtype: ncclDataType_t value.
extern "C" int dpfs_rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                                    hipStream_t s) {
  ncclResult_t r = ncclAllReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, (ncclComm_t)comm, s);
  return r == ncclSuccess ? 0 : fail("ncclAllReduce", r);
}

extern "C" int dpfs_rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t recvcount, int dtype, int op,
                                        hipStream_t s) {
  ncclResult_t r =
      ncclReduceScatter(send, recv, recvcount, (ncclDataType_t)dtype, (ncclRedOp_t)op, (ncclComm_t)comm, s);
  return r == ncclSuccess ? 0 : fail("ncclReduceScatter", r);
}

extern "C" int dpfs_rccl_all_gather(void* comm, const void* send, void* recv, size_t sendcount, int dtype,
                                    hipStream_t s) {
  ncclResult_t r = ncclAllGather(send, recv, sendcount, (ncclDataType_t)dtype, (ncclComm_t)comm, s);
  return r == ncclSuccess ? 0 : fail("ncclAllGather", r);
}

extern "C" int dpfs_rccl_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                                   hipStream_t s) {
  ncclResult_t r = ncclBroadcast(send, recv, count, (ncclDataType_t)dtype, root, (ncclComm_t)comm, s);
  return r == ncclSuccess ? 0 : fail("ncclBroadcast", r);
}

// Several collectives as one RCCL group (one fused launch when RCCL can).
extern "C" int dpfs_rccl_group_start() { return ncclGroupStart() == ncclSuccess ? 0 : 1; }
extern "C" int dpfs_rccl_group_end() {
  ncclResult_t r = ncclGroupEnd();
  return r == ncclSuccess ? 0 : fail("ncclGroupEnd", r);
}
