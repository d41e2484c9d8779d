// RCCL communicator: the framework's GPU collective backend.
//
// Reference: the only collectives are the ones torch.nn.DataParallel issues internally -- broadcast of
// every parameter on each forward, NCCL reduce of the gradients to GPU0 once per backward() -- from a
// single process (Runner_P128_QuantumNAT_onchipQNN.py:135-153).
//
// Here: one process per MI355X, one RCCL communicator per process, every collective stream-ordered on a
// stream the CALLER chooses.  There is no progress/watchdog thread and no per-collective event: a
// collective is one RCCL kernel on that stream, so it is captured into a HIP graph like any other kernel
// and ordered against the step's compute by the graph's own edges.  (torch.distributed's ProcessGroupNCCL
// adds a watchdog thread that polls an end event per collective; a poll that lands while ANOTHER thread
// captures a graph fails under HIP's global capture bookkeeping and aborts the process --
// docs/CONCURRENCY.md, "captured collectives".)
//
// RCCL is not linked at build time: qd_comm_load() binds the librccl the process already uses (torch's
// copy), so there is exactly one RCCL -- and one HIP runtime -- per process.
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#define QD_API extern "C" __attribute__((visibility("default")))

namespace {

struct RcclApi {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                 hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

RcclApi g_api;

template <typename F>
bool bind(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g_api.handle, name));
  return f != nullptr;
}

// status codes returned to Python: >= 0 an ncclResult_t, or one of these
constexpr int kNotLoaded = -1;
constexpr int kBadArg = -2;

// the framework's dtype / op codes (parallel/comm.py mirrors them)
bool to_dtype(int code, ncclDataType_t* t) {
  switch (code) {
    case 0: *t = ncclFloat32; return true;
    case 1: *t = ncclBfloat16; return true;
    case 2: *t = ncclFloat64; return true;
    case 3: *t = ncclInt32; return true;
    case 4: *t = ncclInt64; return true;
    case 5: *t = ncclUint8; return true;
    default: return false;
  }
}

bool to_op(int code, ncclRedOp_t* op) {
  switch (code) {
    case 0: *op = ncclSum; return true;
    case 1: *op = ncclMax; return true;
    case 2: *op = ncclMin; return true;
    default: return false;
  }
}

}  // namespace

// Bind the RCCL entry points from `path` (the librccl already mapped into the process: RTLD_NOLOAD first,
// so a second copy is never loaded beside torch's).  Returns 0, or kNotLoaded when a symbol is missing.
QD_API int qd_comm_load(const char* path) {
  if (g_api.handle != nullptr) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
  if (h == nullptr) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (h == nullptr) return kNotLoaded;
  g_api.handle = h;
  bool ok = bind(g_api.get_unique_id, "ncclGetUniqueId") && bind(g_api.comm_init_rank, "ncclCommInitRank") &&
            bind(g_api.comm_destroy, "ncclCommDestroy") && bind(g_api.comm_abort, "ncclCommAbort") &&
            bind(g_api.comm_async_error, "ncclCommGetAsyncError") && bind(g_api.comm_count, "ncclCommCount") &&
            bind(g_api.all_reduce, "ncclAllReduce") && bind(g_api.reduce_scatter, "ncclReduceScatter") &&
            bind(g_api.all_gather, "ncclAllGather") && bind(g_api.broadcast, "ncclBroadcast") &&
            bind(g_api.group_start, "ncclGroupStart") && bind(g_api.group_end, "ncclGroupEnd") &&
            bind(g_api.get_version, "ncclGetVersion") && bind(g_api.error_string, "ncclGetErrorString");
  if (!ok) {
    g_api = RcclApi{};
    return kNotLoaded;
  }
  return 0;
}

QD_API int qd_comm_version(int* v) {
  if (g_api.get_version == nullptr) return kNotLoaded;
  return (int)g_api.get_version(v);
}

QD_API const char* qd_comm_error_string(int status) {
  if (status == kNotLoaded) return "RCCL not loaded (qd_comm_load)";
  if (status == kBadArg) return "invalid dtype / op / argument";
  if (g_api.error_string == nullptr) return "RCCL not loaded";
  return g_api.error_string((ncclResult_t)status);
}

// rank 0 draws the communicator id; the caller distributes the NCCL_UNIQUE_ID_BYTES bytes to every rank
QD_API int qd_comm_unique_id(uint8_t* out, int nbytes) {
  if (g_api.get_unique_id == nullptr) return kNotLoaded;
  if (nbytes != NCCL_UNIQUE_ID_BYTES) return kBadArg;
  ncclUniqueId id;
  ncclResult_t r = g_api.get_unique_id(&id);
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return (int)r;
}

QD_API int qd_comm_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

// collective init of one rank on the CURRENT HIP device (the caller sets it first)
QD_API int qd_comm_init(void** comm, int nranks, const uint8_t* id_bytes, int rank) {
  if (g_api.comm_init_rank == nullptr) return kNotLoaded;
  if (nranks < 1 || rank < 0 || rank >= nranks) return kBadArg;
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  ncclResult_t r = g_api.comm_init_rank(&c, nranks, id, rank);
  *comm = (void*)c;
  return (int)r;
}

QD_API int qd_comm_count(void* comm, int* n) {
  if (g_api.comm_count == nullptr) return kNotLoaded;
  return (int)g_api.comm_count((ncclComm_t)comm, n);
}

QD_API int qd_comm_async_error(void* comm, int* err) {
  if (g_api.comm_async_error == nullptr) return kNotLoaded;
  ncclResult_t e = ncclSuccess;
  ncclResult_t r = g_api.comm_async_error((ncclComm_t)comm, &e);
  *err = (int)e;
  return (int)r;
}

QD_API int qd_comm_destroy(void* comm, int abort) {
  if (g_api.comm_destroy == nullptr) return kNotLoaded;
  return (int)(abort ? g_api.comm_abort((ncclComm_t)comm) : g_api.comm_destroy((ncclComm_t)comm));
}

// sum / max / min over ranks; send == recv is the in-place form
QD_API int qd_comm_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                              void* stream) {
  if (g_api.all_reduce == nullptr) return kNotLoaded;
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!to_dtype(dtype, &t) || !to_op(op, &o)) return kBadArg;
  return (int)g_api.all_reduce(send, recv, count, t, o, (ncclComm_t)comm, (hipStream_t)stream);
}

// recv (recv_count elements) = this rank's 1/nranks block of the sum of every rank's send
QD_API int qd_comm_reduce_scatter(void* comm, const void* send, void* recv, size_t recv_count, int dtype, int op,
                                  void* stream) {
  if (g_api.reduce_scatter == nullptr) return kNotLoaded;
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!to_dtype(dtype, &t) || !to_op(op, &o)) return kBadArg;
  return (int)g_api.reduce_scatter(send, recv, recv_count, t, o, (ncclComm_t)comm, (hipStream_t)stream);
}

// recv (nranks * send_count elements) = every rank's send, in rank order
QD_API int qd_comm_all_gather(void* comm, const void* send, void* recv, size_t send_count, int dtype, void* stream) {
  if (g_api.all_gather == nullptr) return kNotLoaded;
  ncclDataType_t t;
  if (!to_dtype(dtype, &t)) return kBadArg;
  return (int)g_api.all_gather(send, recv, send_count, t, (ncclComm_t)comm, (hipStream_t)stream);
}

QD_API int qd_comm_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                             void* stream) {
  if (g_api.broadcast == nullptr) return kNotLoaded;
  ncclDataType_t t;
  if (!to_dtype(dtype, &t)) return kBadArg;
  return (int)g_api.broadcast(send, recv, count, t, root, (ncclComm_t)comm, (hipStream_t)stream);
}

// several collectives issued between these two calls are launched as ONE fused RCCL operation
QD_API int qd_comm_group_start() {
  if (g_api.group_start == nullptr) return kNotLoaded;
  return (int)g_api.group_start();
}

QD_API int qd_comm_group_end() {
  if (g_api.group_end == nullptr) return kNotLoaded;
  return (int)g_api.group_end();
}
