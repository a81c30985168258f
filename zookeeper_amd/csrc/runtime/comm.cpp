// Native RCCL communicator: a thin C ABI over RCCL's own C API
// for the bucketed gradient all-reduce, so collectives can be issued straight
// onto a HIP stream -- and therefore captured into a HIP graph together with
// the backward kernels that produce the buckets -- without ProcessGroupNCCL's
// work objects and internal streams.
//
// RCCL is not linked: the process already holds one (torch's bundled
// librccl.so, loaded by ProcessGroupNCCL's library).  zk_comm_load(path)
// dlopens that exact file -- the same handle when torch has loaded it, never
// a second RCCL -- and resolves the entry points by name.  Everything here is
// host code; the unique id travels between ranks through the torch store
// (parallel/rccl.py).
//
// Types / enums mirror rccl.h (NCCL 2.x ABI): ncclUniqueId is 128 opaque
// bytes, ncclComm_t an opaque pointer, ncclResult_t an int; data types
// float32 = 7, bfloat16 = 9; reductions sum = 0, max = 2, min = 3, avg = 4.
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <mutex>

#define ZK_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct UniqueId {
  char internal[128];
};
typedef void* Comm;
typedef int Result;

typedef Result (*GetUniqueIdFn)(UniqueId*);
typedef Result (*CommInitRankFn)(Comm*, int, UniqueId, int);
typedef Result (*CommDestroyFn)(Comm);
typedef Result (*CommAbortFn)(Comm);
typedef Result (*CommCountFn)(Comm, int*);
typedef Result (*AllReduceFn)(const void*, void*, size_t, int, int, Comm, void*);
typedef Result (*BroadcastFn)(const void*, void*, size_t, int, int, Comm, void*);
typedef Result (*GroupFn)();
typedef const char* (*ErrStrFn)(Result);
typedef Result (*AsyncErrFn)(Comm, Result*);

struct Api {
  void* lib = nullptr;
  GetUniqueIdFn get_unique_id = nullptr;
  CommInitRankFn comm_init_rank = nullptr;
  CommDestroyFn comm_destroy = nullptr;
  CommAbortFn comm_abort = nullptr;
  CommCountFn comm_count = nullptr;
  AllReduceFn all_reduce = nullptr;
  BroadcastFn broadcast = nullptr;
  GroupFn group_start = nullptr;
  GroupFn group_end = nullptr;
  ErrStrFn err_str = nullptr;
  AsyncErrFn async_error = nullptr;  // optional (ncclCommGetAsyncError)
};

Api g_api;
std::mutex g_mu;

template <typename F>
bool resolve(void* lib, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(lib, name));
  return out != nullptr;
}

}  // namespace

// Resolve RCCL from `path` (torch's bundled librccl.so).  0 on success,
// 1 dlopen failed, 2 a required symbol is missing.  Idempotent.
ZK_EXPORT int zk_comm_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.lib) return 0;
  void* lib = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!lib) return 1;
  Api a;
  a.lib = lib;
  bool ok = resolve(lib, "ncclGetUniqueId", a.get_unique_id) &&
            resolve(lib, "ncclCommInitRank", a.comm_init_rank) &&
            resolve(lib, "ncclCommDestroy", a.comm_destroy) &&
            resolve(lib, "ncclCommAbort", a.comm_abort) &&
            resolve(lib, "ncclCommCount", a.comm_count) &&
            resolve(lib, "ncclAllReduce", a.all_reduce) &&
            resolve(lib, "ncclBroadcast", a.broadcast) &&
            resolve(lib, "ncclGroupStart", a.group_start) &&
            resolve(lib, "ncclGroupEnd", a.group_end) &&
            resolve(lib, "ncclGetErrorString", a.err_str);
  if (!ok) return 2;
  resolve(lib, "ncclCommGetAsyncError", a.async_error);  // optional
  g_api = a;
  return 0;
}

ZK_EXPORT int zk_comm_loaded() { return g_api.lib != nullptr; }

// Human-readable RCCL error text (empty if RCCL is not loaded).
ZK_EXPORT const char* zk_comm_error_string(int result) {
  return g_api.err_str ? g_api.err_str(result) : "";
}

// 128-byte unique id of a new communicator (rank 0 creates it, the store
// distributes it).  Returns the RCCL result (0 = success; -1: not loaded).
ZK_EXPORT int zk_comm_unique_id(void* out128) {
  if (!g_api.lib || !out128) return -1;
  UniqueId id;
  const Result r = g_api.get_unique_id(&id);
  if (r == 0) memcpy(out128, id.internal, sizeof(id.internal));
  return r;
}

// Collective: every rank calls it with the same id (the current HIP device
// is the communicator's device).  *comm_out receives the opaque handle.
ZK_EXPORT int zk_comm_init(const void* id128, int nranks, int rank, void** comm_out) {
  if (!g_api.lib || !id128 || !comm_out || nranks < 1 || rank < 0 || rank >= nranks) return -1;
  UniqueId id;
  memcpy(id.internal, id128, sizeof(id.internal));
  Comm c = nullptr;
  const Result r = g_api.comm_init_rank(&c, nranks, id, rank);
  *comm_out = r == 0 ? c : nullptr;
  return r;
}

ZK_EXPORT int zk_comm_count(void* comm, int* count) {
  if (!g_api.lib || !comm || !count) return -1;
  return g_api.comm_count(comm, count);
}

// In-place (sendbuf == recvbuf allowed) all-reduce of `count` elements of
// RCCL data type `dtype` with reduction `op` on `stream` (a hipStream_t).
ZK_EXPORT int zk_comm_all_reduce(void* comm, const void* send, void* recv, int64_t count,
                                 int dtype, int op, void* stream) {
  if (!g_api.lib || !comm || count < 0) return -1;
  return g_api.all_reduce(send, recv, (size_t)count, dtype, op, comm, stream);
}

ZK_EXPORT int zk_comm_broadcast(void* comm, const void* send, void* recv, int64_t count,
                                int dtype, int root, void* stream) {
  if (!g_api.lib || !comm || count < 0) return -1;
  return g_api.broadcast(send, recv, (size_t)count, dtype, root, comm, stream);
}

// Several collectives fused into one launch group (ncclGroupStart/End).
ZK_EXPORT int zk_comm_group_start() { return g_api.lib ? g_api.group_start() : -1; }
ZK_EXPORT int zk_comm_group_end() { return g_api.lib ? g_api.group_end() : -1; }

// Asynchronous error state of a communicator (ncclCommGetAsyncError): *err
// receives the RCCL result of the failed background operation, 0 if none.
// Returns -1 if RCCL is not loaded, -2 if this RCCL lacks the entry point.
ZK_EXPORT int zk_comm_async_error(void* comm, int* err) {
  if (!g_api.lib || !comm || !err) return -1;
  if (!g_api.async_error) return -2;
  Result e = 0;
  const Result r = g_api.async_error(comm, &e);
  *err = e;
  return r;
}

// abort = 1: ncclCommAbort (a peer failed; do not wait for it).
ZK_EXPORT int zk_comm_destroy(void* comm, int abort) {
  if (!g_api.lib || !comm) return -1;
  return abort ? g_api.comm_abort(comm) : g_api.comm_destroy(comm);
}
