// Native RCCL data plane of the parameter server (C ABI, loaded with ctypes after `import torch`).
//
// Replaces the reference's gRPC transport (reference: src/communication/ps_pb2_grpc.py:28-121,
// src/parameter_server/server.py:370-393, src/workers/worker.py:199-311) for the bulk tensors:
//   sync  : reduce(sum) of the fp16 gradient wire to rank 0, broadcast of the weight wire from 0
//   async : send/recv between a worker and the rank-0 server (ncclSend/ncclRecv, paired by the
//           shared-memory control mailbox because RCCL has no any-source receive)
// Every operation is enqueued on the CALLER's HIP stream (normally the compute stream), so a sync
// round is plain stream order — no cross-stream events as with torch.distributed's internal
// communication stream — and the collectives can sit inside a captured HIP graph.
//
// RCCL itself is not linked at build time: psx_comm_load() dlopens the librccl.so that PyTorch
// already loaded (torch/lib/librccl.so) so the process holds ONE RCCL instance, falling back to
// /opt/rocm/lib/librccl.so. The unique id is created on rank 0 and shared by the caller (the
// gloo control group), then ncclCommInitRank builds the communicator over xGMI.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <unordered_map>

namespace {

struct Api {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclCommAbort) comm_abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclCommCount) comm_count = nullptr;  // optional
};

Api g_api;
std::mutex g_enqueue;  // RCCL communicators are not safe for concurrent enqueue from several threads

// Registry of the communicators this process created. ncclCommAbort frees the communicator, and
// the liveness watchdog calls it from its own thread while the training thread (or the native
// sync loop) may be about to enqueue on it. Handles given to the caller are generation ids, never
// the ncclComm_t address: a key is never reused, so a stale handle of an aborted communicator can
// never match a later one that RCCL allocated at the same address (the shrink's ncclCommInitRank).
// Every call takes the communicator out of the registry with an in-use count (acquire / release);
// abort first marks the entry dead (no new user can start), then waits up to kAbortDrainMs for the
// in-use count to drain before it frees. The remaining window: a user blocked INSIDE RCCL past that
// wait (an enqueue stuck on a dead peer — exactly what the abort must unblock) still holds the
// pointer when RCCL frees it; RCCL's abort contract is what covers that call. The registry has its
// own mutex (never g_enqueue: a stuck enqueue holds that one).
struct Entry {
  ncclComm_t comm = nullptr;
  int state = 0;  // 1 = live, 0 = aborted / destroyed
  int inuse = 0;
};
std::mutex g_live_mu;
std::condition_variable g_live_cv;
std::unordered_map<uintptr_t, Entry> g_live;
uintptr_t g_next_id = 1;
constexpr int kAbortDrainMs = 2000;

// psx dtype codes (parallel/rccl.py DTYPES) -> RCCL
bool to_nccl(int code, ncclDataType_t* out) {
  switch (code) {
    case 0: *out = ncclUint8; return true;
    case 1: *out = ncclFloat16; return true;
    case 2: *out = ncclFloat32; return true;
    case 3: *out = ncclBfloat16; return true;
    case 4: *out = ncclInt32; return true;
    default: return false;
  }
}

template <typename F>
bool sym(void* lib, const char* name, F* fn) {
  *fn = reinterpret_cast<F>(dlsym(lib, name));
  return *fn != nullptr;
}

constexpr int kNotLoaded = -1000;
constexpr int kBadDtype = -1001;
constexpr int kAborted = -1002;

// the communicator of a live handle with its in-use count raised, or nullptr (aborted / unknown)
ncclComm_t acquire(void* h) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.find((uintptr_t)h);
  if (!h || it == g_live.end() || it->second.state != 1) return nullptr;
  ++it->second.inuse;
  return it->second.comm;
}

void release(void* h) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.find((uintptr_t)h);
  if (it != g_live.end() && it->second.inuse > 0 && --it->second.inuse == 0) g_live_cv.notify_all();
}

// RAII user of a handle for the duration of one call
struct Use {
  void* h;
  ncclComm_t c;
  explicit Use(void* h_) : h(h_), c(acquire(h_)) {}
  ~Use() {
    if (c) release(h);
  }
  Use(const Use&) = delete;
  Use& operator=(const Use&) = delete;
};

// marks the handle dead and returns its communicator once the in-use count drained (or the
// drain wait ran out); nullptr when it was not live (a second abort / destroy is a no-op)
ncclComm_t retire_handle(void* h, bool wait_users) {
  std::unique_lock<std::mutex> lk(g_live_mu);
  auto it = g_live.find((uintptr_t)h);
  if (!h || it == g_live.end() || it->second.state != 1) return nullptr;
  it->second.state = 0;
  if (wait_users)
    g_live_cv.wait_for(lk, std::chrono::milliseconds(kAbortDrainMs), [&] { return it->second.inuse == 0; });
  return it->second.comm;
}

}  // namespace

extern "C" {

// Returns 0 on success; negative if the library or a symbol is missing.
int psx_comm_load(const char* path) {
  if (g_api.lib) return 0;
  void* lib = dlopen(path && path[0] ? path : "librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    fprintf(stderr, "psx_comm_load: %s\n", dlerror());
    return -1;
  }
  Api a;
  a.lib = lib;
  bool ok = sym(lib, "ncclGetUniqueId", &a.get_unique_id) && sym(lib, "ncclCommInitRank", &a.comm_init_rank) &&
            sym(lib, "ncclCommDestroy", &a.comm_destroy) && sym(lib, "ncclCommAbort", &a.comm_abort) &&
            sym(lib, "ncclCommGetAsyncError", &a.async_error) && sym(lib, "ncclReduce", &a.reduce) &&
            sym(lib, "ncclBroadcast", &a.broadcast) && sym(lib, "ncclAllReduce", &a.all_reduce) &&
            sym(lib, "ncclReduceScatter", &a.reduce_scatter) && sym(lib, "ncclAllGather", &a.all_gather) &&
            sym(lib, "ncclSend", &a.send) && sym(lib, "ncclRecv", &a.recv) &&
            sym(lib, "ncclGroupStart", &a.group_start) && sym(lib, "ncclGroupEnd", &a.group_end) &&
            sym(lib, "ncclGetErrorString", &a.error_string);
  sym(lib, "ncclCommCount", &a.comm_count);  // optional (not in every stand-in)
  if (!ok) {
    fprintf(stderr, "psx_comm_load: missing RCCL symbol in %s\n", path ? path : "librccl.so");
    return -2;
  }
  g_api = a;
  return 0;
}

int psx_comm_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

int psx_comm_unique_id(char* out) {
  if (!g_api.lib) return kNotLoaded;
  ncclUniqueId id;
  const ncclResult_t r = g_api.get_unique_id(&id);
  if (r == ncclSuccess) memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return (int)r;
}

// Creates the communicator of `rank` among `nranks` on HIP device `device`; *out = handle.
int psx_comm_init(const char* id_bytes, int nranks, int rank, int device, void** out) {
  if (!g_api.lib) return kNotLoaded;
  if (hipSetDevice(device) != hipSuccess) return -2;
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  const ncclResult_t r = g_api.comm_init_rank(&comm, nranks, id, rank);
  *out = nullptr;
  if (r == ncclSuccess) {
    std::lock_guard<std::mutex> lk(g_live_mu);
    const uintptr_t key = g_next_id++;
    Entry& e = g_live[key];
    e.comm = comm;
    e.state = 1;
    *out = (void*)key;
  }
  return (int)r;
}

int psx_comm_destroy(void* h) {
  if (!g_api.lib) return 0;
  ncclComm_t c = retire_handle(h, true);
  return c ? (int)g_api.comm_destroy(c) : 0;
}

// Safe from any thread, also while another thread is blocked inside RCCL on this communicator;
// a second abort / destroy of the same handle is a no-op.
int psx_comm_abort(void* h) {
  if (!g_api.lib) return 0;
  ncclComm_t c = retire_handle(h, true);
  return c ? (int)g_api.comm_abort(c) : 0;
}

// number of ranks of the communicator as RCCL reports it (ncclCommCount)
int psx_comm_count(void* h, int* n) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  if (!g_api.comm_count) return -3;
  return (int)g_api.comm_count(u.c, n);
}

int psx_comm_async_error(void* h) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = g_api.async_error(u.c, &e);
  return r != ncclSuccess ? (int)r : (int)e;
}

const char* psx_comm_error_string(int code) {
  if (code == kNotLoaded) return "RCCL not loaded (psx_comm_load)";
  if (code == kBadDtype) return "unsupported dtype code";
  if (code == kAborted) return "communicator aborted or destroyed (liveness watchdog / recovery)";
  return g_api.lib ? g_api.error_string((ncclResult_t)code) : "RCCL not loaded";
}

// sum-reduce `count` elements of `send` into `recv` on `root` (recv may alias send)
int psx_comm_reduce_sum(void* h, const void* send, void* recv, long count, int dtype, int root, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.reduce(send, recv, (size_t)count, t, ncclSum, root, u.c, st);
}

int psx_comm_all_reduce_sum(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.all_reduce(send, recv, (size_t)count, t, ncclSum, u.c, st);
}

// Sharded server (parallel/sharded.py): rank r receives the sum of every rank's
// send[r*count, (r+1)*count) in recv (recv may be send + r*count: in place).
int psx_comm_reduce_scatter_sum(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.reduce_scatter(send, recv, (size_t)count, t, ncclSum, u.c, st);
}

// rank r's `count` elements land at recv + r*count on every rank (send == recv + r*count: in place)
int psx_comm_all_gather(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.all_gather(send, recv, (size_t)count, t, u.c, st);
}

int psx_comm_broadcast(void* h, void* buf, long count, int dtype, int root, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.broadcast(buf, buf, (size_t)count, t, root, u.c, st);
}

int psx_comm_send(void* h, const void* buf, long count, int dtype, int peer, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.send(buf, (size_t)count, t, peer, u.c, st);
}

int psx_comm_recv(void* h, void* buf, long count, int dtype, int peer, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.recv(buf, (size_t)count, t, peer, u.c, st);
}

int psx_comm_group_start() { return g_api.lib ? (int)g_api.group_start() : kNotLoaded; }
int psx_comm_group_end() { return g_api.lib ? (int)g_api.group_end() : kNotLoaded; }

// Gather equal-size buffers to root: rank r's `send` lands in recv + r*count*elem on root
// (point-to-point inside one group; RCCL has no gather collective). recv unused off-root.
int psx_comm_gather(void* h, const void* send, void* recv, long count, int dtype, int elem_bytes, int root,
                    int rank, int nranks, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  Use u(h);
  if (!u.c) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  ncclResult_t r = g_api.group_start();
  if (r != ncclSuccess) return (int)r;
  if (rank == root) {
    for (int p = 0; p < nranks; ++p) {
      char* dst = (char*)recv + (size_t)p * (size_t)count * (size_t)elem_bytes;
      if (p == root) {
        if (hipMemcpyAsync(dst, send, (size_t)count * elem_bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) {
          g_api.group_end();
          return -3;
        }
      } else if ((r = g_api.recv(dst, (size_t)count, t, p, u.c, st)) != ncclSuccess) {
        g_api.group_end();
        return (int)r;
      }
    }
  } else if ((r = g_api.send(send, (size_t)count, t, root, u.c, st)) != ncclSuccess) {
    g_api.group_end();
    return (int)r;
  }
  return (int)g_api.group_end();
}

}  // extern "C"
