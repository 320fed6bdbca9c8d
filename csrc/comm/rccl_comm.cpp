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
// sync loop) may be about to enqueue on it: once a handle is aborted or destroyed every later
// call on it returns kAborted instead of touching freed memory. The registry has its own mutex
// (never g_enqueue: an enqueue stuck inside RCCL on a dead peer holds that one, and the abort is
// exactly what must get through to unblock it).
std::mutex g_live_mu;
std::unordered_map<void*, int> g_live;  // 1 = live, 0 = aborted / destroyed

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

bool live(void* h) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  auto it = g_live.find(h);
  return h && it != g_live.end() && it->second == 1;
}

void retire_handle(void* h) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  g_live[h] = 0;
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
  *out = r == ncclSuccess ? (void*)comm : nullptr;
  if (r == ncclSuccess) {
    std::lock_guard<std::mutex> lk(g_live_mu);
    g_live[(void*)comm] = 1;
  }
  return (int)r;
}

int psx_comm_destroy(void* h) {
  if (!g_api.lib || !live(h)) return 0;
  retire_handle(h);
  return (int)g_api.comm_destroy((ncclComm_t)h);
}

// Safe from any thread, also while another thread is blocked inside RCCL on this communicator;
// a second abort / destroy of the same handle is a no-op.
int psx_comm_abort(void* h) {
  if (!g_api.lib || !live(h)) return 0;
  retire_handle(h);
  return (int)g_api.comm_abort((ncclComm_t)h);
}

// number of ranks of the communicator as RCCL reports it (ncclCommCount)
int psx_comm_count(void* h, int* n) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  if (!g_api.comm_count) return -3;
  return (int)g_api.comm_count((ncclComm_t)h, n);
}

int psx_comm_async_error(void* h) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = g_api.async_error((ncclComm_t)h, &e);
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
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.reduce(send, recv, (size_t)count, t, ncclSum, root, (ncclComm_t)h, st);
}

int psx_comm_all_reduce_sum(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.all_reduce(send, recv, (size_t)count, t, ncclSum, (ncclComm_t)h, st);
}

// Sharded server (parallel/sharded.py): rank r receives the sum of every rank's
// send[r*count, (r+1)*count) in recv (recv may be send + r*count: in place).
int psx_comm_reduce_scatter_sum(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.reduce_scatter(send, recv, (size_t)count, t, ncclSum, (ncclComm_t)h, st);
}

// rank r's `count` elements land at recv + r*count on every rank (send == recv + r*count: in place)
int psx_comm_all_gather(void* h, const void* send, void* recv, long count, int dtype, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.all_gather(send, recv, (size_t)count, t, (ncclComm_t)h, st);
}

int psx_comm_broadcast(void* h, void* buf, long count, int dtype, int root, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.broadcast(buf, buf, (size_t)count, t, root, (ncclComm_t)h, st);
}

int psx_comm_send(void* h, const void* buf, long count, int dtype, int peer, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.send(buf, (size_t)count, t, peer, (ncclComm_t)h, st);
}

int psx_comm_recv(void* h, void* buf, long count, int dtype, int peer, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
  ncclDataType_t t;
  if (!to_nccl(dtype, &t)) return kBadDtype;
  std::lock_guard<std::mutex> lk(g_enqueue);
  return (int)g_api.recv(buf, (size_t)count, t, peer, (ncclComm_t)h, st);
}

int psx_comm_group_start() { return g_api.lib ? (int)g_api.group_start() : kNotLoaded; }
int psx_comm_group_end() { return g_api.lib ? (int)g_api.group_end() : kNotLoaded; }

// Gather equal-size buffers to root: rank r's `send` lands in recv + r*count*elem on root
// (point-to-point inside one group; RCCL has no gather collective). recv unused off-root.
int psx_comm_gather(void* h, const void* send, void* recv, long count, int dtype, int elem_bytes, int root,
                    int rank, int nranks, hipStream_t st) {
  if (!g_api.lib) return kNotLoaded;
  if (!live(h)) return kAborted;
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
      } else if ((r = g_api.recv(dst, (size_t)count, t, p, (ncclComm_t)h, st)) != ncclSuccess) {
        g_api.group_end();
        return (int)r;
      }
    }
  } else if ((r = g_api.send(send, (size_t)count, t, root, (ncclComm_t)h, st)) != ncclSuccess) {
    g_api.group_end();
    return (int)r;
  }
  return (int)g_api.group_end();
}

}  // extern "C"
