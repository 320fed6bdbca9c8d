// TEST-ONLY stand-in for librccl.so: the RCCL subset psx uses (csrc/comm/rccl_comm.cpp), for
// several processes that share ONE GPU. RCCL refuses that ("Duplicate GPU detected"), so the
// multi-rank code paths of psx (NativeComm, the sync channels, the async server loop's remote
// workers) could otherwise only run on a multi-GPU node. Loaded by tests through
// psx_comm_load(path) (PSX_RCCL_LIB=<this library>); it refuses to initialise a communicator
// unless PSX_FAKECOMM_TEST=1, so it can never be picked up by a real job.
//
// Design: every call is HOST-synchronous (not graph-capturable, not overlapped — a correctness
// harness, not a data plane). Ranks rendezvous through a POSIX shared-memory segment named after
// the unique id; device buffers are exchanged with HIP IPC handles (hipIpcGetMemHandle of the
// allocation base + offset, opened once per peer allocation and cached).
//   collectives: stream sync -> publish my buffer (slot[rank], op sequence number) -> barrier ->
//                each rank moves / reduces the bytes it owns from the peers' mappings (sum in
//                fp32, rank order) -> device sync -> barrier (peers' buffers no longer read)
//   send / recv: per ordered pair a ring of 8 message slots (posted / done sequence numbers);
//                inside ncclGroupStart/End the operations are queued and run at GroupEnd as
//                post-all-sends, then all receives, then wait for the sends' completion, so a
//                group of mutual sends and receives cannot deadlock.
// Every wait has a deadline (PSX_FAKECOMM_TIMEOUT_S, default 120 s): a stalled peer turns into
// ncclRemoteError and a sticky async error instead of a hang.
// Streams: every copy and reduction kernel runs on a private non-blocking stream of the calling
// thread, waited for with hipStreamSynchronize — never the legacy null stream (hipMemcpy,
// hipDeviceSynchronize): a null-stream call from the server's comm thread invalidates a graph
// capture that the co-located worker's thread has open, in every capture mode
// (scripts/dev/capture_probe.py, profiles/r6_capture_probe.jsonl).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <map>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxRanks = 32;
constexpr int kRing = 8;

struct Pub {  // one published device buffer
  hipIpcMemHandle_t h;
  unsigned long long off;
  unsigned long long raw;  // the pointer itself (valid in the publisher's process only)
  int pid;
};

struct P2PSlot {
  Pub buf;
  unsigned long long bytes;
};

struct Shm {
  std::atomic<int> joined;
  std::atomic<int> left;
  std::atomic<int> aborted;
  int nranks;
  std::atomic<unsigned long long> bar_count;  // monotonic arrivals; generation = count / nranks
  Pub slot[kMaxRanks];
  std::atomic<unsigned long long> slot_seq[kMaxRanks];
  P2PSlot ring[kMaxRanks][kMaxRanks][kRing];          // [src][dst][k % kRing]
  std::atomic<unsigned long long> posted[kMaxRanks][kMaxRanks];
  std::atomic<unsigned long long> done[kMaxRanks][kMaxRanks];
};

struct Comm {
  Shm* shm = nullptr;
  std::string name;
  int rank = 0, nranks = 0;
  unsigned long long op = 0;       // collectives issued by this rank
  unsigned long long bar_mine = 0;  // barriers passed by this rank
  unsigned long long sent[kMaxRanks] = {};
  unsigned long long recvd[kMaxRanks] = {};
  ncclResult_t async_err = ncclSuccess;
  std::map<std::string, void*> mapped;  // IPC handle bytes -> mapped base
};

struct QOp {
  bool send;
  Comm* c;
  void* buf;
  size_t bytes;
  int peer;
  hipStream_t st;
};

thread_local int g_group = 0;
thread_local std::vector<QOp> g_queue;

double timeout_s() {
  const char* e = getenv("PSX_FAKECOMM_TIMEOUT_S");
  return e ? atof(e) : 120.0;
}

size_t dsize(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// spin until pred() or deadline / abort; false on failure
template <typename P>
bool wait_for(Comm* c, P pred) {
  const auto t0 = std::chrono::steady_clock::now();
  const double lim = timeout_s();
  int spins = 0;
  while (!pred()) {
    if (c->shm->aborted.load()) return false;
    if (++spins > 64) {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
    }
  }
  return true;
}

// the calling thread's private non-blocking stream (see the header)
hipStream_t priv() {
  thread_local hipStream_t s = nullptr;
  if (!s && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
  return s;
}

bool copy_d2d(void* dst, const void* src, size_t bytes) {
  hipStream_t s = priv();
  return s && hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
}

ncclResult_t fail(Comm* c, ncclResult_t e) {
  c->async_err = e;
  return e;
}

bool barrier(Comm* c) {
  const unsigned long long target = (c->bar_mine + 1) * (unsigned long long)c->nranks;
  c->shm->bar_count.fetch_add(1);
  c->bar_mine++;
  return wait_for(c, [&] { return c->shm->bar_count.load() >= target; });
}

bool publish_ptr(const void* p, Pub* out) {
  memset(out, 0, sizeof(*out));
  out->raw = (unsigned long long)p;
  out->pid = (int)getpid();
  if (!p) return true;
  void* base = nullptr;
  size_t sz = 0;
  if (hipMemGetAddressRange(&base, &sz, (void*)p) != hipSuccess) return false;
  if (hipIpcGetMemHandle(&out->h, base) != hipSuccess) return false;
  out->off = (unsigned long long)((const char*)p - (const char*)base);
  return true;
}

void* open_ptr(Comm* c, const Pub& pub) {
  if (pub.pid == (int)getpid()) return (void*)pub.raw;
  std::string key((const char*)&pub.h, sizeof(pub.h));
  auto it = c->mapped.find(key);
  void* base = nullptr;
  if (it == c->mapped.end()) {
    hipIpcMemHandle_t h = pub.h;
    if (hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
    c->mapped[key] = base;
  } else {
    base = it->second;
  }
  return (char*)base + pub.off;
}

// dst[i] = sum_k src_k[i] (fp32 accumulation in source order); dst may alias a source
template <typename T>
__device__ float ldf(const T* p, size_t i);
template <>
__device__ float ldf<float>(const float* p, size_t i) { return p[i]; }
template <>
__device__ float ldf<__half>(const __half* p, size_t i) { return __half2float(p[i]); }
template <>
__device__ float ldf<unsigned short>(const unsigned short* p, size_t i) {
  return __uint_as_float(((unsigned)p[i]) << 16);
}
__device__ void stf(float* p, size_t i, float v) { p[i] = v; }
__device__ void stf(__half* p, size_t i, float v) { p[i] = __float2half(v); }
__device__ void stf(unsigned short* p, size_t i, float v) {
  unsigned u = __float_as_uint(v);
  u += 0x7fffu + ((u >> 16) & 1u);
  p[i] = (unsigned short)(u >> 16);
}
__device__ float ldi(const int* p, size_t i) { return (float)p[i]; }

struct Srcs {
  const void* p[kMaxRanks];
  int n;
};

template <typename T>
__global__ void sum_kernel(Srcs s, T* dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < s.n; ++k) a += ldf<T>((const T*)s.p[k], i);
    stf(dst, i, a);
  }
}
__global__ void sum_i32_kernel(Srcs s, int* dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    long long a = 0;
    for (int k = 0; k < s.n; ++k) a += ((const int*)s.p[k])[i];
    dst[i] = (int)a;
  }
}

bool sum_into(const std::vector<const void*>& srcs, void* dst, size_t n, ncclDataType_t t) {
  Srcs s{};
  s.n = (int)srcs.size();
  for (int k = 0; k < s.n; ++k) s.p[k] = srcs[k];
  hipStream_t ps = priv();
  if (!ps) return false;
  size_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  switch (t) {
    case ncclFloat32: hipLaunchKernelGGL(sum_kernel<float>, dim3(g), dim3(256), 0, ps, s, (float*)dst, n); break;
    case ncclFloat16: hipLaunchKernelGGL(sum_kernel<__half>, dim3(g), dim3(256), 0, ps, s, (__half*)dst, n); break;
    case ncclBfloat16:
      hipLaunchKernelGGL(sum_kernel<unsigned short>, dim3(g), dim3(256), 0, ps, s, (unsigned short*)dst, n);
      break;
    case ncclInt32: hipLaunchKernelGGL(sum_i32_kernel, dim3(g), dim3(256), 0, ps, s, (int*)dst, n); break;
    default: return false;
  }
  return hipStreamSynchronize(ps) == hipSuccess;
}

// one collective step: publish `mine`, barrier, body(peer mappings), device sync, barrier
template <typename B>
ncclResult_t collective(Comm* c, const void* mine, hipStream_t st, B body) {
  if (c->async_err != ncclSuccess) return c->async_err;
  if (hipStreamSynchronize(st) != hipSuccess) return fail(c, ncclUnhandledCudaError);
  c->op++;
  if (!publish_ptr(mine, &c->shm->slot[c->rank])) return fail(c, ncclUnhandledCudaError);
  c->shm->slot_seq[c->rank].store(c->op);
  if (!barrier(c)) return fail(c, ncclRemoteError);
  std::vector<void*> peer(c->nranks, nullptr);
  for (int r = 0; r < c->nranks; ++r) {
    if (c->shm->slot_seq[r].load() != c->op) return fail(c, ncclInternalError);  // collective order mismatch
    if (c->shm->slot[r].raw) {
      peer[r] = open_ptr(c, c->shm->slot[r]);
      if (!peer[r]) return fail(c, ncclUnhandledCudaError);
    }
  }
  const bool ok = body(peer);  // its copies / kernels completed on priv() before it returned
  if (!ok) return fail(c, ncclUnhandledCudaError);
  if (!barrier(c)) return fail(c, ncclRemoteError);
  return ncclSuccess;
}

ncclResult_t do_send(Comm* c, const void* buf, size_t bytes, int peer) {
  const unsigned long long k = c->sent[peer]++;
  Shm* s = c->shm;
  if (!wait_for(c, [&] { return k - s->done[c->rank][peer].load() < (unsigned long long)kRing; }))
    return fail(c, ncclRemoteError);
  P2PSlot& sl = s->ring[c->rank][peer][k % kRing];
  if (!publish_ptr(buf, &sl.buf)) return fail(c, ncclUnhandledCudaError);
  sl.bytes = bytes;
  s->posted[c->rank][peer].store(k + 1);
  return ncclSuccess;
}

ncclResult_t wait_sent(Comm* c, int peer) {
  const unsigned long long k = c->sent[peer];
  if (!wait_for(c, [&] { return c->shm->done[c->rank][peer].load() >= k; })) return fail(c, ncclRemoteError);
  return ncclSuccess;
}

ncclResult_t do_recv(Comm* c, void* buf, size_t bytes, int peer) {
  const unsigned long long k = c->recvd[peer]++;
  Shm* s = c->shm;
  if (!wait_for(c, [&] { return s->posted[peer][c->rank].load() > k; })) return fail(c, ncclRemoteError);
  P2PSlot& sl = s->ring[peer][c->rank][k % kRing];
  if (sl.bytes != bytes) return fail(c, ncclInvalidUsage);
  void* src = open_ptr(c, sl.buf);
  if (!src) return fail(c, ncclUnhandledCudaError);
  if (!copy_d2d(buf, src, bytes)) return fail(c, ncclUnhandledCudaError);
  s->done[peer][c->rank].store(k + 1);
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id->internal, 0, sizeof(id->internal));
  snprintf(id->internal, sizeof(id->internal), "/psxfake_%d_%llx", (int)getpid(),
           (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count());
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
  const char* gate = getenv("PSX_FAKECOMM_TEST");
  if (!gate || strcmp(gate, "1") != 0) {
    fprintf(stderr, "psx fakecomm: test-only library (set PSX_FAKECOMM_TEST=1 in a test)\n");
    return ncclInvalidUsage;
  }
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  Comm* c = new Comm();
  c->name.assign(id.internal, strnlen(id.internal, sizeof(id.internal)));
  const int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, sizeof(Shm)) != 0) {
    delete c;
    return ncclSystemError;
  }
  void* m = mmap(nullptr, sizeof(Shm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    delete c;
    return ncclSystemError;
  }
  c->shm = (Shm*)m;  // zero-filled by ftruncate; every field is a valid initial state at zero
  c->rank = rank;
  c->nranks = nranks;
  c->shm->nranks = nranks;
  c->shm->joined.fetch_add(1);
  if (!wait_for(c, [&] { return c->shm->joined.load() >= nranks; })) {
    munmap(m, sizeof(Shm));
    delete c;
    return ncclRemoteError;
  }
  *out = (ncclComm_t)c;
  return ncclSuccess;
}

static ncclResult_t release(Comm* c, bool abort) {
  if (!c) return ncclSuccess;
  if (abort) {
    // ncclCommAbort may come from another thread while this rank's collectives spin on the
    // segment (the liveness watchdog): flag every rank and keep the mapping alive (leaked)
    c->shm->aborted.store(1);
    return ncclSuccess;
  }
  barrier(c);  // every rank is done reading the others' buffers
  for (auto& kv : c->mapped) hipIpcCloseMemHandle(kv.second);
  if (c->shm->left.fetch_add(1) + 1 == c->nranks) shm_unlink(c->name.c_str());
  munmap(c->shm, sizeof(Shm));
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) { return release((Comm*)comm, false); }
ncclResult_t ncclCommAbort(ncclComm_t comm) { return release((Comm*)comm, true); }

ncclResult_t ncclCommGetAsyncError(ncclComm_t comm, ncclResult_t* err) {
  Comm* c = (Comm*)comm;
  *err = c->shm->aborted.load() ? ncclRemoteError : c->async_err;
  return ncclSuccess;
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
  *count = ((Comm*)comm)->nranks;
  return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
  switch (r) {
    case ncclSuccess: return "no error (fakecomm)";
    case ncclUnhandledCudaError: return "HIP error (fakecomm)";
    case ncclSystemError: return "system error (fakecomm)";
    case ncclInternalError: return "collective order mismatch (fakecomm)";
    case ncclInvalidArgument: return "invalid argument (fakecomm)";
    case ncclInvalidUsage: return "invalid usage (fakecomm)";
    case ncclRemoteError: return "peer timeout / abort (fakecomm)";
    default: return "unknown (fakecomm)";
  }
}

ncclResult_t ncclReduce(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op, int root,
                        ncclComm_t comm, hipStream_t st) {
  Comm* c = (Comm*)comm;
  if (op != ncclSum || !dsize(t)) return ncclInvalidArgument;
  return collective(c, send, st, [&](std::vector<void*>& peer) {
    if (c->rank != root) return true;
    std::vector<const void*> srcs(peer.begin(), peer.end());
    return sum_into(srcs, recv, count, t);
  });
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t st) {
  Comm* c = (Comm*)comm;
  if (op != ncclSum || !dsize(t)) return ncclInvalidArgument;
  // sum into a private buffer first: recv may alias send, which the peers still read
  void* tmp = nullptr;
  if (hipMalloc(&tmp, count * dsize(t)) != hipSuccess) return ncclUnhandledCudaError;
  ncclResult_t r = collective(c, send, st, [&](std::vector<void*>& peer) {
    std::vector<const void*> srcs(peer.begin(), peer.end());
    return sum_into(srcs, tmp, count, t);
  });
  if (r == ncclSuccess && !copy_d2d(recv, tmp, count * dsize(t)))
    r = ncclUnhandledCudaError;
  hipFree(tmp);
  return r;
}

ncclResult_t ncclReduceScatter(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                               ncclComm_t comm, hipStream_t st) {
  Comm* c = (Comm*)comm;
  const size_t es = dsize(t);
  if (op != ncclSum || !es) return ncclInvalidArgument;
  void* tmp = nullptr;
  if (hipMalloc(&tmp, count * es) != hipSuccess) return ncclUnhandledCudaError;
  ncclResult_t r = collective(c, send, st, [&](std::vector<void*>& peer) {
    std::vector<const void*> srcs;
    for (void* p : peer) srcs.push_back((const char*)p + (size_t)c->rank * count * es);
    return sum_into(srcs, tmp, count, t);
  });
  if (r == ncclSuccess && !copy_d2d(recv, tmp, count * es))
    r = ncclUnhandledCudaError;
  hipFree(tmp);
  return r;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t st) {
  Comm* c = (Comm*)comm;
  const size_t es = dsize(t);
  if (!es) return ncclInvalidArgument;
  // send may be recv + rank*count (in place): peers read from send before anyone writes recv
  void* tmp = nullptr;
  if (hipMalloc(&tmp, count * es * c->nranks) != hipSuccess) return ncclUnhandledCudaError;
  ncclResult_t r = collective(c, send, st, [&](std::vector<void*>& peer) {
    for (int p = 0; p < c->nranks; ++p)
      if (!copy_d2d((char*)tmp + (size_t)p * count * es, peer[p], count * es))
        return false;
    return true;
  });
  if (r == ncclSuccess && !copy_d2d(recv, tmp, count * es * c->nranks))
    r = ncclUnhandledCudaError;
  hipFree(tmp);
  return r;
}

ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, ncclDataType_t t, int root, ncclComm_t comm,
                           hipStream_t st) {
  Comm* c = (Comm*)comm;
  const size_t es = dsize(t);
  if (!es) return ncclInvalidArgument;
  return collective(c, c->rank == root ? send : nullptr, st, [&](std::vector<void*>& peer) {
    if (c->rank == root) {
      return send == recv || copy_d2d(recv, send, count * es);
    }
    return copy_d2d(recv, peer[root], count * es);
  });
}

ncclResult_t ncclGroupStart() {
  g_group++;
  return ncclSuccess;
}

static ncclResult_t run_queue(std::vector<QOp>& q) {
  for (auto& o : q)
    if (hipStreamSynchronize(o.st) != hipSuccess) return ncclUnhandledCudaError;
  ncclResult_t r = ncclSuccess;
  for (auto& o : q)
    if (o.send && (r = do_send(o.c, o.buf, o.bytes, o.peer)) != ncclSuccess) return r;
  for (auto& o : q)
    if (!o.send && (r = do_recv(o.c, o.buf, o.bytes, o.peer)) != ncclSuccess) return r;
  for (auto& o : q)
    if (o.send && (r = wait_sent(o.c, o.peer)) != ncclSuccess) return r;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_group <= 0) return ncclInvalidUsage;
  if (--g_group > 0) return ncclSuccess;
  std::vector<QOp> q;
  q.swap(g_queue);
  return run_queue(q);
}

static ncclResult_t p2p(bool send, const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                        hipStream_t st) {
  Comm* c = (Comm*)comm;
  if (!dsize(t) || peer < 0 || peer >= c->nranks || peer == c->rank) return ncclInvalidArgument;
  if (c->async_err != ncclSuccess) return c->async_err;
  QOp o{send, c, (void*)buf, count * dsize(t), peer, st};
  if (g_group > 0) {
    g_queue.push_back(o);
    return ncclSuccess;
  }
  std::vector<QOp> q{o};
  return run_queue(q);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t st) {
  return p2p(true, buf, count, t, peer, comm, st);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t st) {
  return p2p(false, buf, count, t, peer, comm, st);
}

}  // extern "C"
