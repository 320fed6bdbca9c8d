// Native asynchronous parameter-server event loop (rank 0), on HIP streams.
//
// The reference serves async pushes on a 20-thread gRPC pool that applies each gradient under a
// Python lock as soon as it arrives, after a staleness check (reference:
// src/parameter_server/server.py:171-186, 239-304, 370-393). Here one native thread runs the
// whole server role of an async job:
//
//   control   worker -> server requests arrive on the shared-memory mailbox (HELLO, FETCH, PUSH,
//             DONE, HEARTBEAT, STOP; csrc/runtime/mailbox.cpp); replies go to per-worker slots.
//   decisions registration, staleness = global_step - local_step, reject above the bound,
//             weight max(0.1, 1/(1+0.1 s)), heartbeat timeouts: the native core
//             (csrc/runtime/ps_core.cpp), no Python in the loop.
//   data      RCCL point-to-point (csrc/comm/rccl_comm.cpp), one communicator and one
//             communication stream PER WORKER (a 2-rank communicator {server, worker}, see
//             parallel/rccl.py RcclTransport.open_pairs): the pushes and fetches of different
//             workers are independent streams of work, so 7 workers drive 7 xGMI links at once and
//             no worker's transfer waits behind another's. A PUSH posts ncclRecv into the worker's
//             gradient slot (RCCL has no any-source receive — the mailbox message names the peer);
//             a FETCH sends a per-worker snapshot of the fetch payload (bf16conv: bf16 weight image
//             + fp32 remainder; fp32: the whole fp32 arena, the reference's payload).
//   updates   one update stream serializes every apply (the reference's param_lock): the fused
//             SGD kernel (momentum / weight decay as the Python server) waits on the slot's receive
//             event, updates the fp32 master arena and rewrites the bf16 image in the same pass
//             (csrc/kernels/optim.hip); pushes complete in any order across workers. Snapshots are
//             taken on the same stream, so a fetch never sees a half-applied update and a send
//             in flight never races the next update (it reads its own snapshot).
//   local     the co-located worker of rank 0 calls psx_loop_local_push / _fetch / _done; the
//             loop thread serves them between mailbox messages, ordered on the update stream
//             against the caller's stream by events.
//
// Checkpoints (--ckpt-every): after the apply that reaches a multiple of the period the loop
// waits for that apply (an event on the update stream) and calls back into the host
// (ParameterServer.maybe_checkpoint). The loop thread runs in relaxed stream-capture mode, so
// neither that wait nor its other runtime calls invalidate a HIP graph the co-located worker
// captures on another thread.
//
// Failures (the reference tolerates leaving / failing workers: JobFinished server.py:306-318,
// keepalive :375-377). A remote worker is dropped when
//   * its heartbeats stop (--heartbeat-timeout, the native core's timeouts),
//   * one of its transfers is still in flight --transfer-timeout s after it was posted,
//   * it sends no request for --stall-timeout s (alive but stalled: heartbeats alone never
//     notice a hung training loop),
//   * a transfer on its communicator fails.
// Dropping w aborts its pair communicator when a receive or snapshot send is in flight
// (ncclCommAbort: what unblocks RCCL kernels waiting on a dead peer), discards its pending
// receive, marks it dead in the core (the wait-for-N barrier and the end-of-job count go on
// without it) and answers its later requests with R_DROPPED. The other workers keep being
// served; SERVER_FINAL_METRICS reports dead_workers.
//
// The loop ends when the expected number of workers finished or were dropped and no receive is
// pending, or on STOP. Every HIP runtime call is checked (a failure ends the loop with an
// error). Kernels and runtime functions are bound by dlsym from the already-loaded psx
// libraries (paths passed by the caller).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "psx_comm.h"

namespace {

// mailbox message types (parallel/control.py)
enum { HELLO = 1, PUSH = 2, FETCH = 3, DONE = 4, HEARTBEAT = 5, STOP = 6 };
enum { R_REGISTERED = 11, R_PUSHED = 12, R_FETCHED = 13, R_ACK = 14, R_DROPPED = 15 };
enum { PSX_APPLY = 1 };

struct Rt {  // libpsx_runtime.so + libpsx_kernels.so entry points
  int (*mbox_recv)(void*, long long*, double);
  int (*mbox_reply)(void*, int, int, int, int, long long, long long);
  int (*ps_register)(void*, const char*, int, double);
  void (*ps_heartbeat)(void*, int, double);
  long long (*ps_on_fetch)(void*, int, double);
  int (*ps_on_push)(void*, int, long long, double, float*, int*, long long*);
  void (*ps_on_applied)(void*, double);
  void (*ps_record_update_time)(void*, double);
  int (*ps_job_finished)(void*, int);
  int (*ps_mark_dead)(void*, int);
  int (*ps_check_timeouts)(void*, double, double, int*, int);
  long long (*ps_global_step)(void*);
  int (*sgd_apply)(float*, const void*, float*, long, float, float, float, float, int, int, void*, hipStream_t);
  int (*gather_f32)(const float*, const long*, long, float*, hipStream_t);
};

template <typename F>
bool bind(void* lib, const char* name, F* fn) {
  *fn = reinterpret_cast<F>(dlsym(lib, name));
  if (!*fn) fprintf(stderr, "psx event loop: missing symbol %s\n", name);
  return *fn != nullptr;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct LocalReq {
  int kind;  // 0 push, 1 fetch, 2 done
  int wid;
  const void* grads;
  float* dst;
  long long local_step;
  hipStream_t stream;
  // results
  int accepted = 0;
  long long staleness = 0, global_step = 0;
  bool done = false;
};

}  // namespace

struct PsxLoopCfg {  // mirrored by parallel/native_loop.py (ctypes.Structure)
  void* mbox;
  void* core;
  void* const* comms;      // worker id -> communicator of its data plane (host array [max_wid])
  const int* comm_peer;    // worker id -> the worker's rank in that communicator
  float* arena;            // fp32 master arena (params | buffers) on the device
  const long* small_idx;   // device int64 arena indices of the fp32 remainder of the fetch payload
  const int* remote_rank;  // worker id -> transport rank (-1: not remote), host array [max_wid]
  long n_params, small_n, arena_numel;
  float lr, momentum, weight_decay;
  int device, grad_fp16, max_wid, expected;
  int fetch_fp32;          // 1: fetch payload = whole fp32 arena; 0: bf16 image + fp32 remainder
  int mom_first;           // momentum buffer not yet initialised (no update since start / resume)
  float* mom_buf;          // device momentum buffer [n_params] (nullptr: plain SGD)
  double heartbeat_timeout, poll_s;
  // update stream: the co-located worker's compute stream when there is one (its pushes and
  // fetches are then plain stream order, as with a single stream), else a stream of the loop
  hipStream_t upd_stream;
  int own_upd_stream;
  long long ckpt_every;
  int (*ckpt_cb)(long long global_step);  // host checkpoint hook (nullptr: none)
  const int* comm_owned;   // worker id -> 1: comms[w] is w's own pair communicator (abortable)
  double transfer_timeout;  // s, 0 = off: a receive / snapshot send in flight longer drops the worker
  double stall_timeout;     // s, 0 = off: a remote worker without any request that long is dropped
};

struct PsxLoop {
  PsxLoopCfg c;
  Rt rt;
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<LocalReq*> local;
  int err = 0;
  bool stopped = false;
  // device state
  hipStream_t s_upd = nullptr;
  uint16_t* img = nullptr;  // server bf16 image of the parameters (rewritten by every apply)
  std::vector<hipStream_t> s_comm;  // per worker: communication stream
  std::vector<void*> slot;  // per worker: gradient receive buffer
  std::vector<uint16_t*> snap_img;
  std::vector<float*> snap_small;  // fp32 remainder (bf16conv) or the whole arena (fp32 fetch)
  std::vector<hipEvent_t> sent;  // per worker: last snapshot send done (snapshot reusable)
  std::vector<double> sent_t;    // per worker: when that send was posted
  struct Pending {
    int wid;
    long long local_step;
    hipEvent_t ev;
    double t_post;
  };
  std::deque<Pending> pending;
  struct WState {
    bool seen = false;      // registered through the mailbox (a remote worker)
    bool finished = false;  // counted towards `expected` (DONE or dropped)
    bool dead = false;      // dropped
    bool aborted = false;   // its pair communicator was aborted
    double last_req = 0;
  };
  std::vector<WState> ws;
  int finished = 0;
  long long applies = 0;
  // events created once: an ordering ring (a wait enqueued on a stream captures the record at
  // call time, so the event is re-recordable right after) and timing pairs around the applies,
  // whose DEVICE time feeds average_update_time_seconds (reference server.py:128,140-141) when
  // they complete
  enum { NORDER = 16 };
  hipEvent_t order[NORDER] = {};
  int order_pos = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> tfree;   // timing pairs available
  std::deque<std::pair<hipEvent_t, hipEvent_t>> tbusy;    // recorded, not yet read
  hipEvent_t ckpt_ev = nullptr;
};

namespace {

size_t gbytes(const PsxLoop* L) { return (size_t)L->c.n_params * (L->c.grad_fp16 ? 2 : 4); }

// HIP runtime calls of the loop: a failure is recorded (first one wins) and ends the loop
#define PSX_HIP(L, call)                                                                          \
  do {                                                                                            \
    const hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "psx event loop: %s failed: %s\n", #call, hipGetErrorString(e_));           \
      if (!(L)->err) (L)->err = -50;                                                              \
    }                                                                                             \
  } while (0)

// a is ordered after everything enqueued on b so far (an event of the ordering ring)
void stream_after(PsxLoop* L, hipStream_t a, hipStream_t b) {
  if (!L->order[L->order_pos]) PSX_HIP(L, hipEventCreateWithFlags(&L->order[L->order_pos], hipEventDisableTiming));
  hipEvent_t ev = L->order[L->order_pos];
  L->order_pos = (L->order_pos + 1) % PsxLoop::NORDER;
  PSX_HIP(L, hipEventRecord(ev, b));
  PSX_HIP(L, hipStreamWaitEvent(a, ev, 0));
}

// completed apply timings -> the core's update-time statistics (block: wait for all)
void read_timings(PsxLoop* L, bool block) {
  while (!L->tbusy.empty()) {
    auto p = L->tbusy.front();
    if (block) {
      PSX_HIP(L, hipEventSynchronize(p.second));
    } else if (hipEventQuery(p.second) != hipSuccess) {
      break;  // in order on the update stream: later pairs are not done either
    }
    float ms = 0.f;
    PSX_HIP(L, hipEventElapsedTime(&ms, p.first, p.second));
    L->rt.ps_record_update_time(L->c.core, 1e-3 * (double)ms);
    L->tbusy.pop_front();
    L->tfree.push_back(p);
  }
}

int alloc_worker(PsxLoop* L, int w) {
  if (L->slot[w]) return 0;
  if (!L->c.comms[w]) return -24;  // a remote request from a worker without a data-plane communicator
  if (hipStreamCreateWithFlags(&L->s_comm[w], hipStreamNonBlocking) != hipSuccess) return -25;
  if (hipMalloc(&L->slot[w], gbytes(L)) != hipSuccess) return -20;
  if (!L->c.fetch_fp32 && hipMalloc((void**)&L->snap_img[w], (size_t)L->c.n_params * 2) != hipSuccess) return -21;
  const long nsmall = L->c.fetch_fp32 ? L->c.arena_numel : std::max(1L, L->c.small_n);
  if (hipMalloc((void**)&L->snap_small[w], (size_t)nsmall * 4) != hipSuccess) return -22;
  if (hipEventCreateWithFlags(&L->sent[w], hipEventDisableTiming) != hipSuccess) return -23;
  if (hipEventRecord(L->sent[w], L->s_comm[w]) != hipSuccess) return -23;
  return 0;
}

// the fused SGD apply of one gradient with the core's weight (+ the bf16 image of the updated
// state when the fetch payload carries it; the fp32 fetch never reads one)
int apply(PsxLoop* L, const void* g, float weight) {
  read_timings(L, false);
  std::pair<hipEvent_t, hipEvent_t> tp{nullptr, nullptr};
  if (!L->tfree.empty()) {
    tp = L->tfree.back();
    L->tfree.pop_back();
  } else {
    PSX_HIP(L, hipEventCreate(&tp.first));
    PSX_HIP(L, hipEventCreate(&tp.second));
  }
  PSX_HIP(L, hipEventRecord(tp.first, L->s_upd));
  // the kernel wrappers report hipGetLastError(): clear what an earlier hipEventQuery (a
  // hipErrorNotReady of a transfer still in flight) left in this thread's error slot
  (void)hipGetLastError();
  const int e = L->rt.sgd_apply(L->c.arena, g, L->c.mom_buf, L->c.n_params, L->c.lr, weight, L->c.momentum,
                                L->c.weight_decay, L->c.mom_first, L->c.grad_fp16, L->img, L->s_upd);
  PSX_HIP(L, hipEventRecord(tp.second, L->s_upd));
  L->tbusy.push_back(tp);
  L->c.mom_first = 0;
  L->rt.ps_on_applied(L->c.core, -1.0);  // device time recorded when the pair completes
  ++L->applies;
  if (!e && L->c.ckpt_cb && L->c.ckpt_every > 0) {
    const long long gs = L->rt.ps_global_step(L->c.core);
    if (gs % L->c.ckpt_every == 0) {
      // the checkpoint reads the arena from another stream: wait for this apply only (an event,
      // not a stream synchronize)
      if (!L->ckpt_ev) PSX_HIP(L, hipEventCreateWithFlags(&L->ckpt_ev, hipEventDisableTiming));
      PSX_HIP(L, hipEventRecord(L->ckpt_ev, L->s_upd));
      PSX_HIP(L, hipEventSynchronize(L->ckpt_ev));
      if (L->c.ckpt_cb(gs)) return -32;
    }
  }
  return e;
}

bool in_flight(PsxLoop* L, int w) {
  for (const auto& p : L->pending)
    if (p.wid == w) return true;
  return L->sent[w] && hipEventQuery(L->sent[w]) == hipErrorNotReady;
}

// Drop worker w (see the header): abort its pair communicator if a transfer is in flight, discard
// its pending receive, mark it dead in the core, count it as finished.
void drop_worker(PsxLoop* L, int w, const char* why, bool core_marked = false) {
  PsxLoop::WState& s = L->ws[w];
  if (s.dead) return;
  s.dead = true;
  const bool busy = in_flight(L, w);
  fprintf(stderr, "[psx native loop] worker %d %s: dropped%s; serving the others\n", w, why,
          busy && L->c.comm_owned && L->c.comm_owned[w] ? " (pair communicator aborted)" : "");
  if (busy && L->c.comm_owned && L->c.comm_owned[w] && L->c.comms[w]) {
    psx_comm_abort(L->c.comms[w]);  // RCCL kernels waiting on the dead peer exit
    s.aborted = true;
  }
  for (auto it = L->pending.begin(); it != L->pending.end();) {
    if (it->wid == w) {
      hipEventDestroy(it->ev);  // never waited on: the update stream does not depend on it
      it = L->pending.erase(it);
    } else {
      ++it;
    }
  }
  if (!core_marked) L->rt.ps_mark_dead(L->c.core, w);
  if (!s.finished) {
    s.finished = true;
    ++L->finished;
  }
}

int serve_fetch(PsxLoop* L, int w, int rank) {
  if (int e = alloc_worker(L, w)) return e;
  // snapshot on the update stream (after every apply so far), once the previous send of this
  // worker's snapshot has finished
  PSX_HIP(L, hipStreamWaitEvent(L->s_upd, L->sent[w], 0));
  if (L->c.fetch_fp32) {
    PSX_HIP(L, hipMemcpyAsync(L->snap_small[w], L->c.arena, (size_t)L->c.arena_numel * 4, hipMemcpyDeviceToDevice,
                              L->s_upd));
  } else {
    PSX_HIP(L, hipMemcpyAsync(L->snap_img[w], L->img, (size_t)L->c.n_params * 2, hipMemcpyDeviceToDevice, L->s_upd));
    (void)hipGetLastError();  // see apply()
    if (L->c.small_n && L->rt.gather_f32(L->c.arena, L->c.small_idx, L->c.small_n, L->snap_small[w], L->s_upd))
      return -26;
  }
  stream_after(L, L->s_comm[w], L->s_upd);
  void* comm = L->c.comms[w];
  int e;
  if (L->c.fetch_fp32) {
    e = psx_comm_send(comm, L->snap_small[w], L->c.arena_numel, PSX_F32, rank, L->s_comm[w]);
  } else {
    e = psx_comm_send(comm, L->snap_img[w], L->c.n_params, PSX_BF16, rank, L->s_comm[w]);
    if (!e && L->c.small_n) e = psx_comm_send(comm, L->snap_small[w], L->c.small_n, PSX_F32, rank, L->s_comm[w]);
  }
  PSX_HIP(L, hipEventRecord(L->sent[w], L->s_comm[w]));
  L->sent_t[w] = now_s();
  return e;
}

int post_recv(PsxLoop* L, int w, int rank, long long local_step) {
  if (int e = alloc_worker(L, w)) return e;
  // the slot is free: its previous gradient was applied on s_upd before this worker could push
  // again (the worker waits for the reply, which follows the apply's enqueue) -> order the
  // receive after the update stream
  stream_after(L, L->s_comm[w], L->s_upd);
  const int e = psx_comm_recv(L->c.comms[w], L->slot[w], L->c.n_params, L->c.grad_fp16 ? PSX_F16 : PSX_F32, rank,
                              L->s_comm[w]);
  if (e) return e;
  hipEvent_t ev;
  PSX_HIP(L, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  PSX_HIP(L, hipEventRecord(ev, L->s_comm[w]));
  L->pending.push_back({w, local_step, ev, now_s()});
  return 0;
}

// deadlines of in-flight transfers and silent workers
void check_deadlines(PsxLoop* L, double t) {
  if (L->c.transfer_timeout > 0) {
    for (size_t i = 0; i < L->pending.size(); ++i) {
      const PsxLoop::Pending p = L->pending[i];
      if (t - p.t_post > L->c.transfer_timeout && hipEventQuery(p.ev) == hipErrorNotReady) {
        drop_worker(L, p.wid, "gradient receive overdue (--transfer-timeout)");
        i = (size_t)-1;  // the deque changed: rescan
      }
    }
    for (int w = 0; w < L->c.max_wid; ++w)
      if (!L->ws[w].dead && L->sent[w] && t - L->sent_t[w] > L->c.transfer_timeout &&
          hipEventQuery(L->sent[w]) == hipErrorNotReady)
        drop_worker(L, w, "snapshot send overdue (--transfer-timeout)");
  }
  if (L->c.stall_timeout > 0)
    for (int w = 0; w < L->c.max_wid; ++w) {
      const PsxLoop::WState& s = L->ws[w];
      if (s.seen && !s.finished && t - s.last_req > L->c.stall_timeout)
        drop_worker(L, w, "sent no request (--stall-timeout)");
    }
}

void complete_pending(PsxLoop* L) {
  // in completion order: every worker has its own stream, so a slow transfer does not hold back
  // the others (each worker has at most one push in flight: it waits for the reply)
  for (auto it = L->pending.begin(); it != L->pending.end();) {
    PsxLoop::Pending& p = *it;
    const hipError_t q = hipEventQuery(p.ev);
    if (q == hipErrorNotReady) {
      ++it;
      continue;
    }
    if (q != hipSuccess) {
      fprintf(stderr, "psx event loop: receive event of worker %d: %s\n", p.wid, hipGetErrorString(q));
      if (!L->err) L->err = -50;
      return;
    }
    float weight = 0.f;
    int ncontrib = 0;
    long long st = 0;
    const int d = L->rt.ps_on_push(L->c.core, p.wid, p.local_step, now_s(), &weight, &ncontrib, &st);
    int accepted = 0;
    if (d == PSX_APPLY) {
      PSX_HIP(L, hipStreamWaitEvent(L->s_upd, p.ev, 0));
      if (apply(L, L->slot[p.wid], weight)) L->err = -30;
      accepted = 1;
    }
    L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[p.wid], R_PUSHED, p.wid, accepted,
                     L->rt.ps_global_step(L->c.core), st);
    PSX_HIP(L, hipEventDestroy(p.ev));
    it = L->pending.erase(it);
  }
}

void serve_local(PsxLoop* L) {
  std::deque<LocalReq*> q;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    q.swap(L->local);
  }
  for (LocalReq* r : q) {
    if (r->kind == 0) {  // push: the caller's gradient is ready at this point of its stream
      float weight = 0.f;
      int ncontrib = 0;
      long long st = 0;
      const int d = L->rt.ps_on_push(L->c.core, r->wid, r->local_step, now_s(), &weight, &ncontrib, &st);
      const bool same = r->stream == L->s_upd;
      if (d == PSX_APPLY) {
        if (!same) stream_after(L, L->s_upd, r->stream);
        if (apply(L, r->grads, weight)) L->err = -31;
        r->accepted = 1;
      }
      r->staleness = st;
      r->global_step = L->rt.ps_global_step(L->c.core);
      if (!same) stream_after(L, r->stream, L->s_upd);  // the caller's gradient buffer is free again
    } else if (r->kind == 1) {  // fetch: fp32 arena copy, ordered after every apply so far
      r->global_step = L->rt.ps_on_fetch(L->c.core, r->wid, now_s());
      const bool same = r->stream == L->s_upd;
      if (!same) stream_after(L, L->s_upd, r->stream);
      PSX_HIP(L, hipMemcpyAsync(r->dst, L->c.arena, (size_t)L->c.arena_numel * 4, hipMemcpyDeviceToDevice,
                                L->s_upd));
      if (!same) stream_after(L, r->stream, L->s_upd);
    } else {
      L->rt.ps_job_finished(L->c.core, r->wid);
      if (!L->ws[r->wid].finished) {
        L->ws[r->wid].finished = true;
        ++L->finished;
      }
    }
    {
      std::lock_guard<std::mutex> lk(L->mu);
      r->done = true;
    }
    L->cv.notify_all();
  }
}

void run(PsxLoop* L) {
  PSX_HIP(L, hipSetDevice(L->c.device));
  // relaxed capture mode: this thread's runtime calls (event waits, allocations, the checkpoint
  // callback's copies) never invalidate a graph capture of the co-located worker's thread
  hipStreamCaptureMode cm = hipStreamCaptureModeRelaxed;
  PSX_HIP(L, hipThreadExchangeStreamCaptureMode(&cm));
  if (L->c.own_upd_stream)
    PSX_HIP(L, hipStreamCreateWithFlags(&L->s_upd, hipStreamNonBlocking));
  else
    L->s_upd = L->c.upd_stream;
  if (!L->c.fetch_fp32) {
    // initial bf16 image of the state: an lr-0 apply of a zero gradient writes bf16(p) exactly
    // (lr 0, no momentum buffer: the state is untouched). The fp32 fetch has no image.
    void* zero = nullptr;
    PSX_HIP(L, hipMalloc((void**)&L->img, (size_t)L->c.n_params * 2));
    PSX_HIP(L, hipMalloc(&zero, gbytes(L)));
    PSX_HIP(L, hipMemsetAsync(zero, 0, gbytes(L), L->s_upd));
    (void)hipGetLastError();
    if (!L->err && L->rt.sgd_apply(L->c.arena, zero, nullptr, L->c.n_params, 0.f, 1.f, 0.f, 0.f, 0, L->c.grad_fp16,
                                   L->img, L->s_upd))
      L->err = -33;
    PSX_HIP(L, hipStreamSynchronize(L->s_upd));
    PSX_HIP(L, hipFree(zero));
  }
  double last_to = now_s();
  std::vector<int> dead(L->c.max_wid + 1);
  long long m[6];
  bool need_drain = false;  // a long iteration happened: drain the mailbox before any timeout check
  while (!L->err) {
    const double t_iter = now_s();
    const int got = L->rt.mbox_recv(L->c.mbox, m, L->c.poll_s);
    if (got > 0) {
      const int type = (int)m[0], src = (int)m[1], wid = (int)m[2];
      const bool known = wid >= 0 && wid < L->c.max_wid;
      const double t = now_s();
      if (known && type != HEARTBEAT) L->ws[wid].last_req = t;
      if (type == HELLO && known && L->ws[wid].dead) {
        L->rt.mbox_reply(L->c.mbox, src, R_DROPPED, wid, 0, 0, 0);  // a dropped id does not come back
      } else if (type == HELLO) {
        char name[32];
        snprintf(name, sizeof name, "rank%d", src);
        const int id = L->rt.ps_register(L->c.core, name, wid, t);
        if (id >= 0 && id < L->c.max_wid) {
          L->ws[id].seen = true;
          L->ws[id].last_req = t;
        }
        L->rt.mbox_reply(L->c.mbox, src, R_REGISTERED, id, L->c.expected, 0, 0);
      } else if (known && L->ws[wid].dead && type != HEARTBEAT) {
        // a dropped worker (e.g. one that stalled past --stall-timeout and woke up): no transfer
        // is posted for it any more; DONE is acknowledged, everything else refused
        L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[wid], type == DONE ? R_ACK : R_DROPPED, wid, 0,
                         L->rt.ps_global_step(L->c.core), 0);
      } else if (type == FETCH && known) {
        const long long gs = L->rt.ps_on_fetch(L->c.core, wid, t);
        if (int e = serve_fetch(L, wid, L->c.comm_peer[wid])) {
          drop_worker(L, wid, "snapshot send failed");
          L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[wid], R_DROPPED, wid, e, gs, 0);
        } else {
          L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[wid], R_FETCHED, wid, 0, gs, 0);
        }
      } else if (type == PUSH && known) {
        if (int e = post_recv(L, wid, L->c.comm_peer[wid], m[4])) {
          drop_worker(L, wid, "gradient receive failed");
          L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[wid], R_DROPPED, wid, e, L->rt.ps_global_step(L->c.core), 0);
        }
      } else if (type == DONE && known) {
        L->rt.ps_job_finished(L->c.core, wid);
        if (!L->ws[wid].finished) {
          L->ws[wid].finished = true;
          ++L->finished;
        }
        L->rt.mbox_reply(L->c.mbox, L->c.remote_rank[wid], R_ACK, wid, 0, 0, 0);
      } else if (type == HEARTBEAT && known) {
        L->rt.ps_heartbeat(L->c.core, wid, t);
      } else if (type == STOP) {
        break;
      }
    }
    complete_pending(L);
    serve_local(L);
    const double t = now_s();
    // after a long iteration (a blocking transfer call) the live workers' queued heartbeats and
    // requests are seen first: no timeout check until the mailbox has been drained once
    if (t - t_iter > 0.5) need_drain = true;
    if (got <= 0) need_drain = false;
    if (!need_drain && t - last_to > 0.25) {
      last_to = t;
      if (L->c.heartbeat_timeout > 0) {
        const int n = L->rt.ps_check_timeouts(L->c.core, t, L->c.heartbeat_timeout, dead.data(), L->c.max_wid);
        for (int i = 0; i < n && i < L->c.max_wid; ++i)
          if (dead[i] >= 0 && dead[i] < L->c.max_wid) drop_worker(L, dead[i], "missed heartbeats", true);
      }
      check_deadlines(L, t);
    }
    if (L->finished >= L->c.expected && L->pending.empty()) break;
  }
  // drain: the communication streams of live workers (a dropped worker's stream may hold a
  // transfer its aborted communicator never completes), then the update stream
  for (size_t w = 0; w < L->s_comm.size(); ++w)
    if (L->s_comm[w] && !L->ws[w].dead) PSX_HIP(L, hipStreamSynchronize(L->s_comm[w]));
  PSX_HIP(L, hipStreamSynchronize(L->s_upd));
  read_timings(L, true);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stopped = true;
  }
  L->cv.notify_all();
}

}  // namespace

extern "C" {

int psx_loop_cfg_size() { return (int)sizeof(PsxLoopCfg); }

// Binds the runtime/kernel entry points (the libraries are already loaded by the caller).
void* psx_loop_create(const PsxLoopCfg* cfg, const char* runtime_path, const char* kernels_path) {
  void* rt = dlopen(runtime_path, RTLD_NOW | RTLD_NOLOAD);
  if (!rt) rt = dlopen(runtime_path, RTLD_NOW);
  void* kn = dlopen(kernels_path, RTLD_NOW | RTLD_NOLOAD);
  if (!kn) kn = dlopen(kernels_path, RTLD_NOW);
  if (!rt || !kn) {
    fprintf(stderr, "psx_loop_create: %s\n", dlerror());
    return nullptr;
  }
  PsxLoop* L = new PsxLoop();
  L->c = *cfg;
  Rt& r = L->rt;
  const bool ok = bind(rt, "psx_mbox_recv", &r.mbox_recv) && bind(rt, "psx_mbox_reply", &r.mbox_reply) &&
                  bind(rt, "psx_ps_register", &r.ps_register) && bind(rt, "psx_ps_heartbeat", &r.ps_heartbeat) &&
                  bind(rt, "psx_ps_on_fetch", &r.ps_on_fetch) && bind(rt, "psx_ps_on_push", &r.ps_on_push) &&
                  bind(rt, "psx_ps_on_applied", &r.ps_on_applied) &&
                  bind(rt, "psx_ps_record_update_time", &r.ps_record_update_time) &&
                  bind(rt, "psx_ps_job_finished", &r.ps_job_finished) && bind(rt, "psx_ps_mark_dead", &r.ps_mark_dead) &&
                  bind(rt, "psx_ps_check_timeouts", &r.ps_check_timeouts) &&
                  bind(rt, "psx_ps_global_step", &r.ps_global_step) && bind(kn, "psx_sgd_apply", &r.sgd_apply) &&
                  bind(kn, "psx_gather_f32", &r.gather_f32);
  if (!ok) {
    delete L;
    return nullptr;
  }
  const int n = cfg->max_wid;
  L->slot.assign(n, nullptr);
  L->s_comm.assign(n, nullptr);
  L->snap_img.assign(n, nullptr);
  L->snap_small.assign(n, nullptr);
  L->sent.assign(n, nullptr);
  L->sent_t.assign(n, 0.0);
  L->ws.assign(n, PsxLoop::WState{});
  return L;
}

int psx_loop_start(void* h) {
  PsxLoop* L = (PsxLoop*)h;
  L->th = std::thread(run, L);
  return 0;
}

// Blocks until the loop has ended; returns its error code (0 = clean).
int psx_loop_join(void* h) {
  PsxLoop* L = (PsxLoop*)h;
  if (L->th.joinable()) L->th.join();
  return L->err;
}

long long psx_loop_applies(void* h) { return ((PsxLoop*)h)->applies; }

// After join: the dropped workers (ids into out[cap]) and, per id, whether their pair
// communicator was aborted by the loop (aborted[cap], nullable: the caller must not destroy it).
int psx_loop_dropped(void* h, int* out, int* aborted, int cap) {
  PsxLoop* L = (PsxLoop*)h;
  int n = 0;
  for (size_t w = 0; w < L->ws.size(); ++w)
    if (L->ws[w].dead) {
      if (n < cap) {
        out[n] = (int)w;
        if (aborted) aborted[n] = L->ws[w].aborted ? 1 : 0;
      }
      ++n;
    }
  return n;
}

static int local_call(PsxLoop* L, LocalReq* r) {
  {
    std::unique_lock<std::mutex> lk(L->mu);
    if (L->stopped) return L->err ? L->err : -40;
    L->local.push_back(r);
    L->cv.wait(lk, [&] { return r->done || L->stopped; });
    if (!r->done) return L->err ? L->err : -41;
  }
  return L->err;
}

// Co-located worker push: `grads` is ready at the current point of `stream`; on return the
// update is enqueued and `stream` waits for it. out = [accepted, staleness, global_step].
int psx_loop_local_push(void* h, int wid, const void* grads, long long local_step, hipStream_t stream,
                        long long* out) {
  LocalReq r{0, wid, grads, nullptr, local_step, stream};
  const int e = local_call((PsxLoop*)h, &r);
  out[0] = r.accepted;
  out[1] = r.staleness;
  out[2] = r.global_step;
  return e;
}

// Co-located worker fetch: copies the whole fp32 arena (params + BN buffers, as the reference's
// fetch overwrites the worker's running statistics) into `dst` in order on `stream`; returns the
// global step (negative: error).
long long psx_loop_local_fetch(void* h, int wid, float* dst, hipStream_t stream) {
  LocalReq r{1, wid, nullptr, dst, 0, stream};
  const int e = local_call((PsxLoop*)h, &r);
  return e ? e : r.global_step;
}

int psx_loop_local_done(void* h, int wid) {
  LocalReq r{2, wid, nullptr, nullptr, 0, nullptr};
  return local_call((PsxLoop*)h, &r);
}

void psx_loop_destroy(void* h) {
  PsxLoop* L = (PsxLoop*)h;
  if (!L) return;
  if (L->th.joinable()) L->th.join();
  for (size_t w = 0; w < L->slot.size(); ++w) {
    if (L->ws[w].dead && L->s_comm[w] && hipStreamQuery(L->s_comm[w]) == hipErrorNotReady) {
      // a dropped worker's transfer never completed: keep its buffers (a late kernel may still
      // touch them) rather than free memory under it
      fprintf(stderr, "[psx native loop] worker %d: transfer still pending at teardown; buffers kept\n", (int)w);
      continue;
    }
    if (L->slot[w]) hipFree(L->slot[w]);
    if (L->snap_img[w]) hipFree(L->snap_img[w]);
    if (L->snap_small[w]) hipFree(L->snap_small[w]);
    if (L->sent[w]) hipEventDestroy(L->sent[w]);
  }
  for (size_t w = 0; w < L->s_comm.size(); ++w)
    if (L->s_comm[w] && !(L->ws[w].dead && hipStreamQuery(L->s_comm[w]) == hipErrorNotReady))
      hipStreamDestroy(L->s_comm[w]);
  if (L->img) hipFree(L->img);
  if (L->s_upd && L->c.own_upd_stream) hipStreamDestroy(L->s_upd);
  for (hipEvent_t ev : L->order)
    if (ev) hipEventDestroy(ev);
  for (auto& p : L->tfree) {
    hipEventDestroy(p.first);
    hipEventDestroy(p.second);
  }
  for (auto& p : L->tbusy) {  // the loop drained the update stream: these are complete
    hipEventDestroy(p.first);
    hipEventDestroy(p.second);
  }
  if (L->ckpt_ev) hipEventDestroy(L->ckpt_ev);
  delete L;
}

}  // extern "C"
