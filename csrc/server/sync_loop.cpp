// Native synchronous parameter-server rounds of the dedicated server rank (rank 0 of the
// 1 server + N-1 workers layout), on HIP streams.
//
// The reference's sync handler counts pushes under a lock and applies the average when the
// last worker's gradient arrives (reference: src/parameter_server/server.py:264-288, :145-169,
// :126-143); its workers then fetch the new state (:213-230). Here the server rank runs every
// round of the job inside ONE native call — no Python per round — issuing exactly the
// collective sequence the workers' sync channels issue (parallel/worker.py
// SyncCollectiveChannel, parallel/overlap.py OverlapSyncChannel):
//
//   serial round     fetch: broadcast of the fp32 arena (or of the WeightWire: bf16 image of the
//                    parameters + fp32 remainder, republished from the arena);
//                    push:  one group of ncclRecv, one per worker rank (every worker on its own
//                    xGMI link) -> sgd_apply_multi: the W wires decoded and summed in fp32 in
//                    worker order, p -= lr * sum / W (+ momentum / weight decay, + the image)
//   overlapped round per gradient bucket k (backward order): gather(k) on the communication
//                    stream; the apply of bucket k on the update stream once its gather is done,
//                    written straight into the bucket's fetch-wire segment (fp32: the arena slice
//                    itself is broadcast; bf16conv: the apply writes the bf16 image into the
//                    segment and the fp32 entries are gathered after it), then broadcast(k) on
//                    the communication stream — gather(k+1) is already queued ahead of it, as on
//                    the workers. The first round starts with one broadcast of the whole wire.
//
// The native core (csrc/runtime/ps_core.cpp) records every round: on_fetch / on_push per member
// (the wait-for-N barrier completes on the last), on_applied. Checkpoints (--ckpt-every) call
// back into the host after an event wait on the round's apply. At most two rounds are in flight
// on the device (the host waits for round r-2's completion event), and the number of rounds
// whose device work has completed is published for the liveness watchdog
// (parallel/liveness.py RoundWatchdog polls psx_sync_progress). Every HIP call is checked.
//
// Events are created once per loop, not per call: a ring of ordering events (a wait enqueued on
// a stream captures the event's record at call time, so an event is re-recordable right after),
// one receive event per bucket, and per in-flight round slot its completion event plus a timing
// pair around every apply range. The update time the core reports
// (average_update_time_seconds, reference server.py:128,140-141) is the DEVICE time of the
// round's apply kernels, read when the round retires — not the host's launch time.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <mutex>
#include <vector>

#include "psx_comm.h"

namespace {

enum { PSX_APPLY_ = 1 };

struct SyncRt {
  long long (*ps_on_fetch)(void*, int, double);
  int (*ps_on_push)(void*, int, long long, double, float*, int*, long long*);
  void (*ps_on_applied)(void*, double);
  void (*ps_record_update_time)(void*, double);
  long long (*ps_global_step)(void*);
  int (*sgd_apply_multi)(float*, const void* const*, int, float*, long, float, float, float, float, int, int, void*,
                         hipStream_t);
  int (*gather_f32)(const float*, const long*, long, float*, hipStream_t);
};

template <typename F>
bool bindf(void* lib, const char* name, F* fn) {
  *fn = reinterpret_cast<F>(dlsym(lib, name));
  if (!*fn) fprintf(stderr, "psx sync loop: missing symbol %s\n", name);
  return *fn != nullptr;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

}  // namespace

// One gradient bucket of the overlapped round (mirrors parallel/overlap.py Bucket + BucketWire).
struct PsxSyncBucket {
  long lo, hi;          // parameter range [lo, hi)
  void* seg;            // its fetch-wire segment (device)
  long seg_bytes;       // bytes broadcast (the workers' segment size)
  const long* small;    // bf16conv: device arena indices of the fp32 entries (nullptr: fp32 kind)
  long nsmall;
  float* seg_small;     // bf16conv: where they go in the segment
};

struct PsxSyncCfg {  // mirrored by parallel/native_sync.py (ctypes.Structure)
  void* comm;           // the job communicator (rank 0 = this server)
  void* core;
  float* arena;         // fp32 master arena (params | buffers)
  long n_params, arena_numel;
  int nworkers;         // worker ranks 1..nworkers (dedicated topology: world = nworkers + 1)
  const int* members;   // worker ids of the round, in core order [nworkers]
  void* const* gbufs;   // per worker rank 1..nworkers: its gathered gradient wire [nworkers]
  int grad_fp16;
  float lr, momentum, weight_decay;
  float* mom_buf;
  int mom_first;
  // fetch payload of the serial round: 0 = the fp32 arena (broadcast in place); 1 = WeightWire
  int image;
  void* wire_buf;       // WeightWire: [bf16 image | fp32 remainder] (device)
  long wire_bytes;
  uint16_t* wire_img;   // its image part (the apply writes it)
  const long* small_idx;  // its remainder's arena indices
  long small_n;
  float* wire_small;
  // overlapped round (nbuckets > 0): buckets in backward order, the first round's whole-wire
  // broadcast, the BN-buffer segment
  int nbuckets;
  const PsxSyncBucket* buckets;
  void* full_wire;
  long full_wire_bytes;
  int primed;           // the first round's full fetch already happened (resume of a channel)
  hipStream_t upd_stream;   // compute / update stream of the server rank
  hipStream_t comm_stream;  // the overlapped round's communication stream
  long long ckpt_every;
  int (*ckpt_cb)(long long global_step);
  // sync job that survives a lost worker (parallel/elastic.py; nullable): 3 arena snapshots, one
  // per in-flight round slot, each taken at its round's start (stream order: after the previous
  // round's apply) — the state a shrunk job resumes from without a checkpoint rollback
  float* snap;
  float* snap_mom;  // momentum buffer snapshots (3 x n_params; nullable)
};

// one round in flight: its completion event and the timing events around its apply ranges
struct PsxSyncSlot {
  hipEvent_t done = nullptr;
  std::vector<hipEvent_t> t0, t1;  // [max(1, nbuckets)]
  int nt = 0;                      // ranges timed this round
  // per-phase device ranges of the round (psx_sync_phase_us): gather g0/g1 (receive posted ->
  // every worker's wire landed, so it includes waiting for the workers' step) and broadcast
  // c0/c1, one pair per bucket (+1: the first round's whole-wire broadcast); the apply is t0/t1
  std::vector<hipEvent_t> g0, g1, c0, c1;
  int ng = 0, nc = 0;
};

struct PsxSync {
  PsxSyncCfg c;
  SyncRt rt;
  std::atomic<long long> issued{0}, done{0};
  enum { NSLOT = 3, NORDER = 16 };  // at most two rounds in flight + the one being issued
  PsxSyncSlot slot[NSLOT];
  int cur = 0;                 // slot of the round being issued
  std::deque<int> inflight;    // slots of issued rounds not yet retired
  hipEvent_t order[NORDER] = {};
  int order_pos = 0;
  std::vector<hipEvent_t> got;  // per bucket: its gather landed (comm stream)
  hipEvent_t ckpt_ev = nullptr;
  int err = 0;
  // psx_sync_abort (the liveness watchdog's thread): from then on no round counts as done and no
  // new round is issued; `good` = rounds retired before it
  std::mutex mu;
  std::atomic<int> aborting{0};
  long long good = -1;
  int mom_first0 = 0;  // mom_first at creation (a rollback to round 0 restores it)
  // retired rounds' device time per phase, us: [gather, apply, broadcast] (under mu)
  double ph_us[3] = {0, 0, 0};
  long long ph_rounds = 0;
};

namespace {

#define PSX_SHIP(S, call)                                                                        \
  do {                                                                                           \
    const hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "psx sync loop: %s failed: %s\n", #call, hipGetErrorString(e_));            \
      if (!(S)->err) (S)->err = -50;                                                             \
    }                                                                                            \
  } while (0)

#define PSX_SCOMM(S, call)                                                                       \
  do {                                                                                           \
    const int e_ = (call);                                                                       \
    if (e_ && !(S)->err) {                                                                       \
      fprintf(stderr, "psx sync loop: %s failed (%d)\n", #call, e_);                             \
      (S)->err = -60;                                                                            \
    }                                                                                            \
  } while (0)

// stream a waits for everything enqueued on b so far (an event of the ordering ring)
void after(PsxSync* S, hipStream_t a, hipStream_t b) {
  hipEvent_t ev = S->order[S->order_pos];
  S->order_pos = (S->order_pos + 1) % PsxSync::NORDER;
  PSX_SHIP(S, hipEventRecord(ev, b));
  PSX_SHIP(S, hipStreamWaitEvent(a, ev, 0));
}

// the round of slot k finished on the device: its apply time (sum of its timed ranges) goes
// to the core's update-time statistics. After an abort a finished event means nothing (the
// aborted collectives let the stream run on): such rounds are not counted.
void retire_slot(PsxSync* S, int k) {
  PsxSyncSlot& sl = S->slot[k];
  std::lock_guard<std::mutex> lk(S->mu);
  if (S->aborting.load()) {
    sl.nt = 0;
    return;
  }
  double sec = 0;
  for (int i = 0; i < sl.nt; ++i) {
    float ms = 0.f;
    PSX_SHIP(S, hipEventElapsedTime(&ms, sl.t0[i], sl.t1[i]));
    sec += 1e-3 * (double)ms;
  }
  if (sl.nt) S->rt.ps_record_update_time(S->c.core, sec);
  auto span_us = [&](const std::vector<hipEvent_t>& a, const std::vector<hipEvent_t>& b, int n) {
    double us = 0;
    for (int i = 0; i < n; ++i) {
      float ms = 0.f;
      PSX_SHIP(S, hipEventElapsedTime(&ms, a[i], b[i]));
      us += 1e3 * (double)ms;
    }
    return us;
  };
  S->ph_us[0] += span_us(sl.g0, sl.g1, sl.ng);
  S->ph_us[1] += 1e6 * sec;
  S->ph_us[2] += span_us(sl.c0, sl.c1, sl.nc);
  S->ph_rounds++;
  sl.nt = sl.ng = sl.nc = 0;
  S->done.fetch_add(1);
}

// rounds whose device work finished (host-side bookkeeping of the in-flight slots)
void retire(PsxSync* S, size_t keep) {
  while (S->inflight.size() > keep) {
    const int k = S->inflight.front();
    PSX_SHIP(S, hipEventSynchronize(S->slot[k].done));
    S->inflight.pop_front();
    retire_slot(S, k);
  }
  while (!S->inflight.empty() && hipEventQuery(S->slot[S->inflight.front()].done) == hipSuccess) {
    const int k = S->inflight.front();
    S->inflight.pop_front();
    retire_slot(S, k);
  }
}

void gather(PsxSync* S, long lo, long n, hipStream_t st) {
  const int dt = S->c.grad_fp16 ? PSX_F16 : PSX_F32;
  const size_t es = S->c.grad_fp16 ? 2 : 4;
  PsxSyncSlot& sl = S->slot[S->cur];
  const bool timed = sl.ng < (int)sl.g0.size();
  if (timed) PSX_SHIP(S, hipEventRecord(sl.g0[sl.ng], st));
  PSX_SCOMM(S, psx_comm_group_start());
  for (int r = 1; r <= S->c.nworkers; ++r)
    PSX_SCOMM(S, psx_comm_recv(S->c.comm, (char*)S->c.gbufs[r - 1] + lo * es, n, dt, r, st));
  PSX_SCOMM(S, psx_comm_group_end());
  if (timed) PSX_SHIP(S, hipEventRecord(sl.g1[sl.ng++], st));
}

// a broadcast of the round, device-timed (phase 2)
void bcast(PsxSync* S, void* buf, long n, int dt, hipStream_t st) {
  PsxSyncSlot& sl = S->slot[S->cur];
  const bool timed = sl.nc < (int)sl.c0.size();
  if (timed) PSX_SHIP(S, hipEventRecord(sl.c0[sl.nc], st));
  PSX_SCOMM(S, psx_comm_broadcast(S->c.comm, buf, n, dt, 0, st));
  if (timed) PSX_SHIP(S, hipEventRecord(sl.c1[sl.nc++], st));
}

// p[lo:hi] -= lr * sum_k g_k[lo:hi] / W (+ momentum / wd), image (nullable) of the range
void apply_range(PsxSync* S, long lo, long hi, void* img, hipStream_t st) {
  const size_t es = S->c.grad_fp16 ? 2 : 4;
  std::vector<const void*> srcs(S->c.nworkers);
  for (int k = 0; k < S->c.nworkers; ++k) srcs[k] = (const char*)S->c.gbufs[k] + lo * es;
  PsxSyncSlot& sl = S->slot[S->cur];
  const bool timed = sl.nt < (int)sl.t0.size();
  if (timed) PSX_SHIP(S, hipEventRecord(sl.t0[sl.nt], st));
  // the kernel wrappers report hipGetLastError(): clear a hipErrorNotReady of an earlier
  // hipEventQuery (retire) from this thread's error slot
  (void)hipGetLastError();
  if (S->rt.sgd_apply_multi(S->c.arena + lo, srcs.data(), S->c.nworkers, S->c.mom_buf ? S->c.mom_buf + lo : nullptr,
                            hi - lo, S->c.lr, 1.f / (float)S->c.nworkers, S->c.momentum, S->c.weight_decay,
                            S->c.mom_first, S->c.grad_fp16, img, st) &&
      !S->err)
    S->err = -61;
  if (timed) PSX_SHIP(S, hipEventRecord(sl.t1[sl.nt++], st));
}

// the core's bookkeeping of one completed round (every member pushed, the barrier completes on
// the last) + the checkpoint hook
void record_round(PsxSync* S) {
  float w = 0.f;
  int nc = 0;
  long long st = 0;
  int d = 0;
  const long long gs = S->rt.ps_global_step(S->c.core);
  for (int k = 0; k < S->c.nworkers; ++k) d = S->rt.ps_on_push(S->c.core, S->c.members[k], gs, now_s(), &w, &nc, &st);
  if (d != PSX_APPLY_ && !S->err) {
    fprintf(stderr, "psx sync loop: the round did not complete on the core (decision %d)\n", d);
    S->err = -62;
  }
  S->rt.ps_on_applied(S->c.core, -1.0);  // the apply's device time follows when the round retires
  S->c.mom_first = 0;
  const long long g2 = S->rt.ps_global_step(S->c.core);
  if (S->c.ckpt_cb && S->c.ckpt_every > 0 && g2 % S->c.ckpt_every == 0) {
    // the apply of this round, not the whole stream
    PSX_SHIP(S, hipEventRecord(S->ckpt_ev, S->c.upd_stream));
    PSX_SHIP(S, hipEventSynchronize(S->ckpt_ev));
    if (S->c.ckpt_cb(g2) && !S->err) S->err = -63;
  }
}

void fetch_bookkeeping(PsxSync* S) {
  for (int k = 0; k < S->c.nworkers; ++k) S->rt.ps_on_fetch(S->c.core, S->c.members[k], now_s());
}

// elastic: this round's starting state into its slot's snapshot
void snapshot(PsxSync* S, hipStream_t st) {
  if (!S->c.snap) return;
  PSX_SHIP(S, hipMemcpyAsync(S->c.snap + (size_t)S->cur * S->c.arena_numel, S->c.arena,
                             (size_t)S->c.arena_numel * 4, hipMemcpyDeviceToDevice, st));
  if (S->c.snap_mom && S->c.mom_buf)
    PSX_SHIP(S, hipMemcpyAsync(S->c.snap_mom + (size_t)S->cur * S->c.n_params, S->c.mom_buf,
                               (size_t)S->c.n_params * 4, hipMemcpyDeviceToDevice, st));
}

void serial_round(PsxSync* S) {
  hipStream_t st = S->c.upd_stream;
  snapshot(S, st);
  fetch_bookkeeping(S);
  if (S->c.image) {
    (void)hipGetLastError();
    if (S->c.small_n && S->rt.gather_f32(S->c.arena, S->c.small_idx, S->c.small_n, S->c.wire_small, st) && !S->err)
      S->err = -64;
    bcast(S, S->c.wire_buf, S->c.wire_bytes, PSX_U8, st);
  } else {
    bcast(S, S->c.arena, S->c.arena_numel, PSX_F32, st);
  }
  gather(S, 0, S->c.n_params, st);
  if (S->err) return;  // a failed gather is never applied
  apply_range(S, 0, S->c.n_params, S->c.image ? S->c.wire_img : nullptr, st);
  record_round(S);
}

void overlap_round(PsxSync* S) {
  hipStream_t cs = S->c.comm_stream, us = S->c.upd_stream;
  snapshot(S, us);
  fetch_bookkeeping(S);
  if (!S->c.primed) {  // first round: the whole wire (every segment + the BN buffers), packed by the host
    after(S, cs, us);
    bcast(S, S->c.full_wire, S->c.full_wire_bytes, PSX_U8, cs);
    S->c.primed = 1;
  }
  std::vector<hipEvent_t>& got = S->got;
  auto issue_gather = [&](int k) {
    const PsxSyncBucket& b = S->c.buckets[k];
    after(S, cs, us);  // the previous apply of this range (and the wire pack) before new data lands
    gather(S, b.lo, b.hi - b.lo, cs);
    PSX_SHIP(S, hipEventRecord(got[k], cs));
  };
  auto finish = [&](int k) {  // apply (+ segment pack) on the update stream, broadcast on cs
    if (S->err) return;  // a failed gather is never applied
    const PsxSyncBucket& b = S->c.buckets[k];
    PSX_SHIP(S, hipStreamWaitEvent(us, got[k], 0));
    if (b.small) {  // bf16conv segment: the apply writes the bf16 image, then the fp32 entries
      apply_range(S, b.lo, b.hi, b.seg, us);
      (void)hipGetLastError();
      if (b.nsmall && S->rt.gather_f32(S->c.arena, b.small, b.nsmall, b.seg_small, us) && !S->err) S->err = -64;
      after(S, cs, us);
      bcast(S, b.seg, b.seg_bytes, PSX_U8, cs);
    } else {  // fp32 segment = the arena slice itself, broadcast in place
      apply_range(S, b.lo, b.hi, nullptr, us);
      after(S, cs, us);
      bcast(S, S->c.arena + b.lo, b.seg_bytes, PSX_U8, cs);
    }
  };
  for (int k = 0; k < S->c.nbuckets; ++k) {
    issue_gather(k);
    if (k > 0) finish(k - 1);
  }
  finish(S->c.nbuckets - 1);
  after(S, us, cs);  // the round ends when its broadcasts are done (next round's applies after them)
  record_round(S);
}

}  // namespace

extern "C" {

void psx_sync_destroy(void* h);

int psx_sync_cfg_size() { return (int)sizeof(PsxSyncCfg); }
int psx_sync_bucket_size() { return (int)sizeof(PsxSyncBucket); }

void* psx_sync_create(const PsxSyncCfg* cfg, const char* runtime_path, const char* kernels_path) {
  void* rt = dlopen(runtime_path, RTLD_NOW | RTLD_NOLOAD);
  if (!rt) rt = dlopen(runtime_path, RTLD_NOW);
  void* kn = dlopen(kernels_path, RTLD_NOW | RTLD_NOLOAD);
  if (!kn) kn = dlopen(kernels_path, RTLD_NOW);
  if (!rt || !kn) {
    fprintf(stderr, "psx_sync_create: %s\n", dlerror());
    return nullptr;
  }
  if (cfg->nworkers < 1 || cfg->nworkers > 32 || !cfg->comm ||
      (cfg->nbuckets > 0 && (!cfg->buckets || !cfg->comm_stream || !cfg->full_wire))) {
    fprintf(stderr, "psx_sync_create: invalid configuration\n");
    return nullptr;
  }
  PsxSync* S = new PsxSync();
  S->c = *cfg;
  S->mom_first0 = cfg->mom_first;
  SyncRt& r = S->rt;
  const bool ok = bindf(rt, "psx_ps_on_fetch", &r.ps_on_fetch) && bindf(rt, "psx_ps_on_push", &r.ps_on_push) &&
                  bindf(rt, "psx_ps_on_applied", &r.ps_on_applied) &&
                  bindf(rt, "psx_ps_record_update_time", &r.ps_record_update_time) &&
                  bindf(rt, "psx_ps_global_step", &r.ps_global_step) &&
                  bindf(kn, "psx_sgd_apply_multi", &r.sgd_apply_multi) && bindf(kn, "psx_gather_f32", &r.gather_f32);
  if (!ok) {
    delete S;
    return nullptr;
  }
  // the loop's events, created once (see the header)
  bool ev_ok = hipEventCreateWithFlags(&S->ckpt_ev, hipEventDisableTiming) == hipSuccess;
  for (int i = 0; i < PsxSync::NORDER; ++i)
    ev_ok = ev_ok && hipEventCreateWithFlags(&S->order[i], hipEventDisableTiming) == hipSuccess;
  S->got.assign(std::max(0, cfg->nbuckets), nullptr);
  for (auto& e : S->got) ev_ok = ev_ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  const int nt = std::max(1, cfg->nbuckets);
  for (PsxSyncSlot& sl : S->slot) {
    ev_ok = ev_ok && hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
    for (auto* v : {&sl.t0, &sl.t1, &sl.g0, &sl.g1, &sl.c0, &sl.c1}) {
      v->assign(v == &sl.c0 || v == &sl.c1 ? nt + 1 : nt, nullptr);
      for (auto& e : *v) ev_ok = ev_ok && hipEventCreate(&e) == hipSuccess;
    }
  }
  if (!ev_ok) {
    fprintf(stderr, "psx_sync_create: hipEventCreate failed\n");
    psx_sync_destroy(S);
    return nullptr;
  }
  return S;
}

// Runs `rounds` sync rounds (blocking the calling thread; ctypes releases the GIL) and returns
// 0 or the first error. The device work of the last round may still be in flight on return
// (psx_sync_drain waits for it).
int psx_sync_run(void* h, long long rounds) {
  PsxSync* S = (PsxSync*)h;
  // relaxed capture mode while the loop runs (its event waits never invalidate a capture on
  // another thread); the caller's mode is restored on return
  hipStreamCaptureMode cm = hipStreamCaptureModeRelaxed;
  PSX_SHIP(S, hipThreadExchangeStreamCaptureMode(&cm));
  for (long long r = 0; r < rounds && !S->err; ++r) {
    if (S->aborting.load()) {  // the watchdog aborted the communicator: issue nothing more
      S->err = -65;
      break;
    }
    PsxSyncSlot& sl = S->slot[S->cur];
    sl.nt = sl.ng = sl.nc = 0;
    if (S->c.nbuckets > 0)
      overlap_round(S);
    else
      serial_round(S);
    if (S->err) break;  // a round that failed to issue is neither counted nor retired
    PSX_SHIP(S, hipEventRecord(S->slot[S->cur].done, S->c.upd_stream));
    S->inflight.push_back(S->cur);
    S->issued.fetch_add(1);
    retire(S, 2);  // at most two rounds in flight on the device: the next slot is free
    S->cur = (S->cur + 1) % PsxSync::NSLOT;
  }
  hipStreamCaptureMode prev = cm;
  PSX_SHIP(S, hipThreadExchangeStreamCaptureMode(&prev));
  return S->err;
}

int psx_sync_drain(void* h) {
  PsxSync* S = (PsxSync*)h;
  retire(S, 0);
  return S->err;
}

// [rounds issued, rounds whose device work completed] (the liveness watchdog's progress)
void psx_sync_progress(void* h, long long* out) {
  PsxSync* S = (PsxSync*)h;
  out[0] = S->issued.load();
  out[1] = S->done.load();
}

int psx_sync_mom_first(void* h) { return ((PsxSync*)h)->c.mom_first; }

// Device time of the retired rounds per phase: out = [rounds, gather us, apply us, broadcast us]
// (sums; the gather range runs from the receives' post to the last worker's wire landing, so it
// holds the workers' step; with bucketed overlap the phases of different buckets overlap).
void psx_sync_phase_us(void* h, double* out) {
  PsxSync* S = (PsxSync*)h;
  std::lock_guard<std::mutex> lk(S->mu);
  out[0] = (double)S->ph_rounds;
  for (int i = 0; i < 3; ++i) out[1 + i] = S->ph_us[i];
}

// Liveness watchdog (another thread): freezes the count of rounds known good, stops the loop from
// issuing more and aborts the communicator (the blocked loop thread then runs out). Returns the
// good count.
long long psx_sync_abort(void* h) {
  PsxSync* S = (PsxSync*)h;
  {
    std::lock_guard<std::mutex> lk(S->mu);
    if (!S->aborting.load()) {
      S->good = S->done.load();
      S->aborting.store(1);
    }
  }
  psx_comm_abort(S->c.comm);
  return S->good;
}

// After a failed or aborted run: waits for the streams, restores the arena (and momentum) to the
// start of the first round not known good and returns the number of rounds kept (of this loop's
// lifetime). -1: no snapshots configured.
long long psx_sync_rollback(void* h) {
  PsxSync* S = (PsxSync*)h;
  if (!S->c.snap) return -1;
  (void)hipStreamSynchronize(S->c.upd_stream);
  if (S->c.comm_stream) (void)hipStreamSynchronize(S->c.comm_stream);
  retire(S, 0);  // rounds finished before an error (not after an abort) still count
  const long long g = S->aborting.load() ? S->good : S->done.load();
  const int k = (int)(g % PsxSync::NSLOT);
  if (hipMemcpy(S->c.arena, S->c.snap + (size_t)k * S->c.arena_numel, (size_t)S->c.arena_numel * 4,
                hipMemcpyDeviceToDevice) != hipSuccess)
    return -2;
  if (S->c.snap_mom && S->c.mom_buf &&
      hipMemcpy(S->c.mom_buf, S->c.snap_mom + (size_t)k * S->c.n_params, (size_t)S->c.n_params * 4,
                hipMemcpyDeviceToDevice) != hipSuccess)
    return -2;
  if (g == 0) S->c.mom_first = S->mom_first0;
  return g;
}
int psx_sync_primed(void* h) { return ((PsxSync*)h)->c.primed; }

void psx_sync_destroy(void* h) {
  PsxSync* S = (PsxSync*)h;
  if (!S) return;
  if (!S->inflight.empty()) retire(S, 0);  // no event is destroyed under a pending record
  if (S->ckpt_ev) hipEventDestroy(S->ckpt_ev);
  for (hipEvent_t ev : S->order)
    if (ev) hipEventDestroy(ev);
  for (hipEvent_t ev : S->got)
    if (ev) hipEventDestroy(ev);
  for (PsxSyncSlot& sl : S->slot) {
    if (sl.done) hipEventDestroy(sl.done);
    for (auto* v : {&sl.t0, &sl.t1, &sl.g0, &sl.g1, &sl.c0, &sl.c1})
      for (hipEvent_t ev : *v)
        if (ev) hipEventDestroy(ev);
  }
  delete S;
}

}  // extern "C"
