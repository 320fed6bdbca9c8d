// psx parameter-server core state machine (see ps_core.h for the contract).
#include "ps_core.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace {

struct WorkerInfo {
  std::string name;
  double registered_at = 0, last_seen = 0;
  bool active = true;  // registered and not finished
  bool dead = false;   // timed out / declared dead
  int64_t pushes = 0;
  int64_t last_staleness = -1;
  bool has_staleness = false;
};

struct PsCore {
  std::mutex mu;
  int mode, total_workers, staleness_bound, semantics;
  float lr;
  double start_time = -1;
  int next_id = 0;
  std::map<int, WorkerInfo> workers;
  int64_t global_step = 0, total_updates = 0, gradients_processed = 0, async_updates = 0;
  // sync barrier: rounds completed at APPLY time (global_step follows in on_applied), so a late
  // push for a round that already completed is recognised as stale, never counted twice
  int64_t rounds_done = 0;
  int64_t rejected = 0, duplicates = 0;
  // sync round
  std::set<int> round;          // barrier semantics: distinct contributors
  std::map<int, int> ref_round;  // reference semantics: worker -> pushes this round
  int ref_count = 0;
  std::vector<int> last_members;
  // stats
  std::vector<double> update_times;  // ring of the last 100 (reference deque(maxlen=100))
  size_t ut_pos = 0;
  std::vector<int64_t> hist;  // accepted staleness histogram, last bucket = overflow
  double stale_sum = 0;
  int64_t stale_n = 0;

  int live_count() const {
    int n = 0;
    for (auto& kv : workers)
      if (kv.second.active && !kv.second.dead) ++n;
    return n;
  }
  // Barrier is complete when every expected, live worker has contributed. Before all
  // expected workers registered, unregistered slots count as outstanding.
  bool barrier_complete() const {
    if (round.empty()) return false;
    int registered = (int)workers.size();
    int outstanding = std::max(0, total_workers - registered);
    if (outstanding > 0) return false;
    for (auto& kv : workers) {
      const WorkerInfo& w = kv.second;
      if (w.active && !w.dead && !round.count(kv.first)) return false;
    }
    return true;
  }
};

PsCore* P(void* h) { return reinterpret_cast<PsCore*>(h); }

}  // namespace

extern "C" {

void* psx_ps_create(int mode, int total_workers, float lr, int staleness_bound, int sync_semantics) {
  auto* c = new PsCore();
  c->mode = mode;
  c->total_workers = total_workers;
  c->lr = lr;
  c->staleness_bound = staleness_bound;
  c->semantics = sync_semantics;
  c->hist.assign(std::max(2, staleness_bound + 2), 0);
  return c;
}

void psx_ps_destroy(void* h) { delete P(h); }

int psx_ps_register(void* h, const char* name, int requested_id, double now) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  if (c->start_time < 0) c->start_time = now;
  int id = requested_id;
  if (id < 0) {
    id = c->next_id++;
  } else {
    c->next_id = std::max(c->next_id, id + 1);
  }
  WorkerInfo& w = c->workers[id];
  w.name = name ? name : "";
  w.registered_at = now;
  w.last_seen = now;
  w.active = true;
  w.dead = false;
  return id;
}

void psx_ps_heartbeat(void* h, int wid, double now) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->workers.find(wid);
  if (it != c->workers.end()) it->second.last_seen = now;
}

int64_t psx_ps_on_fetch(void* h, int wid, double now) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->workers.find(wid);
  if (it != c->workers.end()) it->second.last_seen = now;
  return c->global_step;
}

int psx_ps_on_push(void* h, int wid, int64_t local_step, double now, float* weight, int* ncontrib,
                   int64_t* staleness) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->workers.find(wid);
  if (it == c->workers.end() || it->second.dead) return PSX_UNKNOWN;
  WorkerInfo& w = it->second;
  w.last_seen = now;
  w.pushes++;
  c->gradients_processed++;
  if (weight) *weight = 1.f;
  if (ncontrib) *ncontrib = 1;
  if (staleness) *staleness = 0;

  if (c->mode == PSX_ASYNC) {
    const int64_t s = c->global_step - local_step;
    if (staleness) *staleness = s;
    w.last_staleness = s;  // the reference records rejected pushes too (server.py:300)
    w.has_staleness = true;
    if (s > c->staleness_bound) {
      c->rejected++;
      return PSX_REJECT;
    }
    const size_t b = std::min<size_t>((size_t)std::max<int64_t>(s, 0), c->hist.size() - 1);
    c->hist[b]++;
    c->stale_sum += (double)s;
    c->stale_n++;
    if (weight) *weight = std::max(0.1f, 1.f / (1.f + 0.1f * (float)s));
    c->async_updates++;
    return PSX_APPLY;
  }

  if (c->semantics == PSX_REFERENCE) {
    c->ref_round[wid]++;
    c->ref_count++;
    if (c->ref_count >= c->total_workers) {
      const int n = (int)c->ref_round.size();
      c->last_members.clear();
      for (auto& kv : c->ref_round) c->last_members.push_back(kv.first);
      c->ref_round.clear();
      c->ref_count = 0;
      if (weight) *weight = 1.f / (float)n;
      if (ncontrib) *ncontrib = n;
      return PSX_APPLY;
    }
    return PSX_WAIT;
  }

  // true wait-for-N barrier over live workers
  if (local_step < c->rounds_done || c->round.count(wid)) {
    c->duplicates++;
    return PSX_DUPLICATE;
  }
  c->round.insert(wid);
  if (c->barrier_complete()) {
    const int n = (int)c->round.size();
    c->last_members.assign(c->round.begin(), c->round.end());
    c->round.clear();
    c->rounds_done++;
    if (weight) *weight = 1.f / (float)n;
    if (ncontrib) *ncontrib = n;
    return PSX_APPLY;
  }
  return PSX_WAIT;
}

int psx_ps_round_members(void* h, int* out, int cap) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  const int n = (int)c->last_members.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = c->last_members[i];
  return n;
}

static void record_update_time(PsCore* c, double seconds) {
  if (c->update_times.size() < 100) {
    c->update_times.push_back(seconds);
  } else {
    c->update_times[c->ut_pos] = seconds;
    c->ut_pos = (c->ut_pos + 1) % 100;
  }
}

void psx_ps_on_applied(void* h, double update_seconds) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  c->global_step++;
  c->total_updates++;
  if (update_seconds >= 0) record_update_time(c, update_seconds);
}

void psx_ps_record_update_time(void* h, double update_seconds) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  if (update_seconds >= 0) record_update_time(c, update_seconds);
}

int psx_ps_job_finished(void* h, int wid) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->workers.find(wid);
  if (it != c->workers.end()) it->second.active = false;
  for (auto& kv : c->workers)
    if (kv.second.active && !kv.second.dead) return 0;
  return 1;
}

int psx_ps_mark_dead(void* h, int wid) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  auto it = c->workers.find(wid);
  if (it == c->workers.end()) return 0;
  it->second.dead = true;
  c->round.erase(wid);
  return c->barrier_complete() ? 1 : 0;
}

int psx_ps_check_timeouts(void* h, double now, double timeout, int* dead, int cap) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  int n = 0;
  for (auto& kv : c->workers) {
    WorkerInfo& w = kv.second;
    if (w.active && !w.dead && now - w.last_seen > timeout) {
      w.dead = true;
      c->round.erase(kv.first);
      if (n < cap) dead[n] = kv.first;
      ++n;
    }
  }
  return n;
}

int psx_ps_sync_ready(void* h) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  return c->barrier_complete() ? 1 : 0;
}

int64_t psx_ps_global_step(void* h) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  return c->global_step;
}

void psx_ps_set_global_step(void* h, int64_t s) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  c->global_step = s;
  c->rounds_done = s;
}

// Sync job shrunk after a lost worker (parallel/elastic.py): the rounds after `step` were rolled
// back on the device, so they leave the step and update counts too.
void psx_ps_rollback_to(void* h, int64_t step) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  if (step < c->global_step) c->total_updates -= c->global_step - step;
  c->global_step = step;
  c->rounds_done = step;
  c->round.clear();
}

int psx_ps_num_active(void* h) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  return c->live_count();
}

static double r2(double v) { return std::round(v * 100.0) / 100.0; }
static double r4(double v) { return std::round(v * 10000.0) / 10000.0; }

int psx_ps_metrics_json(void* h, double now, char* buf, int cap) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  const double total = c->start_time < 0 ? 0.0 : now - c->start_time;
  double avg_ut = 0;
  for (double t : c->update_times) avg_ut += t;
  if (!c->update_times.empty()) avg_ut /= (double)c->update_times.size();
  const double ups = total > 0 ? (double)c->total_updates / total : 0.0;
  std::string s;
  char tmp[512];
  snprintf(tmp, sizeof(tmp),
           "{\"type\": \"SERVER_FINAL_METRICS\", \"mode\": \"%s\", \"total_workers\": %d, "
           "\"total_training_time_seconds\": %.2f, \"global_steps_completed\": %lld, "
           "\"total_parameter_updates\": %lld, \"gradients_processed\": %lld, "
           "\"average_update_time_seconds\": %.4f, \"updates_per_second\": %.2f, \"learning_rate\": %g",
           c->mode == PSX_ASYNC ? "async" : "sync", c->total_workers, r2(total), (long long)c->global_step,
           (long long)c->total_updates, (long long)c->gradients_processed, r4(avg_ut), r2(ups), (double)c->lr);
  s += tmp;
  if (c->mode == PSX_ASYNC) {
    double sum = 0;
    int64_t mx = 0;
    int n = 0;
    for (auto& kv : c->workers)
      if (kv.second.has_staleness) {
        sum += (double)kv.second.last_staleness;
        mx = n == 0 ? kv.second.last_staleness : std::max(mx, kv.second.last_staleness);
        ++n;
      }
    if (n > 0) {
      snprintf(tmp, sizeof(tmp),
               ", \"async_updates\": %lld, \"average_gradient_staleness\": %.2f, \"max_staleness_observed\": %lld",
               (long long)c->async_updates, r2(sum / n), (long long)mx);
      s += tmp;
    }
    snprintf(tmp, sizeof(tmp), ", \"staleness_bound\": %d, \"rejected_pushes\": %lld, \"mean_staleness_all\": %.3f",
             c->staleness_bound, (long long)c->rejected, c->stale_n ? c->stale_sum / (double)c->stale_n : 0.0);
    s += tmp;
    s += ", \"staleness_histogram\": [";
    for (size_t i = 0; i < c->hist.size(); ++i) {
      snprintf(tmp, sizeof(tmp), "%s%lld", i ? ", " : "", (long long)c->hist[i]);
      s += tmp;
    }
    s += "]";
  } else {
    snprintf(tmp, sizeof(tmp), ", \"sync_semantics\": \"%s\", \"duplicate_pushes\": %lld",
             c->semantics == PSX_REFERENCE ? "reference" : "barrier", (long long)c->duplicates);
    s += tmp;
  }
  int dead = 0;
  for (auto& kv : c->workers) dead += kv.second.dead ? 1 : 0;
  snprintf(tmp, sizeof(tmp), ", \"dead_workers\": %d}", dead);
  s += tmp;
  const int n = (int)s.size();
  if (buf && cap > 0) {
    const int m = std::min(n, cap - 1);
    memcpy(buf, s.data(), (size_t)m);
    buf[m] = 0;
  }
  return n;
}

int psx_ps_staleness_hist(void* h, int64_t* out, int cap) {
  PsCore* c = P(h);
  std::lock_guard<std::mutex> g(c->mu);
  const int n = (int)c->hist.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = c->hist[i];
  return n;
}

}  // extern "C"
