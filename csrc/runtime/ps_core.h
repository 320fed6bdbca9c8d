// psx parameter-server core: the host-side state machine of the server role.
//
// It owns every decision the reference ParameterServerServicer makes
// (reference: src/parameter_server/server.py:81-368) while the data plane (gradient
// receive, aggregation kernels, RCCL reduce/broadcast/send/recv) lives on the GPU:
//   * worker registry with rank-stable ids (fixes the reference's ever-increasing id,
//     server.py:193-194) and heartbeat / timeout-based failure detection;
//   * sync mode: a true wait-for-N barrier over *live* workers (default) or the reference's
//     count-triggered semantics (server.py:264-288) for comparison;
//   * async mode: staleness = global_step - local_step, reject if > bound, weight
//     max(0.1, 1/(1+0.1 s)) (server.py:171-186,290-304), with the bound actually wired;
//   * statistics for the SERVER_FINAL_METRICS contract (server.py:320-368) plus a full
//     staleness histogram.
// Thread-safe (one mutex); exposed through a C ABI for ctypes.
#pragma once
#include <stdint.h>

extern "C" {

enum PsxMode { PSX_SYNC = 0, PSX_ASYNC = 1 };
enum PsxSyncSemantics { PSX_BARRIER = 0, PSX_REFERENCE = 1 };
enum PsxPushDecision {
  PSX_WAIT = 0,       // sync: contribution recorded, barrier not complete
  PSX_APPLY = 1,      // apply now with *weight (sync: the round is complete, 1/n contributors)
  PSX_REJECT = 2,     // async: too stale
  PSX_DUPLICATE = 3,  // sync barrier: worker already contributed to this round
  PSX_UNKNOWN = 4     // not a registered / live worker
};

void* psx_ps_create(int mode, int total_workers, float lr, int staleness_bound, int sync_semantics);
void psx_ps_destroy(void* h);
// requested_id < 0 -> next free id (reference behaviour: monotonic); otherwise rank-stable id.
int psx_ps_register(void* h, const char* name, int requested_id, double now);
void psx_ps_heartbeat(void* h, int wid, double now);
int64_t psx_ps_on_fetch(void* h, int wid, double now);
// Records a push. For PSX_APPLY, *weight is the gradient scale to use, *ncontrib the number of
// contributions aggregated (sync) and *staleness the computed staleness (async).
int psx_ps_on_push(void* h, int wid, int64_t local_step, double now, float* weight, int* ncontrib,
                   int64_t* staleness);
// Sync: list of worker ids contributing to the completed round (valid after PSX_APPLY).
int psx_ps_round_members(void* h, int* out, int cap);
// update_seconds < 0: the update's time is reported later (psx_ps_record_update_time), e.g. once
// the device events bracketing the apply kernel have completed
void psx_ps_on_applied(void* h, double update_seconds);
// one sample of the average_update_time_seconds ring (reference: server.py:128,140-141)
void psx_ps_record_update_time(void* h, double update_seconds);
int psx_ps_job_finished(void* h, int wid);  // returns 1 when no active workers remain
int psx_ps_mark_dead(void* h, int wid);     // returns 1 if a pending sync round became complete
int psx_ps_check_timeouts(void* h, double now, double timeout, int* dead, int cap);
int psx_ps_sync_ready(void* h);             // 1 if the current sync round is complete
int64_t psx_ps_global_step(void* h);
void psx_ps_set_global_step(void* h, int64_t s);
void psx_ps_rollback_to(void* h, int64_t step);  // rounds after `step` undone (sync shrink)
int psx_ps_num_active(void* h);
// Writes the SERVER_FINAL_METRICS JSON object (no prefix) into buf; returns length.
int psx_ps_metrics_json(void* h, double now, char* buf, int cap);
// Histogram of accepted staleness values (index = staleness, last bucket = overflow).
int psx_ps_staleness_hist(void* h, int64_t* out, int cap);
}
