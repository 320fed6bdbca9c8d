"""Parameter-server semantics of the native core (csrc/runtime/ps_core.cpp) — CPU only."""
import json

import pytest

from psx.parallel.core import APPLY, DUPLICATE, REJECT, UNKNOWN, WAIT, ServerCore


class Clock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def test_register_monotonic_and_rank_stable():
    c = ServerCore("sync", 3, 0.1)
    assert [c.register("a"), c.register("b")] == [0, 1]  # reference: monotonic counter
    assert c.register("c", requested_id=2) == 2
    assert c.register("a-restarted", requested_id=0) == 0  # rank-stable id on restart


def test_sync_barrier_waits_for_all_live_workers():
    c = ServerCore("sync", 3, 0.1)
    for i in range(3):
        c.register(f"w{i}", i)
    r0 = c.on_push(0, 0)
    assert r0.decision == WAIT and r0.accepted
    assert c.on_push(0, 0).decision == DUPLICATE  # a worker may not count twice in a round
    assert c.on_push(1, 0).decision == WAIT
    r = c.on_push(2, 0)
    assert r.decision == APPLY and r.ncontrib == 3 and r.weight == pytest.approx(1 / 3)
    assert sorted(c.round_members()) == [0, 1, 2]
    c.on_applied(0.001)
    assert c.global_step == 1


def test_sync_barrier_waits_for_unregistered_workers():
    c = ServerCore("sync", 2, 0.1)
    c.register("w0", 0)
    assert c.on_push(0, 0).decision == WAIT  # worker 1 not registered yet -> still waiting
    c.register("w1", 1)
    assert c.on_push(1, 0).decision == APPLY


def test_sync_barrier_excludes_finished_and_dead_workers():
    c = ServerCore("sync", 3, 0.1)
    for i in range(3):
        c.register(f"w{i}", i)
    c.job_finished(2)
    c.on_push(0, 0)
    assert c.on_push(1, 0).decision == APPLY  # finished worker no longer gates the barrier
    c.on_push(0, 1)
    assert c.mark_dead(1) is True  # dead worker removed -> round completes
    assert c.sync_ready()


def test_sync_reference_semantics_count_triggered():
    # reference server.py:264-288: a fast worker pushing twice overwrites its entry but bumps
    # the counter, so aggregation triggers with fewer distinct contributors
    c = ServerCore("sync", 3, 0.1, sync_semantics="reference")
    for i in range(3):
        c.register(f"w{i}", i)
    assert c.on_push(0, 0).decision == WAIT
    assert c.on_push(0, 0).decision == WAIT
    r = c.on_push(1, 0)
    assert r.decision == APPLY and r.ncontrib == 2 and r.weight == pytest.approx(0.5)


def test_async_staleness_bound_and_weight():
    c = ServerCore("async", 2, 0.1, staleness_bound=5)
    c.register("w0", 0)
    c.register("w1", 1)
    for _ in range(7):
        c.on_applied(0.0)
    assert c.global_step == 7
    r = c.on_push(0, 7)
    assert r.decision == APPLY and r.staleness == 0 and r.weight == pytest.approx(1.0)
    r = c.on_push(0, 4)
    assert r.staleness == 3 and r.weight == pytest.approx(1 / 1.3)
    r = c.on_push(1, 2)  # staleness 5 == bound -> accepted
    assert r.decision == APPLY and r.weight == pytest.approx(max(0.1, 1 / 1.5))
    r = c.on_push(1, 1)  # staleness 6 > bound -> rejected
    assert r.decision == REJECT and not r.accepted
    m = c.metrics()
    assert m["rejected_pushes"] == 1
    assert m["async_updates"] == 3
    assert m["max_staleness_observed"] == 6  # reference records rejected pushes too
    assert sum(c.staleness_histogram()) == 3


def test_async_weight_floor():
    c = ServerCore("async", 1, 0.1, staleness_bound=1000)
    c.register("w", 0)
    for _ in range(200):
        c.on_applied(0.0)
    r = c.on_push(0, 0)
    assert r.weight == pytest.approx(0.1)  # max(0.1, 1/(1+0.1*200))


def test_unknown_worker_push():
    c = ServerCore("async", 1, 0.1)
    assert c.on_push(42, 0).decision == UNKNOWN


def test_job_finished_and_metrics_contract():
    c = ServerCore("sync", 2, 0.1)
    c.register("w0", 0)
    c.register("w1", 1)
    assert c.job_finished(0) is False
    assert c.job_finished(1) is True
    m = c.metrics()
    for k in ("type", "mode", "total_workers", "total_training_time_seconds", "global_steps_completed",
              "total_parameter_updates", "gradients_processed", "average_update_time_seconds",
              "updates_per_second", "learning_rate"):
        assert k in m, k
    assert m["type"] == "SERVER_FINAL_METRICS" and m["mode"] == "sync"
    json.dumps(m)


def test_heartbeat_timeouts():
    clk = Clock()
    c = ServerCore("async", 2, 0.1, clock=clk)
    c.register("w0", 0)
    c.register("w1", 1)
    clk.t += 5
    c.heartbeat(0)
    clk.t += 6
    assert c.check_timeouts(10.0) == [1]
    assert c.num_active() == 1
    assert c.on_push(1, 0).decision == UNKNOWN
