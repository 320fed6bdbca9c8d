"""CPU tests of the sync-shrink machinery (parallel/elastic.py, parallel/runner.py _PyRollback):

* the survivors' plan agreement over a real TCPStore in separate processes — every member in
  time, and a late joiner that checks in after rank 0 published the plan (it must see itself
  excluded, and the plan must not wait for it);
* which errors count as a lost communicator (only RCCL / watchdog / native codes -60, -65);
* the Python server loop's rollback bookkeeping against a scripted device: at most two rounds in
  flight, and the arena restored to the snapshot of exactly the first round not known good.

Reference behaviour being kept: a departed worker never wedges the sync server
(/root/reference/src/parameter_server/server.py:264-288, :306-318).
"""
import json
import multiprocessing as mp
import os
import socket
import time
from datetime import timedelta

import pytest
import torch

from psx.parallel import elastic
from psx.parallel.liveness import CommLost
from psx.parallel.native_sync import NativeSyncError
from psx.parallel.rccl import RcclError


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, port, delay, grace, q):
    from torch.distributed import TCPStore

    st = TCPStore("127.0.0.1", port, 3, rank == 0, timedelta(seconds=30), wait_for_workers=False)
    time.sleep(delay)
    t0 = time.monotonic()
    plan = elastic.agree(st, "psx/el/test/e1", rank, [0, 1, 2], grace, rounds_kept=7 if rank == 0 else None,
                         new_uid=lambda: b"\x01\x02")
    q.put((rank, plan, time.monotonic() - t0))
    st.set(f"done/{rank}", b"1")
    if rank == 0:  # the store lives here: leave last
        st.wait(["done/1", "done/2"], timedelta(seconds=60))


def _run_ranks(delays, grace):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank_main, args=(r, port, delays[r], grace, q)) for r in range(3)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(3):
        r, plan, dt = q.get(timeout=60)
        out[r] = (plan, dt)
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    return out


def test_agree_all_members():
    out = _run_ranks([0.0, 0.2, 0.4], grace=10.0)
    for r in range(3):
        plan, _ = out[r]
        assert plan == {"members": [0, 1, 2], "rounds": 7, "uid": "0102"}
    assert out[0][1] < 5.0  # rank 0 did not wait out the grace once everyone checked in


def test_agree_late_joiner_excluded():
    """Rank 2 checks in 3 s after the 1 s grace: the plan holds ranks 0 and 1 only, rank 0 waited
    about the grace (not for rank 2), and rank 2 reads a plan without itself."""
    out = _run_ranks([0.0, 0.1, 3.0], grace=1.0)
    plan0, dt0 = out[0]
    assert plan0["members"] == [0, 1] and plan0["rounds"] == 7
    assert 0.9 <= dt0 < 2.5
    assert out[1][0] == plan0
    assert out[2][0] == plan0 and 2 not in out[2][0]["members"]


def test_lost_error_classification():
    assert elastic.lost_error(CommLost("x"))
    assert elastic.lost_error(RcclError("ncclRecv failed"))
    assert elastic.lost_error(NativeSyncError(-65))
    assert elastic.lost_error(NativeSyncError(-60))
    for rc in (-50, -61, -62, -63, -64):  # apply kernel, core, checkpoint, ...: the job fails
        assert not elastic.lost_error(NativeSyncError(rc))
    for rc in (-50, -61):  # after this server's abort(), the loop's first error is often a HIP one
        assert elastic.lost_error(NativeSyncError(rc, aborted=True))
    assert not elastic.lost_error(RuntimeError("native sync server failed (-65)"))  # only the typed error
    assert not elastic.lost_error(ValueError("x"))


# ------------------------------------------------------------------ _PyRollback on a scripted device
class _Dev:
    """A scripted device: round i's event completes once ``done > i``; ``synchronize`` of an
    event completes everything up to it (the host waited)."""

    def __init__(self):
        self.done = 0
        self.next = 0


class _Ev:
    def __init__(self, dev):
        self.dev = dev
        self.i = None

    def record(self, *a):
        self.i = self.dev.next
        self.dev.next += 1

    def query(self):
        return self.dev.done > self.i

    def synchronize(self):
        self.dev.done = max(self.dev.done, self.i + 1)


class _Core:
    def __init__(self):
        self.global_step = 0

    def rollback_to(self, g):
        self.global_step = g


class _Srv:
    def __init__(self):
        self.arena = torch.zeros(4)
        self.momentum_buf = None
        self.core = _Core()
        self._mom_first = True
        self.wire = None


class _Chan:
    watchdog = None
    t = None


def _rounds(monkeypatch, n_rounds, device_done_at_freeze):
    from psx.parallel import runner

    dev = _Dev()
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: _Ev(dev))
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    s = _Srv()
    rb = runner._PyRollback(s, _Chan())
    waits = []
    for n in range(n_rounds):
        before = dev.done
        rb.round_start()
        waits.append(dev.done - before)
        # the round's apply: arena value = number of rounds applied (in issue order)
        s.arena += 1.0
        s.core.global_step += 1
        rb.round_end()
        assert rb.issued - max(dev.done, rb.retired) <= 2  # at most two rounds in flight after issue
    dev.done = max(dev.done, device_done_at_freeze)
    rb.freeze()
    # after the abort the stream runs on (garbage rounds "complete"): must not change the target
    dev.done = dev.next
    if device_done_at_freeze < n_rounds:  # only an unfinished round can leave garbage behind
        s.arena += 100.0
    g = rb.rollback()
    return g, s


@pytest.mark.parametrize("n_rounds,done", [(1, 0), (2, 1), (5, 3), (5, 4), (5, 5), (8, 6)])
def test_py_rollback_restores_first_unfinished_round(monkeypatch, n_rounds, done):
    g, s = _rounds(monkeypatch, n_rounds, done)
    # the host waited for round n-2 at each start, so at least n-2 rounds were observed complete
    expect = max(done, n_rounds - 2, 0)
    assert g == expect
    assert s.core.global_step == expect
    assert float(s.arena[0]) == float(expect)  # the arena as it was at the start of round g


def test_py_rollback_without_freeze_uses_issued(monkeypatch):
    """An RCCL error raised from an enqueue (no watchdog): the failed round never ended, so the
    target is the issued count — the arena at the start of the round that failed."""
    from psx.parallel import runner

    dev = _Dev()
    monkeypatch.setattr(torch.cuda, "Event", lambda *a, **k: _Ev(dev))
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    s = _Srv()
    rb = runner._PyRollback(s, _Chan())
    for _ in range(3):
        rb.round_start()
        s.arena += 1.0
        rb.round_end()
    rb.round_start()  # round 3 starts, its push raises before round_end
    s.arena += 0.5    # a partial apply that must be undone
    g = rb.rollback()
    assert g == 3 and float(s.arena[0]) == 3.0
