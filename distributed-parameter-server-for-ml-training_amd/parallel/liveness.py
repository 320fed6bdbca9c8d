"""Liveness guard of the synchronous round.

The reference's liveness is gRPC keepalive + registration retry (reference
src/workers/worker.py:199-231, src/parameter_server/server.py:372-378): a dead peer surfaces as
an RPC error. Over RCCL a stalled or hung rank instead leaves every other rank's collective
waiting forever — nothing in the communicator times out. ``RoundWatchdog`` watches the round
progress of one rank from a daemon thread:

* the sync channel brackets the host part of every fetch / push (``begin`` / ``end``): a
  blocking transport (gloo / torch.distributed, a host-synchronous communicator) stalls inside
  it; the native RCCL push hands over a HIP event recorded right after its collectives (they
  are stream-ordered, the host does not wait), completed when the device has finished them;
* when no round completes within ``timeout_s`` while one is outstanding, the watchdog polls the
  communicator's asynchronous error (ncclCommGetAsyncError), aborts it (ncclCommAbort — this is
  what unblocks collectives stuck on a dead peer) and terminates the process with exit status 3
  (``os._exit``: no re-exec). torchrun then tears the group down and restarts it; the server
  resumes from its last checkpoint (--ckpt-every / --resume latest) and the workers skip the
  rounds it contains (parallel/worker.py rounds_to_batches).

``--round-timeout 0`` disables it.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from collections import deque

EXIT_STALLED = 3


class CommLost(RuntimeError):
    """The job communicator was aborted (liveness watchdog or an RCCL error): a shrinking sync
    job recovers from it (parallel/elastic.py); otherwise it ends the rank."""


class RoundWatchdog:
    def __init__(self, timeout_s: float, comm=None, name: str = "", poll_s: float = 0.5, on_expire=None,
                 hint: str = ""):
        self.timeout_s = float(timeout_s)
        self.comm = comm  # parallel/rccl.py NativeComm (or None for torch.distributed / gloo)
        self.name = name
        self.hint = hint  # appended to the expiry message (e.g. bench.py's fallback switches)
        self.label = ""   # what the rank was doing last (begin(label)): named in the expiry message
        self.poll_s = poll_s
        self.on_expire = on_expire or self._abort_and_exit
        self._lock = threading.Lock()
        self._events = deque()   # HIP events of issued, not yet observed rounds
        self._blocking = 0       # blocking round calls in progress
        self._progress = time.monotonic()
        self.rounds_done = 0
        self.expired = False
        self._stop = threading.Event()
        self._follow = None       # native run: progress_fn() -> (rounds issued, rounds completed)
        self._follow_done = -1
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name="psx-round-watchdog", daemon=True)
            self._thread.start()

    # ---- channel side
    def begin(self, label: str = ""):
        """The host part of a fetch / push starts."""
        with self._lock:
            if label:
                self.label = label
            if not self._events and not self._blocking:
                self._progress = time.monotonic()  # the clock starts with the first outstanding call
            self._blocking += 1

    def end(self, event=None):
        """The host part returned; ``event``: recorded after stream-ordered collectives that the
        device has yet to finish (None: the call itself completed them)."""
        with self._lock:
            self._blocking -= 1
            if event is None:
                self._progress = time.monotonic()
                self.rounds_done += 1
            else:
                self._events.append(event)

    def follow(self, progress_fn):
        """Watch a native run of rounds (parallel/native_sync.py) instead of bracketed calls:
        ``progress_fn() -> (issued, completed)``; None ends it. While it is set, the watchdog
        expires when the completed count does not move for ``timeout_s``."""
        with self._lock:
            self._follow = progress_fn
            self._follow_done = -1
            self._progress = time.monotonic()
            if progress_fn is not None:
                self.label = "native sync server rounds (csrc/server/sync_loop.cpp)"

    # ---- watchdog thread
    def _poll(self) -> bool:
        """Retire completed rounds; True when the oldest outstanding one is overdue."""
        with self._lock:
            if self._follow is not None:
                _, done = self._follow()
                if done != self._follow_done:
                    self._follow_done = done
                    self._progress = time.monotonic()
                    self.rounds_done = done
                return time.monotonic() - self._progress > self.timeout_s
            while self._events and self._events[0].query():
                self._events.popleft()
                self._progress = time.monotonic()
                self.rounds_done += 1
            pending = bool(self._events) or self._blocking > 0
            return pending and time.monotonic() - self._progress > self.timeout_s

    def _run(self):
        while not self._stop.wait(self.poll_s):
            try:
                overdue = self._poll()
            except Exception as e:  # noqa: BLE001 - a HIP error on query is itself a failed round
                print(f"[psx watchdog{self.name}] round event query failed: {e}", file=sys.stderr, flush=True)
                overdue = True
            if overdue:
                self.expired = True
                self.on_expire(self)
                return

    def describe(self) -> str:
        """The outstanding work: the last labelled call, native progress, queued round events."""
        parts = [f"rounds done {self.rounds_done}"]
        if self.label:
            parts.append(f"outstanding: {self.label}")
        if self._follow is not None:
            try:
                issued, done = self._follow()
                parts.append(f"native rounds issued {issued} / completed {done}")
            except Exception:  # noqa: BLE001
                pass
        parts.append(f"{len(self._events)} round event(s) pending, {self._blocking} blocking call(s)")
        return ", ".join(parts)

    def _abort_and_exit(self, _wd):
        err = None
        if self.comm is not None:
            try:
                err = self.comm.async_error()
            except Exception:  # noqa: BLE001
                pass
        print(f"[psx watchdog{self.name}] no sync round completed for {self.timeout_s:.0f} s "
              f"({self.describe()}, communicator async error {err}): aborting the communicator "
              f"and exiting with status {EXIT_STALLED} so the launcher restarts the group from the last "
              f"checkpoint{self.hint}", file=sys.stderr, flush=True)
        if self.comm is not None:
            try:
                self.comm.destroy(abort=True)
            except Exception:  # noqa: BLE001
                pass
        sys.stdout.flush()
        os._exit(EXIT_STALLED)

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.poll_s + 1)


class WatchedRounds:
    """Mixin of the sync channels (SyncCollectiveChannel and its overlap / graph-round
    subclasses, ShardedSyncChannel): ``fetch`` / ``push`` run the channel's ``_fetch`` /
    ``_push`` under its ``watchdog`` (set by parallel/runner.py run_distributed; None = off)."""

    watchdog = None

    def _native(self) -> bool:
        return bool(getattr(self.t, "native", False))

    def _guard(self, fn, *a, event=False, label=""):
        """Bracket the host call; with ``event`` (native transport: the collectives are
        stream-ordered, the host does not wait for them) completion is ``_round_event()``, an
        event that completes only when the device has finished the call's collectives."""
        wd = self.watchdog
        if wd is None:
            return fn(*a)
        wd.begin(label)
        ev = None
        try:
            r = fn(*a)
            if event:
                ev = self._round_event()
            return r
        finally:
            wd.end(ev)

    def _round_event(self):
        """Event after the last collective the call issued: by default they are all on the
        current (compute) stream; channels that issue them on a communication stream the compute
        stream does not wait for (OverlapSyncChannel) record it there."""
        import torch

        ev = torch.cuda.Event()
        ev.record()
        return ev

    def _check_lost(self):
        if getattr(self.t, "lost", False):
            raise CommLost("the job communicator was aborted (liveness watchdog)")

    # server-side rollback bookkeeping of a shrinking job whose rank 0 also trains (co-located
    # topology; parallel/runner.py _PyRollback): round_start before each fetch, round_end after
    # each push's apply
    rollback = None

    def fetch(self, worker_id, local_arena):
        self._check_lost()
        if self.rollback is not None:
            self.rollback.round_start()
        # native transport: the broadcast is stream-ordered too (a fetch stuck on a dead
        # peer must not count as a finished round)
        return self._guard(self._fetch, worker_id, local_arena, event=self._native(),
                           label=f"fetch of round {getattr(self, '_gs', '?')} (broadcast from rank 0)")

    def push(self, worker_id, grads, local_step, buffers=None):
        self._check_lost()
        r = self._guard(self._push, worker_id, grads, local_step, buffers, event=self._native(),
                        label=f"push of round {local_step} (gradient gather / reduce to rank 0)")
        if self.rollback is not None:
            self.rollback.round_end()
        return r
