"""Python handle on the native parameter-server core (csrc/runtime/ps_core.cpp).

The core owns every decision of the reference servicer (registration ids, sync barrier,
async staleness accept/reject + weight, counters, SERVER_FINAL_METRICS JSON); this wrapper only
marshals arguments. See csrc/runtime/ps_core.h for the contract.
"""
from __future__ import annotations

import ctypes as C
import json
import time

from ..ops._lib import runtime

SYNC, ASYNC = 0, 1
BARRIER, REFERENCE = 0, 1
WAIT, APPLY, REJECT, DUPLICATE, UNKNOWN = 0, 1, 2, 3, 4
DECISIONS = {WAIT: "wait", APPLY: "apply", REJECT: "reject", DUPLICATE: "duplicate", UNKNOWN: "unknown"}


class PushResult:
    __slots__ = ("decision", "weight", "ncontrib", "staleness")

    def __init__(self, decision, weight, ncontrib, staleness):
        self.decision, self.weight, self.ncontrib, self.staleness = decision, weight, ncontrib, staleness

    @property
    def apply(self):
        return self.decision == APPLY

    @property
    def accepted(self):
        """The reference's PushReply.received (True unless rejected / unknown)."""
        return self.decision in (APPLY, WAIT)

    def __repr__(self):
        return (f"PushResult({DECISIONS[self.decision]}, weight={self.weight:.4f}, ncontrib={self.ncontrib}, "
                f"staleness={self.staleness})")


class ServerCore:
    def __init__(self, mode: str, total_workers: int, lr: float, staleness_bound: int = 5,
                 sync_semantics: str = "barrier", clock=time.monotonic):
        self._rt = runtime()
        self.mode = mode
        self.clock = clock
        self._h = self._rt.psx_ps_create(SYNC if mode == "sync" else ASYNC, total_workers, lr, staleness_bound,
                                         BARRIER if sync_semantics == "barrier" else REFERENCE)
        if not self._h:
            raise RuntimeError("psx_ps_create failed")

    def close(self):
        if self._h:
            self._rt.psx_ps_destroy(self._h)
            self._h = None

    __del__ = close

    def register(self, name: str, requested_id: int = -1) -> int:
        return self._rt.psx_ps_register(self._h, name.encode(), requested_id, self.clock())

    def heartbeat(self, wid: int):
        self._rt.psx_ps_heartbeat(self._h, wid, self.clock())

    def on_fetch(self, wid: int) -> int:
        return self._rt.psx_ps_on_fetch(self._h, wid, self.clock())

    def on_push(self, wid: int, local_step: int) -> PushResult:
        w, n, s = C.c_float(0), C.c_int(0), C.c_int64(0)
        d = self._rt.psx_ps_on_push(self._h, wid, local_step, self.clock(), C.byref(w), C.byref(n), C.byref(s))
        return PushResult(d, w.value, n.value, s.value)

    def round_members(self, cap: int = 64) -> list[int]:
        buf = (C.c_int * cap)()
        n = self._rt.psx_ps_round_members(self._h, buf, cap)
        return list(buf[: min(n, cap)])

    def on_applied(self, seconds: float):
        """One update applied (global_step + 1); ``seconds`` < 0: its time follows through
        record_update_time once the device events around the apply have completed."""
        self._rt.psx_ps_on_applied(self._h, seconds)

    def record_update_time(self, seconds: float):
        self._rt.psx_ps_record_update_time(self._h, seconds)

    def job_finished(self, wid: int) -> bool:
        return bool(self._rt.psx_ps_job_finished(self._h, wid))

    def mark_dead(self, wid: int) -> bool:
        return bool(self._rt.psx_ps_mark_dead(self._h, wid))

    def check_timeouts(self, timeout: float) -> list[int]:
        buf = (C.c_int * 64)()
        n = self._rt.psx_ps_check_timeouts(self._h, self.clock(), timeout, buf, 64)
        return list(buf[: min(n, 64)])

    def sync_ready(self) -> bool:
        return bool(self._rt.psx_ps_sync_ready(self._h))

    @property
    def global_step(self) -> int:
        return self._rt.psx_ps_global_step(self._h)

    @global_step.setter
    def global_step(self, v: int):
        self._rt.psx_ps_set_global_step(self._h, int(v))

    def rollback_to(self, step: int):
        """Rounds after ``step`` were undone (sync job shrunk after a lost worker)."""
        self._rt.psx_ps_rollback_to(self._h, int(step))

    def num_active(self) -> int:
        return self._rt.psx_ps_num_active(self._h)

    def metrics(self) -> dict:
        n = self._rt.psx_ps_metrics_json(self._h, self.clock(), None, 0)
        buf = C.create_string_buffer(n + 1)
        self._rt.psx_ps_metrics_json(self._h, self.clock(), buf, n + 1)
        return json.loads(buf.value.decode())

    def staleness_histogram(self) -> list[int]:
        buf = (C.c_int64 * 256)()
        n = self._rt.psx_ps_staleness_hist(self._h, buf, 256)
        return list(buf[: min(n, 256)])
