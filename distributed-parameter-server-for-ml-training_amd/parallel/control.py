"""Control plane: the small host messages of the PS protocol.

The reference's four RPCs (reference: src/communication/ps.proto:4-19) carry two kinds of
payload: small control fields (worker_id, local_step, global_step, received flag, total_workers)
and the bulk tensors. Here bulk tensors move over RCCL/xGMI (parallel/transport.py) while the
control fields travel through a mailbox:

* ``ShmMailbox``  — native lock-free MPMC ring in POSIX shared memory (csrc/runtime/mailbox.cpp),
  one per node, used by every multi-process run; worker -> server requests on the ring, one
  reply slot per worker. A few microseconds per message, no server thread pool.
* ``LocalMailbox`` — in-process queues with the same interface (single-process loopback runs
  and CPU tests).

Messages are 6 integers: (type, src, a, b, c, d).
"""
from __future__ import annotations

import ctypes as C
import queue
import threading
import time

from ..ops._lib import runtime

# request types (worker -> server)
HELLO, PUSH, FETCH, DONE, HEARTBEAT, STOP = 1, 2, 3, 4, 5, 6
# reply types (server -> worker)
R_REGISTERED, R_PUSHED, R_FETCHED, R_ACK, R_DROPPED = 11, 12, 13, 14, 15

NAMES = {HELLO: "HELLO", PUSH: "PUSH", FETCH: "FETCH", DONE: "DONE", HEARTBEAT: "HEARTBEAT", STOP: "STOP",
         R_REGISTERED: "REGISTERED", R_PUSHED: "PUSHED", R_FETCHED: "FETCHED", R_ACK: "ACK", R_DROPPED: "DROPPED"}


class WorkerDropped(RuntimeError):
    """The server declared this worker dead (missed heartbeats, an overdue transfer, a stall) and
    refuses its requests (R_DROPPED): the worker ends its training loop."""


class Msg(tuple):
    __slots__ = ()

    def __new__(cls, type_, src=0, a=0, b=0, c=0, d=0):
        return super().__new__(cls, (int(type_), int(src), int(a), int(b), int(c), int(d)))

    type = property(lambda s: s[0])
    src = property(lambda s: s[1])
    a = property(lambda s: s[2])
    b = property(lambda s: s[3])
    c = property(lambda s: s[4])
    d = property(lambda s: s[5])

    def __repr__(self):
        return f"Msg({NAMES.get(self[0], self[0])}, src={self[1]}, a={self[2]}, b={self[3]}, c={self[4]}, d={self[5]})"


class MailboxTimeout(TimeoutError):
    pass


class ShmMailbox:
    def __init__(self, name: str, nreply: int, owner: bool, capacity: int = 1024, timeout: float = 60.0):
        self._rt = runtime()
        self.name = name
        self._h = self._rt.psx_mbox_open(name.encode(), capacity, nreply, int(owner), timeout)
        if not self._h:
            raise RuntimeError(f"could not {'create' if owner else 'attach'} shared-memory mailbox {name}")
        self._seq = {}

    def close(self):
        if getattr(self, "_h", None):
            self._rt.psx_mbox_close(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def send(self, msg: Msg, timeout: float = 60.0):
        if self._rt.psx_mbox_send(self._h, *msg, timeout) != 0:
            raise MailboxTimeout("mailbox full")

    def recv(self, timeout: float = 0.0) -> Msg | None:
        out = (C.c_longlong * 6)()
        if self._rt.psx_mbox_recv(self._h, out, timeout):
            return Msg(*out)
        return None

    def reply(self, slot: int, msg: Msg):
        if self._rt.psx_mbox_reply(self._h, slot, msg.type, msg.a, msg.b, msg.c, msg.d) != 0:
            raise IndexError(f"reply slot {slot} out of range")

    def wait_reply(self, slot: int, timeout: float = 60.0) -> Msg:
        out = (C.c_longlong * 6)()
        last = self._seq.get(slot, 0)
        seq = self._rt.psx_mbox_wait_reply(self._h, slot, last, out, timeout)
        if seq == 0:
            raise MailboxTimeout(f"no reply on slot {slot} within {timeout}s")
        self._seq[slot] = seq
        return Msg(*out)


class LocalMailbox:
    """Thread-safe in-process mailbox with the ShmMailbox interface."""

    def __init__(self, nreply: int = 64):
        self._q: "queue.Queue[Msg]" = queue.Queue()
        self._replies = [queue.Queue() for _ in range(nreply)]
        self.name = "local"

    def close(self):
        pass

    def send(self, msg: Msg, timeout: float = 60.0):
        self._q.put(msg)

    def recv(self, timeout: float = 0.0) -> Msg | None:
        try:
            return self._q.get(timeout=timeout) if timeout > 0 else self._q.get_nowait()
        except queue.Empty:
            return None

    def reply(self, slot: int, msg: Msg):
        self._replies[slot].put(msg)

    def wait_reply(self, slot: int, timeout: float = 60.0) -> Msg:
        try:
            return self._replies[slot].get(timeout=timeout)
        except queue.Empty as e:
            raise MailboxTimeout(f"no reply on slot {slot} within {timeout}s") from e


class Heartbeat(threading.Thread):
    """Background liveness ping (the reference's intended health-check loop, worker.py:112-119,
    which never ran because run_training was shadowed)."""

    def __init__(self, mbox, worker_id: int, rank: int, period: float = 5.0):
        super().__init__(daemon=True)
        self.mbox, self.worker_id, self.rank, self.period = mbox, worker_id, rank, period
        self._stop = threading.Event()

    def run(self):
        while not self._stop.wait(self.period):
            try:
                self.mbox.send(Msg(HEARTBEAT, self.rank, self.worker_id), timeout=1.0)
            except Exception:
                return

    def stop(self):
        self._stop.set()


def now() -> float:
    return time.monotonic()
