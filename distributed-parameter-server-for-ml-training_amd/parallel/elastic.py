"""Sync mode that survives a lost worker: the job shrinks to the surviving ranks in-process.

The reference's sync handler is count-triggered and its JobFinished drops a worker from the
active set, so a departed worker never wedges the server (reference:
src/parameter_server/server.py:264-288, :306-318); SURVEY §5.3 asks the same of the RCCL data
plane, where a dead or hung rank instead leaves every collective of the round waiting. With
``--on-worker-loss shrink`` (the default of the dedicated sync topology):

1. **Detect.** Every rank's RoundWatchdog (parallel/liveness.py) sees no round complete within
   ``--round-timeout``. Instead of exiting it calls ``on_stall``: freeze the server's count of
   rounds known good (the native loop: ``psx_sync_abort``; the Python loop: its round events),
   then abort the job communicator (ncclCommAbort: RCCL kernels waiting on the dead peer exit;
   the native registry turns every later call on the handle into an error, never a use of freed
   memory — csrc/comm/rccl_comm.cpp). A rank whose collective fails outright (an RCCL error)
   takes the same path. The training thread sees ``CommLost`` / ``RcclError`` at its next call.
2. **Agree.** Through the rendezvous TCPStore (the gloo group is as dead as the communicator):
   every survivor checks in under ``psx/el/<tag>/e<epoch>/alive/<rank>``; rank 0 (the server)
   waits up to the grace period for the others, then publishes the plan — the surviving ranks,
   the number of rounds kept R, and a fresh ncclUniqueId.
3. **Rebuild.** The server restores its arena to the start of round R (a device snapshot taken at
   every round start — no checkpoint rollback, no process restart), marks the lost workers dead
   in the native core (the wait-for-N barrier shrinks: ps_core.cpp psx_ps_mark_dead) and rolls
   its global step back to R. Every survivor builds the new communicator in-process
   (ncclCommInitRank over the survivors, ``ShrunkTransport``) — no re-exec of a GPU process —
   and the workers re-enter their loop at round R (the same fast-forward as a checkpoint resume,
   parallel/worker.py rounds_to_batches). A worker left out of the plan (one that hung past the
   grace period and woke up) exits.

Scope: sync mode, dedicated topology (rank 0 is the server only) or co-located topology (rank 0
is the server and worker 0; a lost rank > 0 — rank 0 holds the server), native RCCL transport; dense
(fp16 / fp32) or top-k wire (BASELINE config 5 — the workers restore their error-feedback residual
to the kept round from a snapshot ring, parallel/worker.py). Rounds in flight at the failure are redone by the survivors; the dead worker's
data shard is not trained further (the reference's lost pushes are lost too).
"""
from __future__ import annotations

import datetime
import json
import os
import sys
import time

import torch

from . import objwire
from .liveness import CommLost
from .rccl import NativeComm, RcclError, RcclTransport

EXCLUDED = 5  # exit status of a rank the survivors' plan left out


def enabled(cfg, transport, world: int) -> bool:
    return (getattr(cfg, "on_worker_loss", "restart") == "shrink" and cfg.mode == "sync"
            and (cfg.topology == "dedicated" or (cfg.topology == "colocated" and not cfg.overlap)) and world > 2 and getattr(transport, "native", False)
            and cfg.codec in ("fp16", "none", "topk") and not cfg.bn_sync)


def lost_error(e: BaseException) -> bool:
    """Errors that mean 'the communicator is gone' (recoverable by shrinking): a watchdog abort
    (CommLost), a failed RCCL call (RcclError), or the native server loop's communicator codes
    (NativeSyncError -60 / -65, or any code once the server's abort() ran). Any other native-loop
    failure (apply kernel, checkpoint
    callback, core bookkeeping) fails the job: shrinking would only repeat it."""
    if isinstance(e, (CommLost, RcclError)):
        return True
    from .native_sync import NativeSyncError

    return isinstance(e, NativeSyncError) and e.comm_lost


def make_on_stall(transport, freeze=None, log=None):
    """RoundWatchdog ``on_expire`` of a shrinking job: freeze the good-round count (server), abort
    the communicator, flag the transport; the training thread recovers."""

    def on_stall(wd):
        msg = (f"[psx elastic{wd.name}] no sync round completed for {wd.timeout_s:.0f} s ({wd.describe()}): "
               "aborting the communicator and shrinking the job to the surviving ranks")
        print(msg, file=sys.stderr, flush=True)
        try:
            if freeze is not None:
                freeze()  # native loop: psx_sync_abort freezes its count and aborts the comm itself
        finally:
            transport.lost = True
            try:
                transport.comm.destroy(abort=True)
            except Exception:  # noqa: BLE001
                pass

    return on_stall


class ShrunkTransport(RcclTransport):
    """The data plane of the survivors: RcclTransport's collectives on a new communicator whose
    ranks are the positions in ``members`` (the original ranks kept, ascending; rank 0 = the
    server), and host control over the rendezvous store among the members (the gloo group still
    counts the dead ranks)."""

    lost = False

    def __init__(self, base, members, comm, tag: str):  # noqa: D107 - no RcclTransport.__init__
        self.base = base
        self.members = list(members)
        self.orig_rank = base.rank
        self.rank = self.members.index(base.rank)
        self.world_size = len(self.members)
        self.device = base.device
        self.backend = base.backend
        self.comm = comm
        self._cstream = base._cstream
        self._pairs, self._pstream = {}, {}
        self.tag = tag
        self._seq = 0
        self.degraded = ()
        self.elastic_tag = getattr(base, "elastic_tag", "job")

    # ---- host control among the members (original ranks) on the store
    @staticmethod
    def _store():
        from torch.distributed import distributed_c10d as c10d

        return c10d._get_default_store()

    def _gather(self, obj):
        self._seq += 1
        key, st = f"{self.tag}/c{self._seq}", self._store()
        st.set(f"{key}/{self.orig_rank}", objwire.dumps(obj))  # JSON, never pickle
        st.wait([f"{key}/{r}" for r in self.members])
        return [objwire.loads(st.get(f"{key}/{r}")) for r in self.members]

    def barrier(self):
        self._gather(None)

    def all_gather_object(self, obj):
        return self._gather(obj)

    def broadcast_object(self, obj):
        return self._gather(obj if self.rank == 0 else None)[0]

    def close(self):
        try:
            torch.cuda.synchronize(self.device)
        finally:
            self.comm.destroy(abort=self.lost)
            self.base.comm.destroy(abort=True)  # already aborted: a no-op on the handle registry
            self._seq += 1
            key, st = f"{self.tag}/close{self._seq}", self._store()
            try:  # the store may live in rank 0's process: rank 0 leaves last
                st.set(f"{key}/{self.orig_rank}", b"1")
                if self.rank == 0:
                    st.wait([f"{key}/{r}" for r in self.members if r != self.orig_rank])
            except Exception:  # noqa: BLE001
                pass
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()


def agree(st, key: str, me: int, old_members, grace_s: float, rounds_kept=None, new_uid=None, poll_s: float = 0.05):
    """The survivors' plan (step 2 of the module docstring) on a key-value store ``st`` (the
    rendezvous TCPStore, or any c10d Store): every rank checks in under ``<key>/alive/<me>``; rank
    0 waits up to ``grace_s`` for the other old members, then publishes the plan {members, rounds,
    uid} — ``new_uid()`` makes the fresh communicator id (bytes). Everyone returns the plan dict;
    a rank that checked in after rank 0 published it is not in ``plan["members"]``. Needs no GPU
    (tests/test_elastic_cpu.py runs it over a TCPStore in several processes)."""
    old_members = list(old_members)
    st.set(f"{key}/alive/{me}", str(me).encode())
    if me == 0:
        deadline = time.monotonic() + grace_s
        others = [r for r in old_members if r != 0]
        while time.monotonic() < deadline:
            if all(st.check([f"{key}/alive/{r}"]) for r in others):
                break
            time.sleep(poll_s)
        members = [0] + [r for r in others if st.check([f"{key}/alive/{r}"])]
        uid = new_uid() if new_uid is not None else b""
        plan = {"members": members, "rounds": int(rounds_kept), "uid": uid.hex()}
        st.set(f"{key}/plan", json.dumps(plan).encode())
        return plan
    st.wait([f"{key}/plan"], datetime.timedelta(seconds=grace_s + 120))
    return json.loads(st.get(f"{key}/plan"))


def shrink(t, epoch: int, grace_s: float, rounds_kept=None, log=print):
    """Collective among the survivors (see the module docstring, steps 2-3). ``t``: the current
    transport (RcclTransport or ShrunkTransport) whose communicator is lost; rank 0 passes
    ``rounds_kept`` (its good rounds). Returns (ShrunkTransport, rounds_kept, dead original ranks)
    — or exits the process with status EXCLUDED when the plan leaves this rank out."""
    base = getattr(t, "base", t)
    tag = f"psx/el/{getattr(base, 'elastic_tag', 'job')}"
    st = ShrunkTransport._store()
    key = f"{tag}/e{epoch}"
    me = getattr(t, "orig_rank", t.rank)
    old_members = list(getattr(t, "members", range(t.world_size)))
    plan = agree(st, key, me, old_members, grace_s, rounds_kept, NativeComm.new_id)
    members = plan["members"]
    dead = [r for r in old_members if r not in members]
    if me not in members:
        print(f"[psx elastic] rank {me} is not among the survivors {members} (it missed the check-in): exiting",
              file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(EXCLUDED)
    comm = NativeComm.from_id(bytes.fromhex(plan["uid"]), len(members), members.index(me), base.device)
    nt = ShrunkTransport(base, members, comm, f"{key}/ctl")
    log(f"[psx elastic] epoch {epoch}: rank {me} continues as rank {nt.rank} of {nt.world_size} "
        f"(lost ranks {dead}); resuming at round {plan['rounds']}")
    return nt, int(plan["rounds"]), dead
