"""The data-parallel worker role.

MI355X-native counterpart of the reference DistributedWorker (reference:
src/workers/worker.py:78-453). The method names and the training-loop contract are kept:
``connect_to_server`` (register), ``setup_data`` (contiguous shard), ``fetch_parameters``,
``train_local_batch``, ``push_gradients``, ``evaluate_model``, ``run_training``,
``print_worker_statistics`` (WORKER_FINAL_METRICS), ``cleanup`` (JobFinished).

The protocol side is a *channel*:

* ``InProcessChannel``  — direct calls into a ParameterServer object (1-process loopback; the
  server may host several simulated workers on one GPU);
* ``SyncCollectiveChannel`` — sync mode over RCCL: push = reduce(sum) of the wire buffer to rank 0,
  where the server applies the averaged update, fetch = broadcast of the arena (all ranks step
  together, so the wait-for-N barrier is the collective itself);
* ``AsyncChannel``      — async mode: control request on the shared-memory mailbox, bulk tensor by
  RCCL send/recv, reply (received flag, global step) on the worker's reply slot;
* ``LocalAsyncChannel`` — the worker co-located with the async server on rank 0 (pushes go to
  the server thread through a queue, fetches are device copies).
"""
from __future__ import annotations

import queue
import threading
import time

import numpy as np
import torch

from ..utils import metrics as M
from ..utils.data import EpochSampler, shard_range
from . import control as CP
from .liveness import WatchedRounds


def rounds_to_batches(rounds: int, steps_per_epoch: int, K: int) -> int:
    """Batches a worker has consumed after ``rounds`` completed push rounds (restart recovery):
    each epoch has ceil(steps/K) rounds (one per --sync-steps window; with --accumulate the last
    window may be partial), and a checkpointed round ends a whole window, so the worker resumes
    at the first batch of the next window."""
    K = max(1, K)
    per_epoch = max(1, -(-steps_per_epoch // K))
    epochs, rem = divmod(max(0, rounds), per_epoch)
    return epochs * steps_per_epoch + min(rem * K, steps_per_epoch)


class InProcessChannel:
    """``wire``: a WeightWire (parallel/codec.py) the worker's step reads its conv weights from
    (ParameterServer.enable_weight_wire must be on). A worker WeightWire of its own receives one
    device copy of the server's 22.5 MB wire per fetch; the server's wire itself (sync rounds: it
    only changes at the apply, after every step of the round) is read in place — the fetch then
    moves no bytes and the fp32 remainder is gathered from the server arena by the step's
    unpack launch (small_source)."""

    def __init__(self, server, emit_on_last: bool = False, wire=None):
        self.server = server
        self.emit_on_last = emit_on_last
        self.image_wire = wire

    def register(self, name, requested_id=-1):
        return self.server.register_worker(name, requested_id)

    def weight_wire(self):
        return self.image_wire

    def small_source(self):
        shared = self.image_wire is not None and self.image_wire is self.server.wire
        return self.server.arena if shared else None

    def fetch(self, worker_id, local_arena):
        if self.image_wire is not None:
            shared = self.image_wire is self.server.wire
            src, gs = self.server.fetch_wire(worker_id, publish_small=not shared)
            if not shared:
                self.image_wire.buf.copy_(src.buf)
            return gs
        arena, gs = self.server.fetch_parameters(worker_id)
        local_arena.copy_(arena)
        return gs

    def push(self, worker_id, grads, local_step, buffers=None):
        return self.server.push_gradients(worker_id, grads, local_step, buffers=buffers)

    def finished(self, worker_id):
        self.server.job_finished(worker_id, emit=self.emit_on_last)


class SyncCollectiveChannel(WatchedRounds):
    """All ranks call push/fetch in lockstep. Rank 0 may or may not train (topology).

    Push (dense wire): the workers' wires are gathered to rank 0 and summed there in fp32 by the
    update kernel, in a fixed worker order — the reference's decode-to-fp32 + average
    (server.py:145-169,232-237), deterministic, and every worker's transfer on its own link.
    ``PSX_SYNC_AGG=reduce`` uses one RCCL sum-reduce of the wires instead (the wire dtype's
    arithmetic at every hop: fp16 for the default codec)."""

    def __init__(self, transport, server=None, members=None, codec=None, wire=None, root_worker=True):
        import os

        self.t = transport
        self.server = server
        self.members = members or []
        self.root_worker = root_worker  # rank 0 contributes a gradient (colocated topology)
        self.agg_mode = os.environ.get("PSX_SYNC_AGG", "gather")
        self._gbufs = None
        self.codec = codec  # FetchCodec (parallel/codec.py); None = raw fp32 arena
        # weight-image fast path (parallel/codec.py WeightWire): this rank's worker-side wire
        # (None on a dedicated server rank); the server's own wire is kept by the apply
        self.image_wire = wire
        self.image = wire is not None or (server is not None and server.wire is not None)

    def register(self, name, requested_id=-1):
        # registrations of every rank are done by the runner on rank 0 (gathered names)
        return requested_id, len(self.members)

    def weight_wire(self):
        return self.image_wire

    def small_source(self):
        """Rank 0's worker reads the server's own wire: its fp32 remainder comes straight from
        the server arena (same stream, same round)."""
        shared = self.server is not None and self.image_wire is not None and self.image_wire is self.server.wire
        return self.server.arena if shared else None

    def _fetch_image(self):
        """One broadcast of the WeightWire; the worker's step consumes it in place."""
        if self.server is not None:
            for w in self.members:
                self.server.core.on_fetch(w)
            # the fp32 remainder is published for the remote workers (rank 0's own worker, on
            # the server's wire, gathers it from the arena)
            remote = len(self.members) > 1 or self.image_wire is not self.server.wire
            sw = self.server.wire_for_fetch(publish_small=remote)
            self.t.broadcast_from_server(sw.buf)
            self.server.bytes_fetched += sw.nbytes * max(0, len(self.members) - 1)
            if self.image_wire is not None and self.image_wire is not sw:  # a separate worker wire
                self.image_wire.buf.copy_(sw.buf)
            return self.server.core.global_step
        self.t.broadcast_from_server(self.image_wire.buf)
        return self._gs_after_fetch()

    def _fetch(self, worker_id, local_arena):
        if self.image:
            return self._fetch_image()
        if self.server is not None:
            for w in self.members:
                self.server.core.on_fetch(w)
            if self.codec is None or self.codec.kind == "fp32":
                # the fp32 payload IS the arena: broadcast it in place (no wire copy; the next
                # apply is stream-ordered after this round's fetch)
                self.t.broadcast_from_server(self.server.arena)
                nbytes = self.server.arena.numel() * 4
            else:
                for buf in self.codec.pack(self.server.arena):
                    self.t.broadcast_from_server(buf)
                nbytes = self.codec.nbytes
            self.server.bytes_fetched += nbytes * max(0, len(self.members) - 1)
            if local_arena is not None and local_arena.data_ptr() != self.server.arena.data_ptr():
                local_arena.copy_(self.server.arena)
            return self.server.core.global_step
        if self.codec is None or self.codec.kind == "fp32":
            self.t.broadcast_from_server(local_arena)  # received straight into the local arena
        else:
            for buf in self.codec.wire:
                self.t.broadcast_from_server(buf)
            self.codec.unpack(local_arena)
        return self._gs_after_fetch()

    def _gs_after_fetch(self):
        # global step advances by exactly one per sync round; workers track it locally
        self._gs = getattr(self, "_gs", 0)
        return self._gs

    def _push(self, worker_id, grads, local_step, buffers=None):
        sparse = grads.dtype == torch.int32  # top-k payloads cannot be summed by a reduce: gather
        world = getattr(self.t, "world_size", 1)
        dense_gather = not sparse and self.agg_mode == "gather" and world > 1
        if sparse:
            gathered = self.t.gather_to_server(grads)
        elif dense_gather:
            if self.server is not None and self._gbufs is None:
                self._gbufs = {r: torch.empty_like(grads) for r in range(1, world)}
            self.t.gather_from_workers(grads, self._gbufs if self.server is not None else None)
        else:
            self.t.reduce_sum_to_server(grads)
        if buffers is not None:
            self.t.reduce_sum_to_server(buffers)
        if self.server is not None:
            steps = [local_step] * len(self.members)
            if sparse:
                self.server.apply_gathered(gathered, self.members, steps, buffers_sum=buffers)
            elif dense_gather:
                srcs = ([grads] if self.root_worker else []) + [self._gbufs[r] for r in sorted(self._gbufs)]
                self.server.apply_sources(srcs, self.members, steps, buffers_sum=buffers)
            else:
                self.server.apply_reduced(grads, self.members, steps, buffers_sum=buffers)
            self.server.maybe_checkpoint()
        else:
            self._gs = getattr(self, "_gs", 0) + 1
        return True

    def finished(self, worker_id):
        pass


class AsyncChannel:
    def __init__(self, transport, mbox, rank, codec=None):
        self.t, self.mbox, self.rank = transport, mbox, rank
        self.codec = codec

    def register(self, name, requested_id=-1):
        self.mbox.send(CP.Msg(CP.HELLO, self.rank, requested_id))
        r = self.mbox.wait_reply(self.rank)
        return r.a, r.b

    def fetch(self, worker_id, local_arena):
        self.mbox.send(CP.Msg(CP.FETCH, self.rank, worker_id))
        bufs = [local_arena] if self.codec is None else self.codec.wire
        works = [self.t.irecv(b, 0) for b in bufs]
        r = self.mbox.wait_reply(self.rank)
        for w in works:
            w.wait()
        if self.codec is not None:
            self.codec.unpack(local_arena)
        return r.c

    def push(self, worker_id, grads, local_step, buffers=None):
        self.mbox.send(CP.Msg(CP.PUSH, self.rank, worker_id, int(buffers is not None), local_step))
        w = self.t.isend(grads, 0)
        if buffers is not None:
            self.t.isend(buffers, 0).wait()
        w.wait()
        r = self.mbox.wait_reply(self.rank)
        self.last_staleness = r.d
        return bool(r.b)

    def finished(self, worker_id):
        self.mbox.send(CP.Msg(CP.DONE, self.rank, worker_id))
        self.mbox.wait_reply(self.rank)


class LocalAsyncChannel:
    def __init__(self, server, q: "queue.Queue"):
        self.server, self.q = server, q

    def register(self, name, requested_id=-1):
        return self.server.register_worker(name, requested_id)

    def fetch(self, worker_id, local_arena):
        gs = self.server.core.on_fetch(worker_id)
        local_arena.copy_(self.server.arena)
        return gs

    def push(self, worker_id, grads, local_step, buffers=None):
        ev, box = threading.Event(), {"bufs": buffers}
        self.q.put(("push", worker_id, grads, local_step, ev, box))
        ev.wait()
        return box["res"].accepted

    def finished(self, worker_id):
        ev, box = threading.Event(), {}
        self.q.put(("done", worker_id, None, 0, ev, box))
        ev.wait()


class Worker:
    def __init__(self, cfg, compute, channel, train_set, test_set=None, worker_name=None, rank=0, log=print,
                 steps_per_epoch=None, requested_id=-1):
        self.cfg = cfg
        self.compute = compute
        self.channel = channel
        self.train_set, self.test_set = train_set, test_set
        self.worker_name = worker_name or cfg.worker_name
        self.rank = rank
        self.log = log if cfg.verbose else (lambda *a, **k: None)
        self.batch_size = cfg.batch_size
        self.learning_rate = cfg.lr
        self.num_epochs = cfg.epochs
        self.local_steps_per_sync = max(1, cfg.sync_steps)
        self.worker_id = None
        self.total_workers = None
        self.requested_id = requested_id
        self._forced_steps = steps_per_epoch
        self.local_step_counter = 0
        self.global_step_cache = 0
        self.training_start_time = None
        self.epoch_times = []
        self.accuracies = []
        self.losses = []
        self.pushes_rejected = 0
        self.images = 0
        self.timer = M.PhaseTimer(device=getattr(compute, "device", None))
        self.sampler = None
        self.topk = None
        if cfg.codec == "topk":
            from .topk import TopKCodec

            self.topk = TopKCodec(compute.layout.param_numel, cfg.topk_ratio, getattr(compute, "device", "cpu"))

    # ---------------------------------------------------------------- reference API
    def connect_to_server(self):
        self.worker_id, self.total_workers = self.channel.register(self.worker_name, self.requested_id)
        self.log(f"Registered as Worker {self.worker_id} (Total workers: {self.total_workers})")
        if hasattr(self.channel, "bind_compute"):  # e.g. the sharded round pads the gradient wire
            self.channel.bind_compute(self.compute)
        wire = self.channel.weight_wire() if hasattr(self.channel, "weight_wire") else None
        if wire is not None:  # fetches land in a WeightWire the step reads in place
            small_from = self.channel.small_source() if hasattr(self.channel, "small_source") else None
            self.compute.use_wire(wire, small_from=small_from)
        # backward-overlapped sync rounds (parallel/overlap.py): every batch is pushed, so the
        # gradient buckets can leave while the rest of the backward pass still runs
        self._overlap = bool(getattr(self.channel, "overlap", False) and self.local_steps_per_sync == 1
                             and hasattr(self.compute, "set_buckets"))
        if self._overlap:
            self.compute.set_buckets(self.channel.buckets)
        # the whole round captured into the step graph (parallel/graph_round.py)
        self._round = bool(getattr(self.channel, "in_graph", False))
        if self._round:
            self.compute.set_buckets(self.channel.buckets)
            self.channel.bind(self.compute.grads)

    def setup_data(self):
        start, end = shard_range(self.worker_id, self.total_workers, len(self.train_set))
        self.sampler = EpochSampler(start, end, self.batch_size, seed=self.cfg.seed + 17 * self.worker_id,
                                    steps=self._forced_steps)
        self.log(f"Worker {self.worker_id} assigned {end - start} training samples (indices {start}-{end - 1}); "
                 f"{len(self.sampler)} batches per epoch")

    def fetch_parameters(self):
        self.global_step_cache = self.channel.fetch(self.worker_id, self.compute.local_arena)
        return self.global_step_cache

    # sync shrink + top-k: the error-feedback residual as it was before each of the last few
    # rounds' encodes (a rollback to round R restores the residual of round R). A rollback target
    # is at most (host run-ahead) + (rounds the server keeps in flight) rounds back: the host runs
    # at most len(compute._meta_ring) steps ahead of the device (HipCompute._set_batch blocks on
    # the ring) and the server keeps at most RSERVER rounds in flight (sync_loop.cpp NSLOT = 3,
    # parallel/runner.py _PyRollback), so _rsnap_depth() slots cover every target.
    RSERVER = 3
    _rsnap = None
    _pushes = 0

    def _rsnap_depth(self) -> int:
        ring = len(getattr(self.compute, "_meta_ring", ())) or 4
        return ring + self.RSERVER + 1

    def push_gradients(self):
        bufs = None
        if self.cfg.bn_sync:
            bufs = self.compute.local_arena[self.compute.layout.param_numel:]
        g = self.compute.grads
        if self.topk is not None:  # --codec topk: error-feedback top-k payload (parallel/topk.py)
            if self.recover is not None:
                self._snapshot_resid()
            g = self.topk.encode(g)
        ok = self.channel.push(self.worker_id, g, self.global_step_cache, buffers=bufs)
        self._pushes += 1
        if not ok:
            self.pushes_rejected += 1
        return ok

    def _snapshot_resid(self):
        r = self.topk.resid
        if self._rsnap is None:
            d = self._rsnap_depth()
            self._rsnap = ([torch.empty_like(r) for _ in range(d)], [-1] * d)
        bufs, rounds = self._rsnap
        k = self._pushes % len(bufs)
        bufs[k].copy_(r)
        rounds[k] = self._pushes

    def _rewind_resid(self, rounds_kept: int):
        """The top-k residual back to its state before round ``rounds_kept``'s encode."""
        if self.topk is None or self._rsnap is None:
            self._pushes = rounds_kept
            return
        bufs, rounds = self._rsnap
        k = rounds_kept % len(bufs)
        if rounds[k] == rounds_kept:
            self.topk.resid.copy_(bufs[k])
        elif rounds_kept != self._pushes:
            raise RuntimeError(f"top-k residual of round {rounds_kept} is not in the snapshot ring "
                               f"(pushed {self._pushes}, ring {rounds})")
        self._pushes = rounds_kept

    _acc = None
    _acc_n = 0

    def window_push(self, batch_idx: int, n_batches: int, K: int) -> bool:
        """After training batch ``batch_idx`` of an epoch: push per the --sync-steps window rule —
        the window's first batch (reference, worker.py:367-377), or with --accumulate the mean
        gradient of the whole window at its last batch. Returns whether a push happened."""
        if self.cfg.accumulate and K > 1:
            self._accumulate_grads(batch_idx % K == 0)
            if batch_idx % K != K - 1 and batch_idx != n_batches - 1:
                return False
            self._finish_window()
        elif batch_idx % K != 0:
            return False
        with self.timer.span("push"):
            self.push_gradients()
        return True

    def _accumulate_grads(self, first: bool):
        """--accumulate: fp32 running sum of this window's batch gradients (stream-ordered)."""
        g = self.compute.grads
        if self._acc is None or self._acc.numel() != g.numel() or self._acc.device != g.device:
            self._acc = torch.zeros(g.numel(), dtype=torch.float32, device=g.device)
        if first:
            self._acc.copy_(g)
            self._acc_n = 1
        else:
            self._acc.add_(g.to(torch.float32))
            self._acc_n += 1

    def _finish_window(self):
        """The window's mean gradient back into the wire buffer the push sends."""
        self.compute.grads.copy_(self._acc.mul_(1.0 / max(1, self._acc_n)))

    def train_local_batch(self, idx):
        if getattr(self, "_round", False):
            self.compute.train_step(self.train_set, idx, round_hooks=self.channel)
        else:
            on_bucket = self.channel.push_bucket if getattr(self, "_overlap", False) else None
            self.compute.train_step(self.train_set, idx, on_bucket=on_bucket)
        self.local_step_counter += 1
        self.images += len(idx)

    def evaluate_model(self):
        if self.test_set is None or (self.cfg.eval_workers == "first" and self.worker_id != 0):
            return None
        acc = self.compute.evaluate(self.test_set)
        self.log(f"  > Worker {self.worker_id} test accuracy: {acc:.2f}%")
        self.accuracies.append(acc)
        return acc

    def _sync(self):
        if torch.cuda.is_available() and getattr(self.compute, "device", torch.device("cpu")).type == "cuda":
            torch.cuda.synchronize()

    recover = None  # sync shrink (parallel/elastic.py): hook(error) -> rounds to skip on the new channel

    def run_training(self, skip_steps: int = 0):
        """The reference training loop (worker.py:350-403). ``skip_steps`` = push rounds that a
        resumed server checkpoint already contains (restart recovery): the worker fast-forwards
        past the batches of those rounds (rounds_to_batches) and keeps each epoch's absolute batch
        index, so the --sync-steps windows (fetch / push points) stay where they were. A shrinking
        sync job (``recover`` set) re-enters the loop the same way at the round the survivors
        resume from when the communicator is lost."""
        if self.sampler is None:
            self.setup_data()
        self.log(f"\n--- Starting distributed training for {self.num_epochs} epochs ---")
        self.training_start_time = time.time()
        try:
            while True:
                try:
                    self._train_loop(skip_steps)
                    break
                except Exception as e:  # noqa: BLE001 - only a lost communicator is recovered
                    from .elastic import lost_error

                    if self.recover is None or not lost_error(e):
                        raise
                    self.log(f"[psx elastic] worker {self.worker_id}: {type(e).__name__}: {e}")
                    skip_steps = self.recover(e)
                    self.local_step_counter = 0
                    self._rewind_resid(skip_steps)
                    if hasattr(self.compute, "rewind"):  # augment stream + BN shifts of the kept round
                        self.compute.rewind(rounds_to_batches(skip_steps, len(self.sampler.epoch_indices(0)),
                                                              self.local_steps_per_sync))
        finally:
            self._sync()
            self.cleanup()
            self.print_worker_statistics()

    def rebind(self, channel):
        """Continue on a new channel (sync shrink): same worker id and data shard."""
        self.channel = channel
        wid, tw = self.worker_id, self.total_workers
        self.requested_id = wid
        self.connect_to_server()
        self.worker_id, self.total_workers = wid, tw

    def _train_loop(self, skip_steps: int):
        K = self.local_steps_per_sync
        self._pushes = skip_steps  # absolute round index of the next push (the snapshot ring's key)
        if skip_steps:
            rounds = skip_steps
            skip_steps = rounds_to_batches(rounds, len(self.sampler.epoch_indices(0)), K)
            self.log(f"[Resume] worker {self.worker_id} skips {rounds} completed rounds ({skip_steps} batches)")
        fi_kind, fi_worker, fi_step, fi_secs = _parse_fault(self.cfg.fault_inject)
        for epoch in range(self.num_epochs):
            self._sync()
            t_ep = time.time()
            batches = self.sampler.epoch_indices(epoch)
            if skip_steps >= len(batches):
                skip_steps -= len(batches)
                self.local_step_counter += len(batches)
                continue
            start = skip_steps
            self.local_step_counter += start
            skip_steps = 0
            for batch_idx in range(start, len(batches)):
                idx = batches[batch_idx]
                if fi_worker == self.worker_id and self.local_step_counter == fi_step:
                    if fi_kind == "hang_worker":  # alive but stalled: only a liveness guard notices
                        import sys

                        print(f"fault injected: worker {self.worker_id} hangs at step {fi_step}"
                              + (f" for {fi_secs:g} s" if fi_secs else ""), file=sys.stderr, flush=True)
                        t_end = time.time() + (fi_secs or float("inf"))
                        while time.time() < t_end:
                            time.sleep(min(3600.0, max(0.0, t_end - time.time())))
                    elif fi_kind == "crash_in_push":  # the channel dies after posting this step's PUSH
                        if not hasattr(type(self.channel), "crash_in_push"):
                            raise ValueError(f"--fault-inject crash_in_push: {type(self.channel).__name__} "
                                             "cannot inject it (the native async channel only)")
                        self.channel.crash_in_push = True
                    elif self.cfg.mode == "async" or self.recover is not None:
                        # the worker's process dies between requests: no JobFinished; the async
                        # server's heartbeat timeout drops it, a shrinking sync job goes on without
                        # it (the restart path instead raises, for the launcher)
                        import os
                        import sys

                        print(f"fault injected: worker {self.worker_id} process exits at step {fi_step}",
                              file=sys.stderr, flush=True)
                        os._exit(17)
                    else:
                        raise _InjectedFault(f"fault injected: worker {self.worker_id} at step {fi_step}")
                if batch_idx % K == 0:
                    with self.timer.span("fetch"):
                        self.fetch_parameters()
                with self.timer.span("compute_issue"):
                    self.train_local_batch(idx)
                self.window_push(batch_idx, len(batches), K)
                if self.cfg.verbose and batch_idx % 50 == 0:
                    loss = self.compute.last_loss()
                    self.losses.append(loss)
                    self.log(f"  Worker {self.worker_id} epoch {epoch + 1} batch {batch_idx}/{len(batches)} "
                             f"loss {loss:.4f} elapsed {time.time() - t_ep:.1f}s")
                if self.cfg.max_steps and self.local_step_counter >= self.cfg.max_steps:
                    break
            self._sync()
            self.epoch_times.append(time.time() - t_ep)
            self.log(f"Epoch {epoch + 1} completed in {self.epoch_times[-1]:.2f}s")
            if self.cfg.eval_every and (epoch + 1) % self.cfg.eval_every == 0:
                self.evaluate_model()
            if self.cfg.max_steps and self.local_step_counter >= self.cfg.max_steps:
                break

    def print_worker_statistics(self):
        if self.training_start_time is None:
            return None
        total = time.time() - self.training_start_time
        avg_ep = float(np.mean(self.epoch_times)) if self.epoch_times else 0.0
        final_acc = self.accuracies[-1] if self.accuracies else 0.0
        rec = {
            "type": "WORKER_FINAL_METRICS",
            "worker_id": self.worker_id,
            "total_workers": self.total_workers,
            "total_training_time_seconds": round(total, 2),
            "average_epoch_time_seconds": round(avg_ep, 2),
            "epoch_times_seconds": [round(t, 2) for t in self.epoch_times],
            "final_test_accuracy_percent": round(final_acc, 2),
            "all_accuracies_percent": [round(a, 2) for a in self.accuracies],
            "local_steps_completed": self.local_step_counter,
            "batch_size": self.batch_size,
            "learning_rate": self.learning_rate,
            "num_epochs": self.num_epochs,
            # psx extensions
            "images_per_second": round(self.images / total, 2) if total > 0 else 0.0,
            "rejected_pushes": self.pushes_rejected,
            "phase_ms": self.timer.summary_ms(),
            "last_loss": round(self.losses[-1], 4) if self.losses else None,
            "rank": self.rank,
        }
        self.log(f"\n--- Worker {self.worker_id} Statistics ---\nTotal training time: {total:.1f} seconds\n"
                 f"Local steps completed: {self.local_step_counter}\n--- End Statistics ---")
        M.emit(rec, self.cfg.log_dir, rank=self.rank)
        self.final_metrics = rec
        return rec

    def cleanup(self):
        try:
            self.channel.finished(self.worker_id)
        except Exception as e:  # reference swallows errors here (worker.py:444-450)
            self.log(f"cleanup: {e}")

    # reference method names
    train_local = train_local_batch


class _InjectedFault(RuntimeError):
    pass


def _parse_fault(spec: str):
    """'kill_worker:K@S' (worker K raises at its step S), 'hang_worker:K@S[:secs]' (worker K stalls
    at step S, process alive — forever, or for secs seconds) or 'crash_in_push:K@S' (async: worker
    K's process exits inside its step-S push, after the PUSH request, before sending the gradient)
    -> (kind, K, S, secs); anything else -> (None, None, None, None). Only armed on the first
    attempt of an elastic job (torchrun sets TORCHELASTIC_RESTART_COUNT), so a restarted job
    resumes instead of failing again."""
    import os

    kind = spec.split(":", 1)[0] if spec else ""
    if kind not in ("kill_worker", "hang_worker", "crash_in_push") or \
            int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")):
        return None, None, None, None
    k, rest = spec.split(":", 1)[1].split("@")
    s, _, secs = rest.partition(":")
    return kind, int(k), int(s), float(secs) if secs else None
