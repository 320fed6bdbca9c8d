"""The parameter server role (rank 0).

MI355X-native counterpart of the reference ParameterServerServicer
(reference: src/parameter_server/server.py:81-368):

* state lives in HBM: one fp32 arena holding the full state_dict (models/layout.py), an
  optional momentum buffer, a staging/aggregation buffer — no pickle, no param_lock: every
  update is one fused kernel (csrc/kernels/optim.hip) ordered on the server's HIP stream;
* decisions (registration ids, sync barrier, async staleness reject/weight, statistics) are
  made by the native core (csrc/runtime/ps_core.cpp, parallel/core.py);
* the reference RPC surface is kept for in-process use and naming parity:
  ``RegisterWorker``/``register_worker``, ``FetchParameters``/``fetch_parameters``,
  ``PushGradrients`` (sic, ps.proto:12) / ``PushGradients`` / ``push_gradients``,
  ``JobFinished``/``job_finished``;
* ``serve_async`` is the server event loop of the multi-process async mode: control
  requests arrive on the shared-memory mailbox, bulk tensors over RCCL point-to-point, and every
  fetch is served from a per-worker snapshot of the arena so in-flight sends never race the
  next update (the double-buffered arena of SURVEY.md §5.2).
"""
from __future__ import annotations

import os
import time

import torch

from ..utils import checkpoint as ckpt
from ..utils import metrics as M
from ..utils import trace
from . import control as CP
from . import topk
from .core import APPLY, WAIT, ServerCore

_TRACE = os.environ.get("PSX_TRACE", "0") == "1"


def arena_sha256(arena: torch.Tensor) -> str:
    """sha256 (hex, first 32 digits) of an fp32 arena's bytes."""
    import hashlib

    return hashlib.sha256(arena.detach().to("cpu", torch.float32).contiguous().numpy().tobytes()).hexdigest()[:32]


class ParameterServer:
    def __init__(self, cfg, layout, init_arena: torch.Tensor, counters: torch.Tensor | None = None, device="cpu",
                 total_workers: int | None = None, log=print):
        self.cfg = cfg
        self.layout = layout
        self.device = torch.device(device)
        self.total_workers = total_workers if total_workers is not None else cfg.workers
        self.lr = cfg.lr
        self.log = log if cfg.verbose else (lambda *a, **k: None)
        self.arena = init_arena.to(self.device, dtype=torch.float32).contiguous()
        self.counters = counters if counters is not None else torch.zeros(max(1, layout.num_counters), dtype=torch.int64)
        self.n = layout.param_numel
        self.params = self.arena[: self.n]
        self.momentum_buf = torch.zeros_like(self.params) if cfg.momentum else None
        self._mom_first = True
        self.agg = None  # fp32 aggregation buffer for in-process sync rounds
        self.wire = None  # WeightWire fetch payload kept current by the apply (enable_weight_wire)
        self._wire_stale = False
        self._pending = {}
        self.core = ServerCore(cfg.mode, self.total_workers, cfg.lr, cfg.staleness_bound, cfg.sync_semantics)
        self.start_time = time.time()
        self.bytes_pushed = 0
        self.bytes_fetched = 0
        self.images_processed = 0
        self.log(f"Initializing Parameter Server in {cfg.mode.upper()} mode on {self.device} "
                 f"({len(layout.entries)} state_dict tensors, {self.n:,} trainable params)")
        if cfg.resume:
            self.resume(cfg.resume)

    # ------------------------------------------------------------------ numerics
    def apply(self, grads: torch.Tensor, weight: float):
        """p <- p - lr * (weight * g [+ wd p]) [momentum]; grads are fp16 wire or fp32."""
        trace.mark("psx.apply")
        t0 = self._time_begin()
        if grads.dtype == torch.int32:  # top-k payload (parallel/topk.py)
            if not self.cfg.momentum and not self.cfg.weight_decay:
                # no optimizer state: scatter straight into the fp32 master parameters
                topk.decode_add(grads, self.params, -self.lr * weight, self._kcap)
                self._wire_stale = True  # the bf16 image was not written by this update
                return self.finish_round_apply(self._time_end(t0))
            grads = self._dense_of(grads)
        self.apply_range(grads[: self.n], weight, 0, self.n)
        return self.finish_round_apply(self._time_end(t0))

    # ------------------------------------------------------------------ update timing
    # The reference times the apply itself (server.py:128,140-141) into average_update_time_seconds.
    # Here the apply is an asynchronous kernel, so its time is the DEVICE time between two timing
    # events recorded around it on the update stream; the pair is read back lazily (when a later
    # apply starts, or at final_metrics) and fed to the core. A round applied in several ranges
    # (gradient buckets of an overlapped round) sums its ranges. CPU arenas use the host clock.
    # Applies captured into a HIP graph cannot be bracketed: they leave no sample.
    _round_ev: list = []
    _ev_pending: list = []
    update_time_source = "none"

    def _time_begin(self):
        if self.device.type != "cuda":
            return time.perf_counter()
        if torch.cuda.is_current_stream_capturing():
            return None
        self._drain_update_times()
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _time_end(self, tok):
        """Closes one timed range; returns the host seconds (CPU) or -1 (device: deferred)."""
        if tok is None:
            return -1.0
        if isinstance(tok, float):
            return time.perf_counter() - tok
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        self._round_ev = self._round_ev + [(tok, end)]
        return -1.0

    def _drain_update_times(self, block: bool = False):
        keep = []
        for pairs in self._ev_pending:
            if block or all(e.query() for _, e in pairs):
                s = sum(b.elapsed_time(e) for b, e in pairs) * 1e-3  # elapsed_time waits for e
                self.core.record_update_time(s)
                self.update_time_source = "device events around the apply kernels"
            else:
                keep.append(pairs)
        self._ev_pending = keep

    @property
    def _kcap(self) -> int:
        return topk.topk_k(self.n, self.cfg.topk_ratio)

    def _dense_of(self, payload: torch.Tensor, out: torch.Tensor | None = None, add: bool = False):
        """Top-k payload -> dense fp32 gradient (into the aggregation buffer by default)."""
        if out is None:
            if self.agg is None:
                self.agg = torch.zeros(self.n, dtype=torch.float32, device=self.device)
            out = self.agg
        if not add:
            out.zero_()
        return topk.decode_add(payload, out, 1.0, self._kcap)

    def apply_range(self, g: torch.Tensor, weight: float, lo: int, hi: int):
        """The update restricted to params[lo:hi] (g holds exactly that slice): one bucket of a
        backward-overlapped sync round (parallel/overlap.py). Several ranges of one round share
        the same momentum 'first step' flag; finish_round_apply closes the round."""
        p = self.params[lo:hi]
        buf = self.momentum_buf[lo:hi] if self.momentum_buf is not None else None
        if self.device.type == "cuda":
            from ..ops import kernels as K

            img = self.wire.img[lo:hi] if self.wire is not None else None  # fetch image, same pass
            K.sgd_apply(p, g, self.lr, gscale=weight, momentum=self.cfg.momentum, wd=self.cfg.weight_decay, buf=buf,
                        first=self._mom_first, n=hi - lo, img=img)
            return
        if self.wire is not None:
            self._wire_stale = True
        d = g.to(torch.float32) * weight
        if self.cfg.weight_decay:
            d = d + self.cfg.weight_decay * p
        if buf is not None:
            if self._mom_first:
                buf.copy_(d)
            else:
                buf.mul_(self.cfg.momentum).add_(d)
            d = buf
        p.sub_(self.lr * d)

    def apply_range_sources(self, srcs: list, weight: float, lo: int, hi: int):
        """apply_range of the fp32 sum of several wires' [lo:hi] (fixed list order): one bucket
        of an overlapped round whose wires were gathered (parallel/overlap.py)."""
        if self.device.type == "cuda":
            from ..ops import kernels as K

            buf = self.momentum_buf[lo:hi] if self.momentum_buf is not None else None
            img = self.wire.img[lo:hi] if self.wire is not None else None
            K.sgd_apply_multi(self.params[lo:hi], [s[lo:hi] for s in srcs], self.lr, gscale=weight,
                              momentum=self.cfg.momentum, wd=self.cfg.weight_decay, buf=buf, first=self._mom_first,
                              n=hi - lo, img=img)
            return
        agg = torch.zeros(hi - lo, dtype=torch.float32, device=self.device)
        for s in srcs:  # fixed order, fp32 accumulation
            agg.add_(s[lo:hi].to(torch.float32))
        self.apply_range(agg, weight, lo, hi)

    def finish_round_apply(self, dt: float = -1.0):
        """Closes one update (global_step + 1). ``dt`` >= 0: its host-measured time (CPU arena);
        else the device ranges timed since the last close (deferred), or none (graph capture)."""
        self._mom_first = False
        if self._round_ev:
            self._ev_pending = self._ev_pending + [self._round_ev]
            self._round_ev = []
            dt = -1.0
        elif dt >= 0:
            self.update_time_source = "host clock (synchronous CPU apply)"
        self.core.on_applied(dt)
        return dt

    def _accumulate(self, grads: torch.Tensor, first: bool):
        if self.agg is None:
            self.agg = torch.zeros(self.n, dtype=torch.float32, device=self.device)
        if grads.dtype == torch.int32:
            self._dense_of(grads, self.agg, add=not first)
            return
        if first:
            self.agg.copy_(grads[: self.n])
        else:
            self.agg.add_(grads[: self.n].to(torch.float32))

    # ------------------------------------------------------------------ RPC surface
    def register_worker(self, worker_name: str = "worker-node", requested_id: int = -1):
        wid = self.core.register(worker_name, requested_id)
        self.log(f"[RegisterWorker] Worker {wid} from {worker_name} registered")
        self.log(f"Active workers: {self.core.num_active()}/{self.total_workers}")
        return wid, self.total_workers

    def fetch_parameters(self, worker_id: int):
        gs = self.core.on_fetch(worker_id)
        self.bytes_fetched += self.arena.numel() * 4
        return self.arena, gs

    # ------------------------------------------------------------------ weight-image fetch path
    def enable_weight_wire(self):
        """Keep a WeightWire (parallel/codec.py) of the current state: the apply kernel writes
        its bf16 image in the same pass as the fp32 update; the fp32 remainder is gathered per
        fetch. Fetches then ship/copy exactly that one buffer."""
        from .codec import WeightWire

        if self.wire is None:
            self.wire = WeightWire(self.layout, self.device)
        self.wire.publish_full(self.arena)
        self._wire_stale = False
        return self.wire

    def wire_for_fetch(self, publish_small: bool = True):
        """The WeightWire holding the current state (fp32 remainder refreshed unless the only
        reader gathers it from the arena itself; the image was written by the apply, or is
        rebuilt here after an out-of-band update)."""
        if self._wire_stale:
            self.wire.publish_full(self.arena)
            self._wire_stale = False
        elif publish_small:
            self.wire.publish_small(self.arena)
        return self.wire

    def fetch_wire(self, worker_id: int, publish_small: bool = True):
        gs = self.core.on_fetch(worker_id)
        w = self.wire_for_fetch(publish_small)
        self.bytes_fetched += w.nbytes
        return w, gs

    def push_gradients(self, worker_id: int, grads: torch.Tensor, local_step: int, buffers=None) -> bool:
        """In-process push (single-process loopback runs). Sync: aggregate until the barrier
        completes, then apply the average. Async: staleness check + weighted apply.
        ``buffers`` (--bn-sync): the worker's BN running statistics, counted only when the core
        takes the push into the round (a duplicate / unknown / rejected push contributes nothing)."""
        self.bytes_pushed += grads[: self.n].numel() * grads.element_size()
        res = self.core.on_push(worker_id, local_step)
        self.last_push = res
        if buffers is not None and (res.decision in (WAIT, APPLY) if self.cfg.mode == "sync" else res.accepted):
            self.push_buffers(worker_id, buffers)
        if self.cfg.mode == "sync":
            if self.cfg.sync_semantics == "reference":
                # reference: pending[worker_id] = grads (overwrites), average over the dict
                # entries when the push counter reaches total_workers (server.py:264-288)
                if res.decision in (WAIT, APPLY):
                    self._pending[worker_id] = (self._dense_of(grads, torch.zeros(self.n, device=self.device))
                                                if grads.dtype == torch.int32
                                                else grads[: self.n].to(torch.float32).clone())
                if res.apply:
                    self._accumulate(sum(self._pending.values()), True)
                    self._pending.clear()
                    self.apply(self.agg, res.weight)
                    self._commit_buffers()
                return True  # the reference always answers received=True in sync mode
            if res.apply and self._round_count == 0:
                # single-contribution round (W == 1): apply straight from the wire buffer — a dense
                # wire through the collective rounds' kernel (apply_sources with one source), so a
                # loopback round and a one-worker RCCL round (a shrunk sync job) give the same bits
                if grads.dtype == torch.int32:  # decoded into the dense buffer first, as apply_gathered
                    self._dense_of(grads)
                    self.apply(self.agg, res.weight)
                else:
                    trace.mark("psx.apply")
                    t0 = self._time_begin()
                    self.apply_range_sources([grads], res.weight, 0, self.n)
                    self.finish_round_apply(self._time_end(t0))
                self._commit_buffers()
                return True
            if res.decision in (WAIT, APPLY):
                self._accumulate(grads, self._round_count == 0)
                self._round_count += 1
            if res.apply:
                self.apply(self.agg, res.weight)
                self._commit_buffers()
                self._round_count = 0
            return res.accepted
        if res.apply:
            self.apply(grads, res.weight)
        return res.accepted

    _round_count = 0
    _pending: dict = {}
    last_push = None
    _buf_acc = None
    _buf_n = 0

    # ------------------------------------------------------------------ BN running stats (--bn-sync)
    def push_buffers(self, worker_id: int, bufs: torch.Tensor):
        """Worker BN running statistics (float buffer region of its local arena). Sync: averaged
        over the round (committed with the round's update); async: blended with weight 1/W."""
        if self.layout.buffer_numel == 0:
            return
        region = self.arena[self.n:]
        if self.cfg.mode == "sync":
            if self._buf_acc is None:
                self._buf_acc = torch.zeros_like(region)
            self._buf_acc.add_(bufs.to(region.device))
            self._buf_n += 1
        else:
            w = 1.0 / max(1, self.total_workers)
            region.mul_(1.0 - w).add_(bufs.to(region.device), alpha=w)

    def _commit_buffers(self):
        if self._buf_n:
            self.arena[self.n:].copy_(self._buf_acc / self._buf_n)
            self._buf_acc.zero_()
            self._buf_n = 0

    def set_buffers_from_sum(self, summed: torch.Tensor, count: int):
        self.arena[self.n:].copy_(summed / max(1, count))

    def job_finished(self, worker_id: int, emit: bool = True) -> str:
        """Reference server.py:306-318: when the last active worker finishes, print the final
        statistics (runners that append job-level fields pass emit=False and emit once)."""
        self.log(f"[JobFinished] Worker {worker_id} completed")
        if self.core.job_finished(worker_id) and emit:
            self.final_metrics(emit=True)
        return "Acknowledged"

    # reference RPC names (ps.proto:4-19, including the PushGradrients typo)
    RegisterWorker = register_worker
    FetchParameters = fetch_parameters
    PushGradients = push_gradients
    PushGradrients = push_gradients
    JobFinished = job_finished

    # ------------------------------------------------------------------ sync (collective) path
    def apply_reduced(self, summed: torch.Tensor, members: list[int], local_steps: list[int],
                      buffers_sum: torch.Tensor | None = None) -> bool:
        """Bookkeeping + update for one sync round whose gradient sum arrived by RCCL reduce."""
        res = None
        for wid, ls in zip(members, local_steps):
            res = self.core.on_push(wid, ls)
        self.bytes_pushed += len(members) * self.n * summed.element_size()
        if res is not None and res.apply:
            self.apply(summed, res.weight)
            if buffers_sum is not None:
                self.set_buffers_from_sum(buffers_sum, len(members))
            return True
        return False

    def apply_sources(self, srcs: list, members: list[int], local_steps: list[int],
                      buffers_sum: torch.Tensor | None = None) -> bool:
        """Sync round whose W dense wires were gathered to rank 0 (one per contributing worker):
        decoded and summed in fp32 in list order inside the update (kernels.sgd_apply_multi),
        then p -= lr * sum / W — the reference's decompress + aggregate + apply
        (server.py:126-169, 232-237) without an fp16 running sum."""
        res = None
        for wid, ls in zip(members, local_steps):
            res = self.core.on_push(wid, ls)
        self.bytes_pushed += sum(s[: self.n].numel() * s.element_size() for s in srcs)
        if res is None or not res.apply:
            return False
        trace.mark("psx.apply")
        t0 = self._time_begin()
        if self.device.type == "cuda":
            from ..ops import kernels as K

            img = self.wire.img[: self.n] if self.wire is not None else None
            K.sgd_apply_multi(self.params, [s[: self.n] for s in srcs], self.lr, gscale=res.weight,
                              momentum=self.cfg.momentum, wd=self.cfg.weight_decay, buf=self.momentum_buf,
                              first=self._mom_first, n=self.n, img=img)
        else:
            if self.agg is None:
                self.agg = torch.zeros(self.n, dtype=torch.float32, device=self.device)
            self.agg.zero_()
            for s in srcs:  # fixed order, fp32 accumulation
                self.agg.add_(s[: self.n].to(torch.float32))
            self.apply_range(self.agg, res.weight, 0, self.n)
        self.finish_round_apply(self._time_end(t0))
        if buffers_sum is not None:
            self.set_buffers_from_sum(buffers_sum, len(members))
        return True

    def apply_gathered(self, payloads: list, members: list[int], local_steps: list[int],
                       buffers_sum: torch.Tensor | None = None) -> bool:
        """Sync round with top-k payloads gathered to rank 0: decode all into one dense fp32
        sum, then the usual averaged apply."""
        res = None
        for wid, ls in zip(members, local_steps):
            res = self.core.on_push(wid, ls)
        self.bytes_pushed += sum(p.numel() * 4 for p in payloads[: max(1, len(members))])
        if res is not None and res.apply:
            for i, p in enumerate(payloads):
                self._dense_of(p, add=i > 0)
            self.apply(self.agg, res.weight)
            if buffers_sum is not None:
                self.set_buffers_from_sum(buffers_sum, len(members))
            return True
        return False

    # ------------------------------------------------------------------ checkpoint
    def checkpoint(self, path: str | None = None) -> str:
        step = self.core.global_step
        path = path or ckpt.path_for(self.cfg.ckpt_dir, step)
        ckpt.save(path, self.layout, self.arena, self.counters, step, self.cfg.mode, self.total_workers, self.lr,
                  self.momentum_buf, self.cfg.to_json())
        self.log(f"[Checkpoint] global step {step} -> {path}")
        return path

    def maybe_checkpoint(self):
        if self.cfg.ckpt_every and self.core.global_step % self.cfg.ckpt_every == 0 and self.core.global_step:
            return self.checkpoint()
        return None

    def resume(self, path: str):
        if path == "latest":
            path = ckpt.latest(self.cfg.ckpt_dir)
            if path is None:
                self.log("[Resume] no checkpoint found; starting fresh")
                return
        arena, counters, step, mom, _ = ckpt.restore(path, self.layout)
        self.arena.copy_(arena.to(self.device))
        self._wire_stale = True
        self.counters = counters
        self.core.global_step = step
        if mom is not None and self.momentum_buf is not None:
            self.momentum_buf.copy_(mom.to(self.device))
            self._mom_first = False
        self.log(f"[Resume] restored global step {step} from {path}")

    # ------------------------------------------------------------------ metrics
    def final_metrics(self, emit: bool = False, extra: dict | None = None) -> dict:
        if self._ev_pending:
            self._drain_update_times(block=True)
        m = self.core.metrics()
        m["update_time_source"] = self.update_time_source
        m["bytes_pushed"] = int(self.bytes_pushed)
        m["bytes_fetched"] = int(self.bytes_fetched)
        if self.images_processed:
            m["images_processed"] = int(self.images_processed)
        # fingerprints of the final master state: sum |p| (order-independent, for tolerance checks)
        # and the sha256 of the fp32 arena bytes (bit-equality checks across runs / modes)
        m["final_param_checksum"] = float(self.arena.double().abs().sum())
        m["final_param_sha256"] = arena_sha256(self.arena)
        if extra:
            m.update(extra)
        if emit:
            self.log(f"\n{'=' * 50}\nPARAMETER SERVER FINAL STATISTICS\n{'=' * 50}")
            self.log(f"Mode: {m['mode'].upper()}  workers: {m['total_workers']}  global steps: "
                     f"{m['global_steps_completed']}  updates/s: {m['updates_per_second']}")
            M.emit(m, self.cfg.log_dir, rank=0)
            self.log("--- End Server Metrics ---")
        return m

    # ------------------------------------------------------------------ async event loop
    def serve_async(self, transport, mbox, rank_of: dict, stop_when_done: bool = True, local_queue=None,
                    poll: float = 0.0005, expected: int | None = None):
        """Multi-process async server loop (runs on rank 0, in its own thread when rank 0 also
        trains). rank_of: worker_id -> transport rank of the *remote* workers. ``local_queue``
        (optional) delivers requests of the co-located worker as (kind, worker_id, grads,
        local_step, event, box). The loop ends once ``expected`` workers finished or died."""
        expected = expected if expected is not None else len(rank_of) + (1 if local_queue is not None else 0)
        finished = set()
        n = self.n
        if self.cfg.codec == "topk":
            words = topk.payload_words(self._kcap)
            slots = {w: torch.empty(words, dtype=torch.int32, device=self.device) for w in rank_of}
        else:
            wire_dtype = torch.float16 if self.cfg.codec == "fp16" else torch.float32
            slots = {w: torch.empty(n, dtype=wire_dtype, device=self.device) for w in rank_of}
        # one fetch snapshot per worker (codec wire buffers): an in-flight send never races the
        # next update of the arena
        from .codec import FetchCodec

        snaps = {w: FetchCodec(self.layout, self.cfg.fetch_codec, self.device) for w in rank_of}
        bufslots = {}
        pending_recv = []   # (wid, local_step, work, buffers_work)
        pending_send = {}   # wid -> [works]
        last_to = time.monotonic()
        while True:
            msg = mbox.recv(timeout=poll)
            if msg is not None and _TRACE:
                print(f"[psx-server] {msg} pending_recv={[p[0] for p in pending_recv]}", flush=True)
            if msg is not None:
                t, wid = msg.type, msg.a
                if t == CP.HELLO:
                    got, total = self.register_worker(f"rank{msg.src}", msg.a)
                    mbox.reply(msg.src, CP.Msg(CP.R_REGISTERED, 0, got, total))
                elif t == CP.FETCH:
                    gs = self.core.on_fetch(wid)
                    for prev in pending_send.pop(wid, []):
                        prev.wait()
                    pending_send[wid] = [transport.isend(b, rank_of[wid]) for b in snaps[wid].pack(self.arena)]
                    self.bytes_fetched += snaps[wid].nbytes
                    mbox.reply(rank_of[wid], CP.Msg(CP.R_FETCHED, 0, wid, 0, gs))
                elif t == CP.PUSH:
                    work = transport.irecv(slots[wid], rank_of[wid])
                    bwork = None
                    if msg.b:  # BN running statistics follow the gradients (--bn-sync)
                        if wid not in bufslots:
                            bufslots[wid] = torch.empty(self.layout.buffer_numel, dtype=torch.float32,
                                                        device=self.device)
                        bwork = transport.irecv(bufslots[wid], rank_of[wid])
                    pending_recv.append((wid, msg.c, work, bwork))
                elif t == CP.DONE:
                    finished.add(wid)
                    self.core.job_finished(wid)
                    mbox.reply(rank_of[wid], CP.Msg(CP.R_ACK, 0, wid))
                    self.log(f"[JobFinished] Worker {wid} completed")
                elif t == CP.HEARTBEAT:
                    self.core.heartbeat(wid)
                elif t == CP.STOP:
                    break
            # complete arrived pushes in arrival order
            keep = []
            for wid, ls, work, bwork in pending_recv:
                if transport.completed(work):  # each work is waited exactly once (gloo!)
                    if bwork is not None:
                        transport.completed(bwork) or bwork.wait()
                    res = self.core.on_push(wid, ls)
                    self.bytes_pushed += slots[wid].numel() * slots[wid].element_size()
                    if res.apply:
                        self.apply(slots[wid], res.weight)
                        if bwork is not None:
                            self.push_buffers(wid, bufslots[wid])
                        self.maybe_checkpoint()
                    mbox.reply(rank_of[wid], CP.Msg(CP.R_PUSHED, 0, wid, int(res.accepted), self.core.global_step,
                                                    res.staleness))
                else:
                    keep.append((wid, ls, work, bwork))
            pending_recv = keep
            stop = False
            if local_queue is not None:
                while True:
                    try:
                        kind, wid, grads, ls, ev, box = local_queue.get_nowait()
                    except Exception:
                        break
                    if kind == "push":
                        res = self.core.on_push(wid, ls)
                        self.bytes_pushed += min(n, grads.numel()) * grads.element_size()
                        if res.apply:
                            self.apply(grads, res.weight)
                            if box.get("bufs") is not None:
                                self.push_buffers(wid, box["bufs"])
                            self.maybe_checkpoint()
                        box["res"] = res
                        box["global_step"] = self.core.global_step
                    else:  # "done"
                        self.log(f"[JobFinished] Worker {wid} completed")
                        self.core.job_finished(wid)
                        finished.add(wid)
                    ev.set()
            now = time.monotonic()
            if self.cfg.heartbeat_timeout and now - last_to > 1.0:
                last_to = now
                for w in self.core.check_timeouts(self.cfg.heartbeat_timeout):
                    self.log(f"[Failure] worker {w} missed heartbeats for {self.cfg.heartbeat_timeout}s; marked dead")
                    finished.add(w)
            if stop_when_done and len(finished) >= expected and not pending_recv:
                break
        for works in pending_send.values():
            for w in works:
                w.wait()

