"""Job orchestration: one process per GPU (torchrun-style env) or a single loopback process.

Replaces the reference's deployment (one gRPC server container + N worker containers,
reference: terraform/main.tf:387-435, server.py:370-433, worker.py:455-506) with a single-node
layout on MI355X:

* ``world_size == 1``: the parameter server and ``--workers`` simulated workers share one
  GPU in one process (loopback): sync rounds aggregate in HBM, async pushes interleave
  round-robin so staleness reaches W-1 like W concurrent workers;
* ``world_size > 1``: RCCL over xGMI. Topology ``colocated`` (default): rank 0 hosts the PS
  state *and* worker 0, ranks 1..N-1 are workers (W = N); ``dedicated``: rank 0 is only the
  PS (W = N-1), the reference's server/worker split.
  - sync:  every step is fetch (RCCL broadcast) -> fwd/bwd -> push (RCCL reduce to rank 0 ->
    fused SGD apply of the average);
  - async: workers talk to the rank-0 server event loop (shared-memory mailbox for control,
    RCCL send/recv for tensors); the co-located worker of rank 0 runs next to the server loop.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
import uuid

import torch

from ..models.layout import ParamLayout
from ..models.resnet import MODEL_INPUT, build_model
from ..utils import metrics as M
from ..utils.data import DeviceDataset, shard_range, steps_per_epoch
from . import control as CP
from . import elastic
from .codec import FetchCodec, WeightWire, weight_image_enabled
from .compute import make_compute
from .graph_round import GraphRoundChannel, graph_round_enabled
from .native_loop import NativeAsyncChannel, NativeLocalChannel, NativeServerLoop, native_loop_enabled
from .overlap import OverlapSyncChannel, plan_buckets
from .server import ParameterServer
from .rccl import make_transport
from .sharded import ShardedSyncChannel
from .transport import LocalTransport, env_world
from .worker import (AsyncChannel, InProcessChannel, LocalAsyncChannel, SyncCollectiveChannel, Worker,
                     rounds_to_batches)


def _device_for(local_rank: int):
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _wire_dtype(cfg):
    """Dtype of the worker's dense gradient buffer: fp16 wire (reference cast), fp32 for the
    uncompressed wire and as the top-k codec's input (the residual is fp32)."""
    return torch.float16 if cfg.codec == "fp16" else torch.float32


def build_state(cfg):
    model = build_model(cfg.model, cfg.num_classes, seed=cfg.seed)
    layout = ParamLayout.from_module(model)
    arena, counters = layout.pack(model)
    return model, layout, arena, counters


def make_datasets(cfg, device, classes):
    (_, h, _), _ = MODEL_INPUT[cfg.model]
    if cfg.data_dir:
        tr = os.path.join(cfg.data_dir, "train.bin")
        te = os.path.join(cfg.data_dir, "test.bin")
        train = DeviceDataset.cifar_binary(tr, max_records=cfg.train_samples, device=device)
        test = DeviceDataset.cifar_binary(te, max_records=cfg.test_samples, device=device) if os.path.exists(te) else None
        return train, test
    gen = DeviceDataset.synthetic_hard if cfg.synthetic_kind == "hard" else DeviceDataset.synthetic
    train = gen(cfg.train_samples, h, classes, seed=cfg.seed, device=device)
    test = None
    if cfg.eval_every and cfg.test_samples:
        test = gen(cfg.test_samples, h, classes, seed=cfg.seed, device=device, offset=10_000_000)
    return train, test


def _common_steps(cfg, W, n):
    return max(steps_per_epoch(e - s, cfg.batch_size) for s, e in (shard_range(w, W, n) for w in range(W)))


# ---------------------------------------------------------------------------- loopback
def run_local(cfg, log=print, depart=None) -> dict:
    """W simulated workers on one device (see _interleave). ``depart`` = {worker id: rounds}: the
    loopback model of a sync shrink (parallel/elastic.py) — after that many sync rounds the worker
    leaves (the server marks it dead, the wait-for-N barrier shrinks) and every survivor forgets
    its BN statistic shifts, as a worker does when it re-enters the loop after a rollback. The
    elastic parity test (tests/test_elastic_gpu.py) compares a shrunk distributed job against it."""
    cfg.resolve_overlap(1)
    device = _device_for(0)
    W = cfg.workers
    model, layout, arena, counters = build_state(cfg)
    classes = model.fc.out_features
    server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W, log=log)
    train, test = make_datasets(cfg, device, classes)
    workers = []
    for w in range(W):
        m = model if w == 0 else build_model(cfg.model, cfg.num_classes, seed=cfg.seed)
        comp = make_compute(m, layout, cfg.batch_size, device, cfg.model, _wire_dtype(cfg), seed=cfg.seed + w,
                            use_graph=cfg.use_graph, dtype=cfg.dtype,
                            deterministic=cfg.deterministic)
        wk = Worker(cfg, comp, make_local_channel(cfg, server, layout, device), train, test,
                    worker_name=f"{cfg.worker_name}-{w}", rank=0, log=log, requested_id=w,
                    steps_per_epoch=_common_steps(cfg, W, len(train)))
        wk.connect_to_server()
        wk.setup_data()
        workers.append(wk)
    t0 = time.time()
    if W == 1 and not depart:
        workers[0].run_training()
    else:
        _interleave(cfg, workers, server, log, depart=depart)
    if device.type == "cuda":
        torch.cuda.synchronize()
    wall = time.time() - t0
    imgs = sum(w.images for w in workers)
    extra = {"images_per_second": round(imgs / wall, 2) if wall > 0 else 0.0, "gpus": 1, "topology": "loopback"}
    sm = server.final_metrics(emit=True, extra=extra)
    return {"server": sm, "workers": [getattr(w, "final_metrics", None) for w in workers]}


def run_local_threads(cfg, steps: int, log=print, emit: bool = True) -> dict:
    """Async PS on ONE device with W worker THREADS in real arrival order.

    The loopback (run_local) interleaves its W workers' pushes round-robin, so every push there
    has staleness exactly W - 1. Here each worker is a host thread with its own HIP stream, engine
    and step graph and its own data shard; all of them fetch from and push into the native event
    loop (csrc/server/event_loop.cpp, psx_loop_local_fetch / _push) as their steps complete, the
    way the reference's 20-thread gRPC pool receives concurrent workers (server.py:171-186,
    290-304): the staleness of a push is whatever number of other workers' updates landed since
    its fetch. The workers share the GPU, so this measures the server's staleness behaviour and
    its throughput over accepted pushes, not multi-GPU scaling.

    Each worker's first step (its HIP graph capture) runs on the main thread, one worker after the
    other (a capture must not overlap another thread's device-wide synchronize); then ``steps``
    more per worker on the threads, timed. Returns the server metrics plus the timed region's
    processed / accepted pushes and images per second counted over ACCEPTED pushes only."""
    assert cfg.mode == "async"
    cfg.resolve_overlap(1)
    device = _device_for(0)
    W = cfg.workers
    model, layout, arena, counters = build_state(cfg)
    server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W, log=log)
    train, test = make_datasets(cfg, device, model.fc.out_features)
    mbox = CP.ShmMailbox(f"/psx_thr_{uuid.uuid4().hex[:12]}", nreply=1, owner=True)
    loop = NativeServerLoop(server, None, mbox, {}, W, update_stream=None)
    workers = []
    try:
        for w in range(W):
            st = torch.cuda.Stream(device)
            with torch.cuda.stream(st):
                m = model if w == 0 else build_model(cfg.model, cfg.num_classes, seed=cfg.seed)
                comp = make_compute(m, layout, cfg.batch_size, device, cfg.model, _wire_dtype(cfg), seed=cfg.seed + w,
                                    use_graph=cfg.use_graph, dtype=cfg.dtype, deterministic=cfg.deterministic)
                wk = Worker(cfg, comp, NativeLocalChannel(server, loop), train, test,
                            worker_name=f"{cfg.worker_name}-{w}", rank=0, log=log, requested_id=w,
                            steps_per_epoch=_common_steps(cfg, W, len(train)))
                wk.connect_to_server()
                wk.setup_data()
                batches = wk.sampler.epoch_indices(0)
                wk.fetch_parameters()  # first step: the graph capture, one worker at a time
                wk.train_local_batch(batches[0])
                wk.push_gradients()
            workers.append((wk, st, batches))
        torch.cuda.synchronize()
        m0 = server.core.metrics()
        go, errs = threading.Barrier(W + 1), []

        def body(wk, st, batches):
            try:
                with torch.cuda.device(device), torch.cuda.stream(st):
                    go.wait()
                    wk.training_start_time = time.time()
                    for i in range(1, steps + 1):
                        wk.fetch_parameters()
                        wk.train_local_batch(batches[i % len(batches)])
                        wk.push_gradients()
                    st.synchronize()
            except Exception as e:  # noqa: BLE001 - reported after the join
                errs.append(e)

        ths = [threading.Thread(target=body, args=x, daemon=True) for x in workers]
        for th in ths:
            th.start()
        go.wait()
        t0 = time.perf_counter()
        for th in ths:
            th.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if errs:
            raise errs[0]
        m1 = server.core.metrics()
        for wk, _, _ in workers:
            wk.epoch_times.append(dt)
            if emit:
                wk.print_worker_statistics()  # WORKER_FINAL_METRICS (utils/results.py aggregates them)
    finally:
        for wk, _, _ in workers:
            wk.channel.finished(wk.worker_id)
        loop.join()
        mbox.close()
    done = int(m1.get("gradients_processed", 0)) - int(m0.get("gradients_processed", 0))
    acc = int(m1.get("async_updates", 0)) - int(m0.get("async_updates", 0))
    extra = {"images_per_second": round(acc * cfg.batch_size / dt, 2), "gpus": 1, "topology": "threads",
             "timed_pushes": done, "timed_accepted_pushes": acc, "timed_seconds": round(dt, 4),
             "images_per_second_all_pushes": round(done * cfg.batch_size / dt, 2)}
    sm = server.final_metrics(emit=emit, extra=extra)
    return {"server": sm, "workers": [getattr(w, "final_metrics", None) for w, _, _ in workers], "timed": extra}


def _interleave(cfg, workers, server, log, depart=None):
    """W simulated workers on one device. Sync: every worker fetches the same version, the last
    push of a round triggers the averaged update. Async: pipelined round-robin (each worker
    pushes gradients computed W-1 updates ago, then fetches), i.e. W equal-speed concurrent
    workers."""
    K = max(1, cfg.sync_steps)
    gone = set()
    for wk in workers:
        wk.training_start_time = time.time()
    steps = len(workers[0].sampler)
    for epoch in range(cfg.epochs):
        t_ep = time.time()
        batches = [wk.sampler.epoch_indices(epoch) for wk in workers]
        if cfg.mode == "async":
            for wk in workers:
                wk.fetch_parameters()
        for b in range(steps):
            if depart and cfg.mode == "sync" and b % K == 0:
                rnd = server.core.global_step
                for wid, after in depart.items():
                    if after == rnd and wid not in gone:
                        gone.add(wid)
                        server.core.mark_dead(wid)
                        for wk in workers:
                            if wk.worker_id not in gone and hasattr(wk.compute, "rewind"):
                                wk.compute.rewind(wk.compute._step)
            for wk, bt in zip(workers, batches):
                if wk.worker_id in gone:
                    continue
                if cfg.mode == "sync" and b % K == 0:
                    wk.fetch_parameters()
                wk.train_local_batch(bt[b])
                wk.window_push(b, steps, K)
                if cfg.mode == "async":
                    wk.fetch_parameters()
            if cfg.verbose and b % 50 == 0:
                log(f"  epoch {epoch + 1} batch {b}/{steps} loss(w0) {workers[0].compute.last_loss():.4f} "
                    f"global_step {server.core.global_step}")
            if cfg.max_steps and max(wk.local_step_counter for wk in workers) >= cfg.max_steps:
                break
        if server.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.time() - t_ep
        for wk in workers:
            wk.epoch_times.append(dt)
            if cfg.eval_every and (epoch + 1) % cfg.eval_every == 0:
                wk.evaluate_model()
        if cfg.max_steps and max(wk.local_step_counter for wk in workers) >= cfg.max_steps:
            break
    for wk in workers:
        wk.cleanup()
        wk.print_worker_statistics()


# ---------------------------------------------------------------------------- distributed
def run_distributed(cfg, log=print) -> dict:
    rank, world, local = env_world()
    cfg.resolve_overlap(world)
    device = _device_for(local)
    t = make_transport(device)
    dedicated = cfg.topology == "dedicated" and world > 1
    sharded = cfg.topology == "sharded"
    worker_ranks = list(range(1, world)) if dedicated else list(range(world))
    W = len(worker_ranks)
    wid_of_rank = {r: i for i, r in enumerate(worker_ranks)}
    if cfg.workers != W:
        if rank == 0 and cfg.verbose:
            log(f"[psx] {world} ranks, topology {cfg.topology}: total workers = {W} (overrides --workers {cfg.workers})")
        cfg.workers = W
    lg = log if rank == 0 else (lambda *a, **k: None)
    model, layout, arena, counters = build_state(cfg)
    classes = model.fc.out_features
    names = t.all_gather_object(f"{cfg.worker_name}-r{rank}")
    server = None
    if rank == 0:
        server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W, log=log)
    elif sharded:  # this rank's share of the server (parallel/sharded.py)
        server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W,
                                 log=lambda *a, **k: None)
    is_worker = rank in wid_of_rank
    train, test = make_datasets(cfg, device, classes) if is_worker else (None, None)
    n_train = max(t.all_gather_object(len(train) if train is not None else 0))
    steps = _common_steps(cfg, W, n_train)
    wk = None
    if is_worker:
        comp = make_compute(model, layout, cfg.batch_size, device, cfg.model, _wire_dtype(cfg),
                            seed=cfg.seed + wid_of_rank[rank], use_graph=cfg.use_graph, dtype=cfg.dtype,
                            deterministic=cfg.deterministic)
    # restart recovery: a server that resumed from a checkpoint tells every rank how many
    # global steps are already done (sync: one round per step; async: spread over workers)
    done = t.broadcast_object(server.core.global_step if rank == 0 else None)
    t0 = time.time()
    # sync job that survives a lost worker (parallel/elastic.py): a job-wide tag for its store keys
    shrink_on = cfg.mode == "sync" and cfg.round_timeout > 0 and elastic.enabled(cfg, t, world)
    ctx = {"t": t, "epoch": 0}
    if shrink_on:
        t.elastic_tag = t.broadcast_object(uuid.uuid4().hex[:12] if rank == 0 else None)
    if cfg.mode == "sync":
        if rank == 0:
            for r in worker_ranks:
                server.register_worker(names[r], wid_of_rank[r])
        if sharded:
            chan = ShardedSyncChannel(cfg, t, server, list(range(W)), layout, device, in_place=device.type == "cuda")
        else:
            chan = make_sync_channel(cfg, t, server, W, layout, device, worker=is_worker)
        chan._gs = done  # non-server ranks track the global step locally
        _attach_watchdog(cfg, chan, t, shrink_on)
        if is_worker:
            wk = Worker(cfg, comp, chan, train, test, worker_name=names[rank], rank=rank, log=lg,
                        requested_id=wid_of_rank[rank], steps_per_epoch=steps)
            wk.connect_to_server()
            if shrink_on and server is not None:  # co-located rank 0: server + worker 0
                chan.rollback = _PyRollback(server, chan)
                wk.recover = lambda e: _colocated_root_shrink(cfg, ctx, wk, server, layout, device, log)
            elif shrink_on:
                wk.recover = lambda e: _worker_shrink(cfg, ctx, wk, layout, device, log)
            wk.run_training(skip_steps=done)
            chan = wk.channel
        else:
            chan = _dedicated_sync_server(cfg, server, chan, steps, device, skip=done, t=t, ctx=ctx if shrink_on else None,
                                          log=log)
        t = ctx["t"]
    else:
        sess = AsyncSession(cfg, t, rank, worker_ranks, server, comp if is_worker else None, train, test, names, lg)
        sess.run_training(skip_steps=done // max(1, W))
        sess.close()
        wk = sess.worker
    if cfg.mode == "sync" and sharded:
        chan.gather_master()  # rank 0's arena = the full trained state (final metrics)
    if cfg.mode == "sync" and getattr(chan, "watchdog", None) is not None:
        chan.watchdog.stop()
    if device.type == "cuda":
        torch.cuda.synchronize()
    wall = time.time() - t0
    imgs = t.all_gather_object(wk.images if wk is not None else 0)
    result = {"worker": getattr(wk, "final_metrics", None)}
    if rank == 0:
        extra = {"images_per_second": round(sum(i for i in imgs if i) / wall, 2) if wall > 0 else 0.0, "gpus": world,
                 "topology": cfg.topology if world > 1 or sharded else "colocated"}
        if getattr(server, "dropped_workers", None):
            extra["dropped_workers"] = list(server.dropped_workers)
        server.images_processed = sum(i for i in imgs if i)
        result["server"] = server.final_metrics(emit=True, extra=extra)
    t.close()
    return result


class AsyncSession:
    """Rank-local roles of a multi-process async job.

    Rank 0 runs the parameter-server event loop (ParameterServer.serve_async: control requests
    on the shared-memory mailbox, tensors over RCCL point-to-point) in a thread, next to the
    co-located worker 0 (``colocated``) or alone (``dedicated``); every other rank is a worker
    talking to it through AsyncChannel, with a heartbeat thread for failure detection."""

    def __init__(self, cfg, t, rank, worker_ranks, server, comp, train, test, names, log):
        W = len(worker_ranks)
        wid_of_rank = {r: i for i, r in enumerate(worker_ranks)}
        rank_of_wid = {i: r for r, i in wid_of_rank.items()}
        self.t, self.rank = t, rank
        self.dropped_ranks = []    # rank 0: the worker ranks the native loop dropped
        self.self_dropped = False  # this worker was dropped by the server
        mbox_name = t.broadcast_object(f"/psx_{uuid.uuid4().hex[:12]}" if rank == 0 else None)
        self.tag = mbox_name.strip("/")
        self.mbox = CP.ShmMailbox(mbox_name, nreply=t.world_size, owner=True) if rank == 0 else None
        t.barrier()
        if rank != 0:
            self.mbox = CP.ShmMailbox(mbox_name, nreply=t.world_size, owner=False)
        remote = {w: r for w, r in rank_of_wid.items() if r != 0}
        if getattr(t, "native", False):  # one communicator + stream per (server, worker) pair
            t.open_pairs(sorted(remote.values()))
        self.worker, self.thread, self.hb, self.loop = None, None, None, None
        native = native_loop_enabled(cfg, t)  # the C++ server loop (parallel/native_loop.py)
        if rank == 0:
            if native:
                self.loop = NativeServerLoop(server, t, self.mbox, remote, W,
                                             update_stream=torch.cuda.current_stream() if rank in wid_of_rank else None)
                if rank in wid_of_rank:
                    self.worker = Worker(cfg, comp, NativeLocalChannel(server, self.loop), train, test,
                                         worker_name=names[0], rank=0, log=log, requested_id=wid_of_rank[0])
            else:
                q = queue.Queue() if rank in wid_of_rank else None
                self.thread = threading.Thread(target=server.serve_async, args=(t, self.mbox, remote),
                                               kwargs={"local_queue": q, "expected": W}, daemon=True)
                self.thread.start()
                if q is not None:
                    self.worker = Worker(cfg, comp, LocalAsyncChannel(server, q), train, test, worker_name=names[0],
                                         rank=0, log=log, requested_id=wid_of_rank[0])
        elif rank in wid_of_rank:
            cls = NativeAsyncChannel if native else AsyncChannel
            chan = cls(t, self.mbox, rank, codec=FetchCodec(comp.layout, cfg.fetch_codec, comp.device))
            self.worker = Worker(cfg, comp, chan, train, test, worker_name=names[rank], rank=rank, log=log,
                                 requested_id=wid_of_rank[rank])
        if self.worker is not None:
            self.worker.connect_to_server()
            if rank != 0:
                self.hb = CP.Heartbeat(self.mbox, self.worker.worker_id, rank,
                                       period=max(1.0, cfg.heartbeat_timeout / 6))
                self.hb.start()

    def run_training(self, skip_steps: int = 0):
        try:
            if self.worker is not None:
                self.worker.run_training(skip_steps=skip_steps)
        except CP.WorkerDropped as e:  # the server declared this worker dead: end cleanly
            self.self_dropped = True
            print(f"[psx] {e}", file=sys.stderr, flush=True)
        finally:
            self._stop()

    def finish(self):
        """End a manually driven worker loop (bench): JobFinished, then wait for the server."""
        try:
            if self.worker is not None:
                self.worker.cleanup()
        finally:
            self._stop()

    def _stop(self):
        if self.hb is not None:
            self.hb.stop()
            self.hb = None
        if self.thread is not None:
            self.thread.join()
            self.thread = None
        if self.loop is not None:
            try:
                self.loop.join()
            finally:
                self.dropped_ranks = list(self.loop.dropped_ranks)
                self.loop = None

    def close(self):
        """End of the async job. Rank 0 publishes the ranks its loop dropped; with none, a normal
        barrier; otherwise the transport continues among the live ranks (DistTransport.degrade)."""
        dead = self._end_state()
        if dead:
            self.t.degrade(dead, self.tag)
        self.t.barrier()
        self.mbox.close()

    def _end_state(self):
        import json

        if not getattr(self.t, "is_distributed", False) or self.t.world_size < 2:
            return []
        st = self.t._store()
        key = f"psx/{self.tag}/end"
        if self.rank == 0:
            st.set(key, json.dumps(sorted(self.dropped_ranks)))
        return json.loads(st.get(key))


def make_sync_channel(cfg, t, server, W, layout, device, worker: bool = True, members=None):
    """Sync-mode channel: bucketed + backward-overlapped when every batch is pushed; otherwise
    the serial round, on the WeightWire fast path when it applies (parallel/codec.py).
    ``members``: the worker ids of a round, in transport-rank order (default 0..W-1; a shrunk
    job's survivors otherwise)."""
    codec = FetchCodec(layout, cfg.fetch_codec, device)
    members = list(range(W)) if members is None else list(members)
    if cfg.overlap and max(1, cfg.sync_steps) == 1 and cfg.codec != "topk":
        buckets = plan_buckets(layout, int(cfg.bucket_mb * (1 << 20)) // 2)
        return OverlapSyncChannel(t, server, members=members, codec=codec, buckets=buckets, device=device,
                                  root_worker=server is None or worker)
    wire = None
    if weight_image_enabled(cfg) and torch.device(device).type == "cuda":
        if server is not None:
            server.enable_weight_wire()
        if graph_round_enabled(cfg, t):
            # rank 0's worker reads the server's wire in place; the others receive theirs
            wire = server.wire if server is not None else WeightWire(layout, device)
            buckets = plan_buckets(layout, int(cfg.bucket_mb * (1 << 20)) // 2)
            return GraphRoundChannel(t, server, list(range(W)), codec, wire, buckets, device)
        if worker:  # rank 0's worker reads the server's wire in place (stream-ordered round)
            wire = server.wire if server is not None else WeightWire(layout, device)
    return SyncCollectiveChannel(t, server, members=members, codec=codec, wire=wire,
                                 root_worker=server is None or worker)


def make_local_channel(cfg, server, layout, device, emit_on_last: bool = False):
    """Loopback channel of one simulated worker (WeightWire fast path when it applies)."""
    wire = None
    if weight_image_enabled(cfg) and torch.device(device).type == "cuda":
        if server.wire is None:
            server.enable_weight_wire()
        # sync rounds: the worker reads the server's wire in place (no per-fetch copy)
        wire = server.wire
    return InProcessChannel(server, emit_on_last=emit_on_last, wire=wire)


def _sync_rounds(cfg, steps, skip_b):
    """Rounds a worker runs (fetch + push every K-th batch of an epoch, --max-steps) from its
    batch ``skip_b`` on: the dedicated server takes part in exactly these."""
    K = max(1, cfg.sync_steps)
    rounds, done = 0, skip_b
    for epoch in range(cfg.epochs):
        for b in range(steps):
            if epoch * steps + b < skip_b:
                continue
            if b % K == 0:
                rounds += 1
            done += 1
            if cfg.max_steps and done >= cfg.max_steps:
                return rounds
    return rounds


def _attach_watchdog(cfg, chan, t, shrink_on: bool, freeze=None):
    """The round watchdog of a sync channel (--round-timeout): exit 3 for a launcher restart, or
    (shrink) abort + recover in-process (parallel/elastic.py)."""
    world = getattr(t, "world_size", 1)
    if cfg.round_timeout > 0 and (world > 1 or getattr(t, "base", None) is not None) and hasattr(chan, "watchdog"):
        from .liveness import RoundWatchdog

        name = f" rank {getattr(t, 'orig_rank', getattr(t, 'rank', 0))}"
        on_expire = elastic.make_on_stall(t, freeze=freeze) if shrink_on else None
        chan.watchdog = RoundWatchdog(cfg.round_timeout, comm=getattr(t, "comm", None), name=name,
                                      on_expire=on_expire)
    return chan


def _shrink_grace(cfg) -> float:
    return cfg.recovery_grace if cfg.recovery_grace > 0 else cfg.round_timeout


def _worker_shrink(cfg, ctx, wk, layout, device, log):
    """A worker's side of a shrink (parallel/elastic.py): check in, build the survivors'
    communicator, rebind to a new channel; returns the rounds the job keeps."""
    old = ctx["t"]
    wd = getattr(wk.channel, "watchdog", None)
    if wd is not None:
        wd.stop()
    # the communicator is aborted only if the watchdog fired; an RcclError raised straight from an
    # enqueue leaves collectives queued for the dead peer spinning, and the synchronize below would
    # then block with no watchdog running. Abort here (a no-op on an already aborted handle).
    old.lost = True
    try:
        old.comm.destroy(abort=True)
    except Exception:  # noqa: BLE001
        pass
    try:
        torch.cuda.synchronize()  # the aborted collectives have run out
    except Exception:  # noqa: BLE001
        pass
    ctx["epoch"] += 1
    nt, rounds, dead = elastic.shrink(old, ctx["epoch"], _shrink_grace(cfg), log=log)
    ctx["t"] = nt
    W = nt.world_size - (1 if cfg.topology == "dedicated" else 0)  # co-located: rank 0 trains too
    chan = make_sync_channel(cfg, nt, None, W, layout, device, worker=True)
    chan._gs = rounds
    _attach_watchdog(cfg, chan, nt, True)
    wk.rebind(chan)
    return rounds


def _colocated_root_shrink(cfg, ctx, wk, server, layout, device, log):
    """Rank 0 of a shrinking co-located job (server + worker 0) when the communicator is lost:
    abort it, roll the arena back to the first round not known complete (the channel's
    _PyRollback, fed by every fetch / push), publish the plan as the server, mark the lost workers
    dead (co-located: worker id = rank) and continue on a new channel over the survivors."""
    old = ctx["t"]
    chan = wk.channel
    if chan.watchdog is not None:
        chan.watchdog.stop()
    old.lost = True
    try:
        old.comm.destroy(abort=True)
    except Exception:  # noqa: BLE001
        pass
    try:
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001
        pass
    kept = chan.rollback.rollback() if chan.rollback is not None else server.core.global_step
    ctx["epoch"] += 1
    nt, rounds, dead = elastic.shrink(old, ctx["epoch"], _shrink_grace(cfg), rounds_kept=kept, log=log)
    if not dead:
        raise RuntimeError(f"sync shrink epoch {ctx['epoch']}: no rank was lost; failing the job")
    ctx["t"] = nt
    for r in dead:
        server.core.mark_dead(r)
    server.dropped_workers = sorted(set(getattr(server, "dropped_workers", None) or []) | set(dead))
    members = list(nt.members)  # worker ids in the new communicator's rank order
    nchan = make_sync_channel(cfg, nt, server, len(members), layout, device, worker=True, members=members)
    nchan._gs = rounds
    _attach_watchdog(cfg, nchan, nt, True)
    nchan.rollback = _PyRollback(server, nchan)
    wk.rebind(nchan)
    return rounds


def _dedicated_sync_server(cfg, server, chan, steps, device, skip=0, t=None, ctx=None, log=print):
    """Rank 0 of the dedicated topology: takes part in every round's collectives with a zero
    gradient contribution and applies the averaged update — all rounds in one native call
    (parallel/native_sync.py) on the native transport, else per round in Python. With ``ctx``
    (sync shrink, parallel/elastic.py) a lost worker ends the current run: the arena goes back to
    the last good round, the survivors rebuild the communicator and the rounds go on from there.
    Returns the channel in use at the end."""
    K = max(1, cfg.sync_steps)
    from .native_sync import NativeSyncServer, native_sync_enabled

    while True:
        try:
            _server_rounds(cfg, server, chan, steps, device, skip, t, ctx)
            return chan
        except Exception as e:  # noqa: BLE001 - only a lost communicator is recovered
            if ctx is None or not elastic.lost_error(e):
                raise
            log(f"[psx elastic] server: {type(e).__name__}: {e}")
            if chan.watchdog is not None:
                chan.watchdog.stop()
            kept = getattr(chan, "_rollback_gs", server.core.global_step)
            ctx["epoch"] += 1
            t, rounds, dead = elastic.shrink(ctx["t"], ctx["epoch"], _shrink_grace(cfg), rounds_kept=kept, log=log)
            ctx["t"] = t
            if not dead:
                # every worker checked in: nothing was lost, so the failure is not a departed peer
                # and another epoch would only repeat it (each shrink must drop at least one rank)
                raise RuntimeError(f"sync shrink epoch {ctx['epoch']}: no rank was lost; failing the job "
                                   f"instead of retrying ({type(e).__name__}: {e})") from e
            for r in dead:  # dedicated topology: worker id = original rank - 1
                server.core.mark_dead(r - 1)
            server.dropped_workers = sorted(set(getattr(server, "dropped_workers", None) or []) | {r - 1 for r in dead})
            members = [r - 1 for r in t.members if r != 0]
            chan = make_sync_channel(cfg, t, server, len(members), server.layout, device, worker=False,
                                     members=members)
            chan._gs = rounds
            _attach_watchdog(cfg, chan, t, True)
            skip = rounds


def _server_rounds(cfg, server, chan, steps, device, skip, t, ctx):
    """One run of the dedicated server's rounds from round ``skip`` on (see _dedicated_sync_server).
    On a lost communicator (shrink) it records on ``chan._rollback_gs`` the global step it rolled
    the arena back to, then re-raises."""
    K = max(1, cfg.sync_steps)
    from .native_sync import NativeSyncServer, native_sync_enabled

    if t is not None and native_sync_enabled(cfg, t, chan, server, getattr(t, "rank", 0)):
        srv = NativeSyncServer(server, t, chan, elastic=ctx is not None)
        if ctx is not None and chan.watchdog is not None:
            chan.watchdog.on_expire = elastic.make_on_stall(t, freeze=srv.abort)
        try:
            srv.run(_sync_rounds(cfg, steps, rounds_to_batches(skip, steps, K)), watchdog=chan.watchdog)
        except Exception:
            if ctx is not None:
                chan._rollback_gs = srv.rollback()
            raise
        finally:
            srv.close()
        if hasattr(chan, "drain"):
            chan.drain()
        return
    if cfg.codec == "topk":
        from .topk import empty_payload

        zeros = empty_payload(server.n, cfg.topk_ratio, device)  # contributes no entries to the gather
    else:
        zeros = torch.zeros(server.n, dtype=_wire_dtype(cfg), device=device)
    zbuf = torch.zeros(server.layout.buffer_numel, dtype=torch.float32, device=device) if cfg.bn_sync else None
    skip_b = rounds_to_batches(skip, steps, K)  # checkpointed rounds -> batches (window aligned)
    done = skip_b
    rb = _PyRollback(server, chan) if ctx is not None else None
    try:
        for epoch in range(cfg.epochs):
            for b in range(steps):
                if epoch * steps + b < skip_b:
                    continue
                if b % K == 0:
                    if rb is not None:
                        rb.round_start()
                    chan.fetch(None, None)
                    if cfg.codec != "topk":
                        zeros.zero_()
                    if zbuf is not None:
                        zbuf.zero_()
                    chan.push(None, zeros, server.core.global_step, buffers=zbuf)
                    if rb is not None:
                        rb.round_end()
                done += 1
                if cfg.max_steps and done >= cfg.max_steps:
                    break
            else:
                continue
            break
    except Exception:
        if rb is not None:
            chan._rollback_gs = rb.rollback()
        raise
    if hasattr(chan, "drain"):
        chan.drain()


class _PyRollback:
    """The Python server loop's side of a shrink (native: sync_loop.cpp snapshots): the arena (and
    momentum) at every round start in one of three snapshot slots, a device event after every
    round; the watchdog thread freezes the count of rounds whose event completed before it
    aborted the communicator (``freeze``).

    As the native loop (retire(S, 2)), at most two rounds are in flight: round n's start waits
    for round n-2's event before it overwrites slot n % 3 (round n-3's snapshot), so every
    rollback target (a round >= the completed count) still has its snapshot. Every unretired
    event is kept, so the completed count never assumes an unobserved round finished."""

    NSLOT = 3

    def __init__(self, server, chan):
        self.s = server
        self.snap = [torch.empty_like(server.arena) for _ in range(self.NSLOT)]
        self.msnap = ([torch.empty_like(server.momentum_buf) for _ in range(self.NSLOT)]
                      if server.momentum_buf is not None else None)
        self.gs0 = server.core.global_step
        self.mom_first0 = server._mom_first
        self.issued = 0        # rounds whose device work was enqueued (round_end)
        self.snapped = -1      # the last round whose starting state is in its slot
        self.retired = 0       # rounds [0, retired) waited on (host-observed complete)
        self.events = []       # (round, event) of every round >= retired
        self.frozen = None
        if chan.watchdog is not None:
            chan.watchdog.on_expire = elastic.make_on_stall(chan.t, freeze=self.freeze)

    def round_start(self):
        n = self.issued
        # bound the rounds in flight: round n-2 done before slot n % 3 (round n-3) is reused
        while self.events and self.events[0][0] <= n - 2:
            i, ev = self.events[0]
            ev.synchronize()
            self.events.pop(0)
            self.retired = i + 1
        k = n % self.NSLOT
        self.snap[k].copy_(self.s.arena)
        if self.msnap is not None:
            self.msnap[k].copy_(self.s.momentum_buf)
        self.snapped = n

    def round_end(self):
        ev = torch.cuda.Event()
        ev.record()
        self.events.append((self.issued, ev))
        self.issued += 1

    def _completed(self) -> int:
        g = self.retired
        for i, ev in list(self.events):
            if not ev.query():
                break
            g = i + 1
        return g

    def freeze(self):
        self.frozen = self._completed()

    def rollback(self) -> int:
        torch.cuda.synchronize()
        g = self.frozen if self.frozen is not None else self.issued  # a failed round never ended
        g = max(min(g, self.issued), self.issued - (self.NSLOT - 1), 0)
        if g <= self.snapped:  # g == issued with no snapshot taken yet: the arena is that state
            self.s.arena.copy_(self.snap[g % self.NSLOT])
            if self.msnap is not None:
                self.s.momentum_buf.copy_(self.msnap[g % self.NSLOT])
        if g == 0:
            self.s._mom_first = self.mom_first0
        self.s.core.rollback_to(self.gs0 + g)
        self.s._wire_stale = self.s.wire is not None
        torch.cuda.synchronize()
        return self.gs0 + g


def run(cfg, log=print) -> dict:
    _, world, _ = env_world()
    if world <= 1:
        return run_local(cfg, log=log)
    return run_distributed(cfg, log=log)


def main(argv=None):
    from ..utils.config import parse

    cfg = parse(argv, description="psx MI355X parameter-server training (rank per GPU)")
    res = run(cfg)
    return 0 if res is not None else 1


if __name__ == "__main__":
    raise SystemExit(main())
