#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node) of ResNet-18 / CIFAR-100-shaped data in the
synchronous parameter-server mode on 1..8 MI355X (BASELINE.json metric), at the reference's
training precision (fp32).

  python bench.py                                   # N=1: server + worker co-located (one RCCL rank)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

One step = fetch (RCCL broadcast from rank 0 of the fp32 parameter state, 44.9 MB — the
reference's FetchParameters payload) -> batch gather + augment -> forward/backward on the HIP
engine (hand-written CDNA4 kernels, fp32 on the exact-f32 MFMA, HIP graphs) -> push (the fp16
wire gradients — the reference's codec — gathered to rank 0 over RCCL point-to-point) -> fused
update on rank 0: every wire decoded and summed in fp32, p -= lr * sum / W (reference
server.py:126-169, 232-237). Batch 128 per worker, lr 0.1, sync period 1 (the reference's CLI
defaults). Topology: N = 1 co-locates the server and the worker on one GPU; N >= 2 runs the
reference's layout (BASELINE configs 2-4): rank 0 = the parameter server only, ranks 1..N-1 =
workers (``--topology dedicated``); ``--topology colocated`` makes rank 0 a worker as well.
W warmup steps are untimed; exactly K steps are timed between barrier+synchronize pairs and
the max over ranks is reported. Data is synthetic CIFAR-100-shaped (no network access), weights
random-init.

Secondary numbers (``"secondary"`` in the JSON line, each measured after the headline with the
same transport, ``--secondary none`` skips them): the bf16 compute path (N = 1) and the
co-located topology (N >= 2).

Liveness at N >= 2: every rank runs a RoundWatchdog (parallel/liveness.py) over its sync rounds
(``--round-timeout``, default 120 s): a rank whose round does not complete in time prints what was
outstanding (the collective, the native server's issued / completed rounds) and the fallback
switches, aborts its communicator and exits with status 3 — a hang never rides to the launcher's
timeout. The JSON reports the ranks the RCCL communicator saw (``rccl_ranks``, ncclCommCount).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel.compute import HipCompute  # noqa: E402
from psx.parallel.liveness import RoundWatchdog  # noqa: E402
from psx.parallel.runner import (AsyncSession, build_state, make_datasets, make_local_channel,  # noqa: E402
                                 make_sync_channel)
from psx.parallel.server import ParameterServer  # noqa: E402
from psx.parallel.sharded import ShardedSyncChannel  # noqa: E402
from psx.parallel.native_sync import NativeSyncServer, native_sync_enabled  # noqa: E402
from psx.parallel.rccl import make_transport  # noqa: E402
from psx.parallel.transport import env_world  # noqa: E402
from psx.parallel.worker import Worker  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402

BASELINE_SYNC_IMG_S = 82.7  # sync PS, 4 workers, measured (experiment_results/sync_4workers.json)
BASELINE_ASYNC_IMG_S = 168.6  # async PS, 8 workers, measured (experiment_results/async_8workers.json)
FALLBACK_HINT = ("; fallbacks to try: PSX_PAIR_COMMS=0 (async point-to-point on the job communicator), "
                 "PSX_SYNC_AGG=reduce (ncclReduce instead of the send/recv gather), --overlap off (serial "
                 "rounds), PSX_NATIVE_SYNC=0 (Python server rounds), PSX_TRANSPORT=torch (torch.distributed)")


class Run:
    """One benchmark configuration on the shared transport: server / worker / channel objects."""

    def __init__(self, a, t, rank, world, device, dtype, topology):
        self.a, self.t, self.rank, self.world = a, t, rank, world
        n_train = a.train_samples or (50000 if a.model == "resnet18" else 4096)
        self.n_train = n_train
        self.cfg = cfg = PSConfig(mode=a.mode, staleness_bound=a.staleness_bound, model=a.model, batch_size=a.batch,
                                  train_samples=n_train, lr=0.1, sync_steps=1, epochs=1, eval_every=0, verbose=0,
                                  codec=a.codec, topk_ratio=a.topk_ratio, use_graph=not a.no_graph,
                                  fetch_codec=a.fetch_codec, bucket_mb=a.bucket_mb,
                                  overlap={"auto": None, "on": True, "off": False}[a.overlap],
                                  topology=topology, dtype=dtype).validate()
        cfg.resolve_overlap(world)
        model, layout, arena, counters = build_state(cfg)
        self.layout = layout
        wire = torch.float16 if a.codec == "fp16" else torch.float32  # topk encodes from fp32 grads
        self.sharded = sharded = topology == "sharded"
        self.dedicated = dedicated = topology == "dedicated" and world > 1
        worker_ranks = list(range(1, world)) if dedicated else list(range(world))
        self.W = W = len(worker_ranks)
        cfg.workers = W
        is_worker = rank in worker_ranks
        self.server = None
        quiet = lambda *x, **k: None  # noqa: E731
        self.async_dist = async_dist = a.mode == "async" and t is not None
        if rank == 0 or sharded:
            self.server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W, log=quiet)
            if not async_dist and rank == 0:
                for i in range(W):
                    self.server.register_worker(f"worker-{i}", i)
        train, _ = make_datasets(cfg, device, model.fc.out_features)
        comp = HipCompute(model, layout, a.batch, device, a.model, wire, seed=rank, use_graph=cfg.use_graph,
                          dtype=cfg.dtype) if is_worker else None
        self.wk = self.sess = self.chan = self.zeros = None
        if async_dist:  # server event loop thread on rank 0, mailbox + RCCL p2p (parallel/runner.py)
            names = [f"worker-r{r}" for r in range(world)]
            self.sess = AsyncSession(cfg, t, rank, worker_ranks, self.server, comp, train, None, names, quiet)
            self.wk = self.sess.worker
        else:
            if sharded:
                self.chan = ShardedSyncChannel(cfg, t, self.server, list(range(W)), layout, device, in_place=True)
            else:
                self.chan = (make_local_channel(cfg, self.server, layout, device) if t is None else
                             make_sync_channel(cfg, t, self.server, W, layout, device, worker=is_worker))
            if is_worker:
                wid = worker_ranks.index(rank)
                self.wk = Worker(cfg, comp, self.chan, train, None, worker_name=f"worker-{wid}", rank=rank, log=quiet,
                                 requested_id=wid)
                self.wk.connect_to_server()
        self.native = None
        self.watchdog = None
        if t is not None and world > 1 and a.round_timeout > 0 and not async_dist:
            self.watchdog = RoundWatchdog(a.round_timeout, comm=getattr(t, "comm", None), name=f" rank {rank}",
                                          hint=FALLBACK_HINT)
            if hasattr(self.chan, "watchdog"):
                self.chan.watchdog = self.watchdog
        stall = a.stall_rank.split("@") if a.stall_rank else None
        self.stall_at = int(stall[1]) if stall and int(stall[0]) == rank else -1
        if self.wk is not None:
            self.wk.setup_data()
            self.batches = self.wk.sampler.epoch_indices(0)
        elif self.sess is not None:
            pass  # dedicated async server rank: its event-loop thread does the work
        elif native_sync_enabled(cfg, t, self.chan, self.server, rank):
            # dedicated sync server rank: every round of a run in one native call (no Python per
            # round; csrc/server/sync_loop.cpp)
            self.native = NativeSyncServer(self.server, t, self.chan)
        elif a.codec == "topk":
            from psx.parallel.topk import empty_payload

            self.zeros = empty_payload(layout.param_numel, a.topk_ratio, device)
        else:
            self.zeros = torch.zeros(layout.param_numel, dtype=wire, device=device)

    def step(self, i):
        if i == self.stall_at:  # test hook (--stall-rank): this rank stops taking part in rounds
            print(f"[bench] rank {self.rank} stalls at step {i} (--stall-rank)", file=sys.stderr, flush=True)
            while True:
                time.sleep(3600)
        if self.wk is not None:
            self.wk.fetch_parameters()
            self.wk.train_local_batch(self.batches[i % len(self.batches)])
            self.wk.push_gradients()
        elif self.sess is not None:
            pass
        else:  # dedicated sync server rank: joins the fetch and push collectives, applies
            self.chan.fetch(None, None)
            if self.a.codec != "topk":
                self.zeros.zero_()
            self.chan.push(None, self.zeros, self.server.core.global_step)

    def barrier_sync(self):
        wd = self.watchdog
        if wd is not None:
            wd.begin("barrier + device synchronize between warmup and timed steps")
        try:
            torch.cuda.synchronize()
            if self.t is not None:
                self.t.barrier()  # host barrier on the gloo control group
            torch.cuda.synchronize()
        finally:
            if wd is not None:
                wd.end()

    def measure(self, steps, warmup):
        """Untimed warmup, then exactly ``steps`` timed steps; returns (max seconds over ranks,
        host issue times of this rank)."""
        self.server_round_us = None
        if self.native is not None:  # the native server rank runs its rounds in one call each
            self.native.run(warmup, watchdog=self.watchdog)
            self.barrier_sync()
            p0 = self.native.phase_totals()  # the warmup rounds are retired (run() drains)
            t0 = time.perf_counter()
            self.native.run(steps, watchdog=self.watchdog)
            p1 = self.native.phase_totals()
            host = None  # no per-step host issue: every round was issued by one native call
            nr = p1[0] - p0[0]
            if nr > 0:  # rank 0's device time per timed round, per phase (sync_loop.cpp psx_sync_phase_us)
                self.server_round_us = {k: round((p1[i] - p0[i]) / nr, 1)
                                        for i, k in ((1, "gather_incl_worker_wait"), (2, "apply"), (3, "broadcast"))}
                self.server_round_us["rounds"] = nr
        else:
            for i in range(warmup):
                self.step(i)
            self.barrier_sync()
            host = []
            t0 = time.perf_counter()
            for i in range(steps):
                h0 = time.perf_counter()
                self.step(warmup + i)
                host.append(time.perf_counter() - h0)
        self.barrier_sync()
        dt = time.perf_counter() - t0
        if self.t is not None:
            dt = max(self.t.all_gather_object(dt))  # the slowest rank's time (gloo control group)
        return dt, host

    def parallelism(self):
        a, W = self.a, self.W
        if self.sharded:
            return (f"sharded sync-PS: {W} ranks, each a worker + 1/{W} of the server; RCCL reduce-scatter(grads) "
                    f"+ all-gather(params) over xGMI")
        if self.t is None:
            return f"{a.mode}-PS: server + 1 worker co-located on 1 GPU"
        agg = os.environ.get("PSX_SYNC_AGG", "gather")
        push = ("RCCL send/recv gather of the fp16 wires to rank 0 + fp32 aggregation" if agg == "gather" else
                "RCCL reduce(grads)")
        if self.native is not None:
            push += " (server rounds in native code)"
        return (f"{a.mode}-PS: rank0 = parameter server{' only' if self.dedicated else ' + worker 0'}, {W} "
                f"data-parallel worker(s); " + (f"{push} + RCCL broadcast(params) over xGMI" if a.mode == "sync" else
                                                 "shm mailbox control + RCCL send/recv over xGMI"))

    def topology_name(self):
        if self.sharded:
            return "sharded"
        if self.dedicated:
            return "dedicated"
        return "colocated" if self.t is not None else "loopback"

    def close(self):
        if self.watchdog is not None:
            self.watchdog.stop()
            self.watchdog = None
        if self.native is not None:
            self.native.close()
        if self.sess is not None:
            self.sess.finish()
            self.sess.close()
        if hasattr(self.chan, "drain"):
            self.chan.drain()


def rccl_choices(path, limit=24):
    """The distinct algorithm / protocol / channel lines of RCCL's INFO log (NCCL_DEBUG_FILE of this
    rank), printed on stderr and returned for the JSON record; [] when there is no log."""
    import re

    seen, out = set(), []
    try:
        with open(path, errors="replace") as f:
            for ln in f:
                if not re.search(r"(?i)algo|proto|channels|rings|trees", ln):
                    continue
                key = re.sub(r"0x[0-9a-f]+|\b\d+\b", "#", ln.split("NCCL INFO")[-1]).strip()
                if key in seen:
                    continue
                seen.add(key)
                out.append(ln.split("NCCL INFO")[-1].strip()[:200])
                if len(out) >= limit:
                    break
    except OSError:
        return []
    for ln in out:
        print(f"[bench rccl] {ln}", file=sys.stderr, flush=True)
    return out


def async_threads(a, W: int) -> dict:
    """BASELINE config 4's async PS with W = 7 workers on ONE GPU: W worker threads, each with its
    own HIP stream, engine and graph, pushing into the native event loop in real arrival order
    (parallel/runner.py run_local_threads). img/s counts ACCEPTED pushes only; the staleness
    histogram is the distribution those arrivals produced (bound --staleness-bound)."""
    from psx.parallel.runner import run_local_threads

    try:
        steps = max(5, min(a.steps, 20))
        cfg = PSConfig(mode="async", staleness_bound=a.staleness_bound, model=a.model, batch_size=a.batch,
                       train_samples=a.train_samples or 50000, lr=0.1, sync_steps=1, epochs=1, eval_every=0,
                       verbose=0, codec="fp16", use_graph=not a.no_graph, fetch_codec="fp32", workers=W,
                       dtype=a.dtype).validate()
        res = run_local_threads(cfg, steps, log=lambda *x, **k: None, emit=False)
        sm, tm = res["server"], res["timed"]
        hist = sm.get("staleness_histogram") or []
        return {"value": tm["images_per_second"], "unit": "images/s (accepted pushes only)",
                "ms_per_round": round(1e3 * tm["timed_seconds"] / steps, 4), "dtype": a.dtype, "workers": W,
                "topology": "threads (W worker threads + native event loop on 1 GPU)", "steps_per_worker": steps,
                "timed_pushes": tm["timed_pushes"], "timed_accepted_pushes": tm["timed_accepted_pushes"],
                "images_per_second_all_pushes": tm["images_per_second_all_pushes"],
                "vs_baseline_async_8w": round(tm["images_per_second"] / BASELINE_ASYNC_IMG_S, 2),
                "async_staleness": {k: sm.get(k) for k in ("average_gradient_staleness", "max_staleness_observed",
                                                           "mean_staleness_all", "async_updates", "rejected_pushes",
                                                           "staleness_histogram", "staleness_bound")},
                "max_staleness_accepted": max((i for i, n in enumerate(hist[: a.staleness_bound + 1]) if n),
                                              default=0)}
    except Exception as e:  # noqa: BLE001 - a secondary number never costs the headline
        return {"error": f"{type(e).__name__}: {e}"[:300]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--model", choices=["resnet18", "resnet50"], default="resnet18",
                    help="resnet18: the headline CIFAR-100 config; resnet50: BASELINE config 5 (ImageNet "
                         "shape, use with --codec topk)")
    ap.add_argument("--train-samples", type=int, default=None,
                    help="synthetic dataset size in HBM (default 50000 for resnet18, 4096 for resnet50)")
    ap.add_argument("--topology", choices=["auto", "colocated", "dedicated", "sharded"], default="auto",
                    help="auto: colocated at N=1, dedicated (1 server + N-1 workers, the reference's layout) at "
                         "N>=2; sharded: every rank is a worker and owns 1/N of the server (parallel/sharded.py)")
    ap.add_argument("--codec", choices=["fp16", "none", "topk"], default="fp16")
    ap.add_argument("--topk-ratio", type=float, default=0.01)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="worker compute precision. fp32 (default, the headline): the reference's training "
                         "precision (worker.py:333-348), every conv product on the exact-f32 MFMA; bf16: bf16 "
                         "operands with fp32 accumulation and fp32 master weights")
    ap.add_argument("--fetch-codec", choices=["auto", "bf16conv", "fp32"], default="auto",
                    help="auto: fp32 for --dtype fp32, bf16conv for bf16. bf16conv: conv weights travel as the "
                         "bf16 bits the workers compute with, everything else fp32; fp32: the reference's full "
                         "fp32 state")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="stream gradient buckets (gather/apply/broadcast) during the backward pass; auto: on "
                         "with >= 2 ranks (sync, dense wire), off at N=1")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--host-timing", action="store_true", help="report host-side issue time per step (stderr)")
    ap.add_argument("--mode", choices=["sync", "async"], default="sync",
                    help="async: workers push/fetch independently (staleness-weighted server updates)")
    ap.add_argument("--staleness-bound", type=int, default=5)
    ap.add_argument("--secondary", choices=["auto", "none"], default="auto",
                    help="auto: after the headline also time the bf16 compute path (N=1) or the co-located "
                         "topology (N>=2), reported under 'secondary'")
    ap.add_argument("--round-timeout", type=float, default=120.0,
                    help="N>=2: a rank whose sync round does not complete within this many seconds reports the "
                         "outstanding collective, aborts its communicator and exits with status 3 (0: off)")
    ap.add_argument("--stall-rank", default="", help=argparse.SUPPRESS)  # test hook "RANK@STEP"
    a = ap.parse_args()

    rank, world, local = env_world()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs MI355X GPUs")
    torch.cuda.set_device(local % torch.cuda.device_count())
    device = torch.device("cuda", torch.cuda.current_device())
    topology = a.topology if a.topology != "auto" else ("dedicated" if world >= 2 else "colocated")
    if a.fetch_codec == "auto":
        a.fetch_codec = "fp32" if a.dtype == "fp32" else "bf16conv"

    rccl_log = None
    if world > 1 and os.environ.get("PSX_RCCL_ALGO_LOG", "1") == "1" and "NCCL_DEBUG" not in os.environ:
        # RCCL's chosen algorithm / protocol per collective (INIT + TUNING subsystems) into a
        # per-rank file; rank 0 prints the distinct choices on stderr after the run
        rccl_log = f"/tmp/psx_rccl_{os.getpid()}.log"
        os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,TUNING", NCCL_DEBUG_FILE=rccl_log)
    t = None
    # sync at N = 1 runs the distributed path too (one rank: psx communicator, rank 0 = server +
    # worker 0), the same code as N > 1; measured equal to or faster than the in-process loopback
    # (one box 1.777/1.778 vs 1.842/1.829 ms/step, another 1.843 vs 1.853 mean of 3 interleaved).
    # PSX_FORCE_DIST=0: in-process loopback.
    force_dist = os.environ.get("PSX_FORCE_DIST", "1" if a.mode == "sync" else "0") == "1"
    if world > 1 or force_dist or topology == "sharded":
        if "RANK" not in os.environ:  # single process without torchrun: a world of one rank
            import socket

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        t = make_transport(device)

    run = Run(a, t, rank, world, device, a.dtype, topology)
    dt, host = run.measure(a.steps, a.warmup)
    W = run.W
    imgs = a.steps * a.batch * W
    value = imgs / dt
    loss = run.wk.compute.last_loss() if run.wk is not None else None
    r18 = a.model == "resnet18"
    cfg = run.cfg
    rec = None
    if rank == 0:
        rec = {
            "metric": ("images/sec (whole node) ResNet-18 sync-PS at 1/2/4/8 MI355X; async staleness" if r18 else
                       "images/sec (whole node) ResNet-50 ImageNet-shape sync-PS + top-k (BASELINE config 5)"),
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * dt / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_SYNC_IMG_S, 2) if r18 else None,
            "dtype": cfg.dtype,
            "data": (f"synthetic CIFAR-100-shaped ({run.n_train}x32x32x3 uint8 in HBM, on-device crop/flip/normalize), "
                     "random-init weights" if r18 else
                     f"synthetic ImageNet-shaped ({run.n_train}x224x224x3 uint8 in HBM, on-device crop/flip/normalize), "
                     "random-init weights"),
            "config": {
                "model": ("resnet18-cifar (11,220,132 params, reference ResNet18(num_classes=100))" if r18 else
                          f"resnet50-imagenet ({run.layout.param_numel:,} params, 1000 classes)"),
                "global_batch": a.batch * W,
                "per_worker_batch": a.batch,
                "seq_len": None,
                "parallelism": run.parallelism(),
                "mode": a.mode,
                "lr": 0.1,
                "sync_steps": 1,
                "codec": a.codec if a.codec != "topk" else f"topk({a.topk_ratio}) + error feedback",
                "fetch_codec": cfg.fetch_codec if t is not None else "in-process",
                "weight_image": getattr(run.chan, "image_wire", None) is not None or run.sharded,
                "overlap": (f"bucketed reduce/apply/broadcast during backward ({len(run.chan.buckets)} buckets)"
                            if getattr(run.chan, "overlap", False) else
                            f"bucketed reduce/apply/broadcast captured in the step graph ({len(run.chan.buckets)} buckets)"
                            if getattr(run.chan, "in_graph", False) else "none"),
                "topology": run.topology_name(),
                "workers": W,
                "transport": (("native RCCL (psx comm)" if getattr(t, "native", False) else "torch.distributed")
                              if t is not None else "in-process"),
                "rccl_ranks": t.comm.count() if getattr(t, "native", False) else None,
                "pair_communicators": len(getattr(t, "_pairs", {}) or {}) if t is not None else 0,
                "hip_graph": cfg.use_graph,
                # exact fixed-point BN statistics (bit-reproducible steps), the engine's default
                "deterministic": (cfg.deterministic if cfg.deterministic is not None
                                  else os.environ.get("PSX_DETERMINISTIC", "1") == "1"),
            },
            "value_per_worker": round(value / W, 2),
            "global_steps": run.server.core.global_step,
            "last_loss": round(loss, 4) if loss is not None else None,
            "baseline_img_s": BASELINE_SYNC_IMG_S if r18 else None,
        }
    if rank == 0 and run.server_round_us is not None:
        # dedicated server: device time per round per phase (bucket phases overlap with --overlap)
        rec["server_round_us"] = run.server_round_us
    if a.host_timing and host:
        wait = getattr(run.wk.compute, "host_wait_s", 0.0) if run.wk is not None else 0.0
        print(json.dumps({"rank": rank, "host_issue_ms_per_step": round(1e3 * sum(host) / len(host), 4),
                          "host_issue_ms_max": round(1e3 * max(host), 4),
                          # time the host spent blocked because it ran len(ring) steps ahead (whole run)
                          "host_wait_ms_total": round(1e3 * wait, 3)}), file=sys.stderr, flush=True)
    run.close()
    if rank == 0 and a.mode == "async":
        sm = run.server.final_metrics()
        # average / max_staleness_observed follow the reference (each worker's LAST push,
        # server.py:300); the histogram and mean_staleness_all cover every push of the run
        rec["async_staleness"] = {k: sm.get(k) for k in ("average_gradient_staleness", "max_staleness_observed",
                                                         "mean_staleness_all", "async_updates", "rejected_pushes",
                                                         "staleness_histogram")}
        hist = sm.get("staleness_histogram") or []
        rec["async_staleness"]["max_staleness_accepted"] = max((i for i, n in enumerate(hist) if n), default=0)
        rec["global_steps"] = run.server.core.global_step

    # secondary numbers (same transport): bf16 compute at N=1, the co-located topology at N>=2
    secondary = {}
    if a.secondary == "auto" and a.mode == "sync" and r18 and topology != "sharded":
        # (name, compute dtype, topology, overrides): N = 1 — the bf16 compute path and the async
        # PS (one worker, in-process: the staleness summary of BASELINE's "async staleness"); N >= 2
        # — the co-located topology and the serial (overlap off) round, a same-box A/B of the
        # bucketed overlap the headline turns on automatically
        if world == 1:
            cases = [("bf16_compute", "bf16", topology, {}), ("async_ps", a.dtype, topology, {"mode": "async"})]
        else:
            cases = ([("colocated_topology", a.dtype, "colocated", {})] if topology == "dedicated" else [])
            cases.append(("overlap_off", a.dtype, topology, {"overlap": "off"}))
        for name, dt_, topo, over in cases:
            try:
                a2 = argparse.Namespace(**vars(a))
                a2.fetch_codec = "fp32" if dt_ == "fp32" else "bf16conv"
                for k, v in over.items():
                    setattr(a2, k, v)
                t2 = None if (a2.mode == "async" and world == 1) else t  # async N=1: in-process loopback
                r2 = Run(a2, t2, rank, world, device, dt_, topo)
                steps2 = max(5, min(a.steps, 20))
                d2, _ = r2.measure(steps2, min(a.warmup, 5))
                v2 = steps2 * a.batch * r2.W / d2
                secondary[name] = {"value": round(v2, 2), "ms_per_step": round(1e3 * d2 / steps2, 4), "dtype": dt_,
                                   "topology": r2.topology_name(), "workers": r2.W, "steps": steps2,
                                   "vs_baseline": round(v2 / BASELINE_SYNC_IMG_S, 2)}
                if over:
                    secondary[name]["overrides"] = over
                if a2.mode == "async" and r2.server is not None:
                    sm = r2.server.final_metrics()
                    secondary[name]["async_staleness"] = {
                        k: sm.get(k) for k in ("average_gradient_staleness", "max_staleness_observed",
                                               "mean_staleness_all", "async_updates", "rejected_pushes",
                                               "staleness_histogram")}
                r2.close()
            except Exception as e:  # noqa: BLE001 - a secondary number never costs the headline
                secondary[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if world == 1:
            secondary["async_w7"] = async_threads(a, 7)
    if rank == 0:
        if secondary:
            rec["secondary"] = secondary
        if rccl_log is not None:
            rec["config"]["rccl_algorithms"] = rccl_choices(rccl_log)
        print(json.dumps(rec), flush=True)
    if t is not None:
        t.close()


if __name__ == "__main__":
    main()
