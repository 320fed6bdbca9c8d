#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node) of ResNet-18 / CIFAR-100-shaped data in the
synchronous parameter-server mode on 1..8 MI355X (BASELINE.json metric).

  python bench.py                                   # N=1: server + worker co-located (one RCCL rank)
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
      --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

One step = fetch (RCCL broadcast from rank 0 of the weight wire: the bf16 image of the
parameters + the fp32 BN/FC remainder, 22.5 MB) -> batch gather + augment -> forward/backward on
the HIP engine (hand-written CDNA4 kernels, HIP graphs) -> push (RCCL reduce of the fp16 wire
gradients to rank 0) -> fused SGD apply of the average on rank 0 (writing the next image). Batch 128 per worker, lr 0.1, sync period 1 (the reference's CLI defaults). Weak
scaling: every rank is a worker (rank 0 also hosts the parameter server, ``--topology
colocated``); ``--topology dedicated`` reproduces the reference's 1 server + (N-1) workers.
W warmup steps are untimed; exactly K steps are timed between barrier+synchronize pairs and
the max over ranks is reported. Data is synthetic CIFAR-100-shaped (no network access), weights
random-init.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel.compute import HipCompute  # noqa: E402
from psx.parallel.runner import (AsyncSession, build_state, make_datasets, make_local_channel,  # noqa: E402
                                 make_sync_channel)
from psx.parallel.server import ParameterServer  # noqa: E402
from psx.parallel.sharded import ShardedSyncChannel  # noqa: E402
from psx.parallel.rccl import make_transport  # noqa: E402
from psx.parallel.transport import env_world  # noqa: E402
from psx.parallel.worker import Worker  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402

BASELINE_SYNC_IMG_S = 82.7  # sync PS, 4 workers, measured (experiment_results/sync_4workers.json)


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
    ap.add_argument("--topology", choices=["colocated", "dedicated", "sharded"], default="colocated",
                    help="sharded: every rank is a worker and owns 1/N of the server (reduce-scatter, "
                         "range apply, all-gather; parallel/sharded.py)")
    ap.add_argument("--codec", choices=["fp16", "none", "topk"], default="fp16")
    ap.add_argument("--topk-ratio", type=float, default=0.01)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="worker compute precision. fp32 (default, the headline): the reference's training "
                         "precision (worker.py:333-348), every conv product on the exact-f32 MFMA; bf16: bf16 "
                         "operands with fp32 accumulation and fp32 master weights (secondary number)")
    ap.add_argument("--fetch-codec", choices=["auto", "bf16conv", "fp32"], default="auto",
                    help="auto: fp32 for --dtype fp32, bf16conv for bf16. bf16conv: conv weights travel as the "
                         "bf16 bits the workers compute with, everything else fp32; fp32: the reference's full "
                         "fp32 state")
    ap.add_argument("--overlap", action="store_true",
                    help="stream gradient buckets (reduce/apply/broadcast) during the backward pass")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--host-timing", action="store_true", help="report host-side issue time per step (stderr)")
    ap.add_argument("--mode", choices=["sync", "async"], default="sync",
                    help="async: workers push/fetch independently (staleness-weighted server updates)")
    ap.add_argument("--staleness-bound", type=int, default=5)
    a = ap.parse_args()

    rank, world, local = env_world()
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs MI355X GPUs")
    torch.cuda.set_device(local % torch.cuda.device_count())
    device = torch.device("cuda", torch.cuda.current_device())
    n_train = a.train_samples or (50000 if a.model == "resnet18" else 4096)
    cfg = PSConfig(mode=a.mode, staleness_bound=a.staleness_bound, model=a.model, batch_size=a.batch, train_samples=n_train, lr=0.1, sync_steps=1, epochs=1,
                   eval_every=0, verbose=0, codec=a.codec, topk_ratio=a.topk_ratio, use_graph=not a.no_graph, fetch_codec=a.fetch_codec,
                   overlap=a.overlap, bucket_mb=a.bucket_mb, topology=a.topology, dtype=a.dtype).validate()
    model, layout, arena, counters = build_state(cfg)
    wire = torch.float16 if a.codec == "fp16" else torch.float32  # topk encodes from fp32 grads

    t = None
    # sync at N = 1 runs the distributed path too (one rank: psx communicator, rank 0 = server +
    # worker 0), the same code as N > 1; measured equal to or faster than the in-process loopback
    # (one box 1.777/1.778 vs 1.842/1.829 ms/step, another 1.843 vs 1.853 mean of 3 interleaved).
    # PSX_FORCE_DIST=0: in-process loopback.
    force_dist = os.environ.get("PSX_FORCE_DIST", "1" if a.mode == "sync" else "0") == "1"
    sharded = a.topology == "sharded"
    if world > 1 or force_dist or sharded:
        if "RANK" not in os.environ:  # single process without torchrun: a world of one rank
            import socket

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(port))
        t = make_transport(device)
    dedicated = a.topology == "dedicated" and world > 1
    worker_ranks = list(range(1, world)) if dedicated else list(range(world))
    W = len(worker_ranks)
    cfg.workers = W
    is_worker = rank in worker_ranks
    server = None
    quiet = lambda *x, **k: None  # noqa: E731
    async_dist = a.mode == "async" and t is not None
    if rank == 0 or sharded:
        server = ParameterServer(cfg, layout, arena, counters, device=device, total_workers=W, log=quiet)
        if not async_dist and rank == 0:
            for i in range(W):
                server.register_worker(f"worker-{i}", i)
    train, _ = make_datasets(cfg, device, model.fc.out_features)
    comp = HipCompute(model, layout, a.batch, device, a.model, wire, seed=rank, use_graph=cfg.use_graph,
                      dtype=cfg.dtype) if is_worker else None
    wk = None
    zeros = None
    sess = None
    chan = None
    if async_dist:  # server event loop thread on rank 0, mailbox + RCCL p2p (parallel/runner.py)
        names = [f"worker-r{r}" for r in range(world)]
        sess = AsyncSession(cfg, t, rank, worker_ranks, server, comp, train, None, names, quiet)
        wk = sess.worker
    else:
        if sharded:
            chan = ShardedSyncChannel(cfg, t, server, list(range(W)), layout, device, in_place=True)
        else:
            chan = (make_local_channel(cfg, server, layout, device) if t is None else
                    make_sync_channel(cfg, t, server, W, layout, device, worker=is_worker))
        if is_worker:
            wid = worker_ranks.index(rank)
            wk = Worker(cfg, comp, chan, train, None, worker_name=f"worker-{wid}", rank=rank, log=quiet,
                        requested_id=wid)
            wk.connect_to_server()
    if wk is not None:
        wk.setup_data()
        batches = wk.sampler.epoch_indices(0)
    elif sess is not None:
        pass  # dedicated async server rank: its event-loop thread does the work
    elif a.codec == "topk":
        from psx.parallel.topk import empty_payload

        zeros = empty_payload(layout.param_numel, a.topk_ratio, device)
    else:
        zeros = torch.zeros(layout.param_numel, dtype=wire, device=device)

    def step(i):
        if wk is not None:
            wk.fetch_parameters()
            wk.train_local_batch(batches[i % len(batches)])
            wk.push_gradients()
        elif sess is not None:
            pass
        else:  # dedicated sync server rank
            chan.fetch(None, None)
            if a.codec != "topk":
                zeros.zero_()
            chan.push(None, zeros, server.core.global_step)

    def barrier_sync():
        torch.cuda.synchronize()
        if t is not None:
            # async: the server thread drives RCCL p2p on the default group, so host barriers
            # use the gloo control group
            t.barrier() if async_dist else dist.barrier()
        torch.cuda.synchronize()

    for i in range(a.warmup):
        step(i)
    barrier_sync()
    host = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        h0 = time.perf_counter()
        step(a.warmup + i)
        host.append(time.perf_counter() - h0)
    barrier_sync()
    dt = time.perf_counter() - t0
    if t is not None and async_dist:
        dt = max(t.all_gather_object(dt))
    elif t is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    imgs = a.steps * a.batch * W
    value = imgs / dt
    loss = wk.compute.last_loss() if wk is not None else None
    if rank == 0:
        r18 = a.model == "resnet18"
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
            "data": (f"synthetic CIFAR-100-shaped ({n_train}x32x32x3 uint8 in HBM, on-device crop/flip/normalize), "
                     "random-init weights" if r18 else
                     f"synthetic ImageNet-shaped ({n_train}x224x224x3 uint8 in HBM, on-device crop/flip/normalize), "
                     "random-init weights"),
            "config": {
                "model": ("resnet18-cifar (11,220,132 params, reference ResNet18(num_classes=100))" if r18 else
                          f"resnet50-imagenet ({layout.param_numel:,} params, 1000 classes)"),
                "global_batch": a.batch * W,
                "per_worker_batch": a.batch,
                "seq_len": None,
                "parallelism": (
                    f"sharded sync-PS: {W} ranks, each a worker + 1/{W} of the server; RCCL reduce-scatter(grads) "
                    f"+ all-gather(bf16 params) over xGMI" if sharded else
                    f"{a.mode}-PS: rank0 = parameter server{' only' if dedicated else ' + worker 0'}, {W} data-parallel "
                    f"worker(s); " + ("RCCL reduce(grads) + broadcast(params) over xGMI" if a.mode == "sync" else
                                      "shm mailbox control + RCCL send/recv over xGMI")
                    if t is not None else f"{a.mode}-PS: server + 1 worker co-located on 1 GPU"),
                "mode": a.mode,
                "lr": 0.1,
                "sync_steps": 1,
                "codec": a.codec if a.codec != "topk" else f"topk({a.topk_ratio}) + error feedback",
                "fetch_codec": cfg.fetch_codec if t is not None else "in-process",
                "weight_image": getattr(chan, "image_wire", None) is not None or sharded,
                "overlap": (f"bucketed reduce/apply/broadcast during backward ({len(chan.buckets)} buckets)"
                            if getattr(chan, "overlap", False) else
                            f"bucketed reduce/apply/broadcast captured in the step graph ({len(chan.buckets)} buckets)"
                            if getattr(chan, "in_graph", False) else "none"),
                "topology": ("sharded" if sharded else "dedicated" if dedicated else
                             ("colocated" if t is not None else "loopback")),
                "transport": (("native RCCL (psx comm)" if getattr(t, "native", False) else "torch.distributed")
                              if t is not None else "in-process"),
                "hip_graph": cfg.use_graph,
            },
            "global_steps": server.core.global_step,
            "last_loss": round(loss, 4) if loss is not None else None,
            "baseline_img_s": BASELINE_SYNC_IMG_S if r18 else None,
        }
    if a.host_timing:
        wait = getattr(wk.compute, "host_wait_s", 0.0) if wk is not None else 0.0
        print(json.dumps({"rank": rank, "host_issue_ms_per_step": round(1e3 * sum(host) / len(host), 4),
                          "host_issue_ms_max": round(1e3 * max(host), 4),
                          # time the host spent blocked because it ran len(ring) steps ahead (whole run)
                          "host_wait_ms_total": round(1e3 * wait, 3)}), file=sys.stderr, flush=True)
    if sess is not None:
        sess.finish()
        sess.close()
    if rank == 0:
        if a.mode == "async":
            sm = server.final_metrics()
            rec["async_staleness"] = {k: sm.get(k) for k in ("average_gradient_staleness", "max_staleness_observed",
                                                             "rejected_pushes", "staleness_histogram")}
            rec["global_steps"] = server.core.global_step
        print(json.dumps(rec), flush=True)
    if hasattr(chan, "drain"):
        chan.drain()
    if t is not None:
        t.close()


if __name__ == "__main__":
    main()
