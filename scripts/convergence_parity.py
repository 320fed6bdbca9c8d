#!/usr/bin/env python3
"""Convergence parity: psx against a torch fp32 autograd run of the same network on one MI355X.

* ``torch_fp32``      models/resnet.py ResNet18 in plain PyTorch (MIOpen convolutions, fp32, no
                      TF32), SGD p -= lr * g applied by hand — the reference's single-process
                      trainer without momentum (reference baseline/baseline_training.py:149-199;
                      the PS server applies plain SGD, server.py:126-143).
* ``torch_fp32_init1`` the same with another weight initialisation: the natural run-to-run spread
                      that any precision difference has to be judged against.
* ``psx_fp32``        the psx parameter server, W = 1 sync loopback (Worker -> InProcessChannel ->
                      ParameterServer), fp32 HIP engine, fp16 gradient wire (the reference codec).
* ``psx_fp32_wire32`` the same with the fp32 wire (--codec none).
* ``psx_bf16``        the bf16 HIP engine (fast path), fp16 wire, bf16conv fetch.
* ``psx_fp32_reference_bn`` psx_fp32 with the reference's BN semantics (no --bn-sync): same
                      training curve, but the evaluation runs on never-learned running statistics.

The psx runs other than the last push their BN running statistics with the gradient (--bn-sync;
with W = 1 the server then holds the worker's statistics, as a single-process trainer does).

All runs start from the same weights (except ``torch_fp32_init1``), see the same batches in the
same order and the same augmented pixels (the torch runs call the psx augmentation kernel with
the engine's seed and step), on class-conditional noise with 20% label noise
(utils/data.py synthetic_hard), so accuracy sits well below 100%. A second part runs the
W = 4 sync loopback with the reference's BN semantics (the server never learns running
statistics, every fetch overwrites the workers' copies) and with --bn-sync.

Writes ``<out>/convergence_parity.json`` and ``<out>/convergence_parity.png``.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import psx  # noqa: E402,F401
from psx.models.engine import CIFAR_MEAN, CIFAR_STD  # noqa: E402
from psx.ops import kernels as K  # noqa: E402
from psx.parallel.compute import make_compute  # noqa: E402
from psx.parallel.runner import _wire_dtype, build_state, make_local_channel, run_local  # noqa: E402
from psx.parallel.server import ParameterServer  # noqa: E402
from psx.parallel.worker import Worker  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402
from psx.utils.data import DeviceDataset, EpochSampler  # noqa: E402

DEV = torch.device("cuda", 0)
ENGINE_SEED = 1234  # HipCompute(seed=0) -> engine augmentation seed


def _noop(*a, **k):
    pass


def batches_for(args):
    """The worker's epoch order (utils/data.py EpochSampler, worker 0 of 1), flattened to steps."""
    sampler = EpochSampler(0, args.train, args.batch, seed=0)
    out = []
    ep = 0
    while len(out) < args.steps:
        out.extend(list(sampler.epoch_indices(ep)))
        ep += 1
    return out[: args.steps]


def run_psx(args, train, test, dtype: str, codec: str, bn_sync: bool = True):
    """bn_sync: the worker pushes its BN running statistics with the gradient (W = 1: the server
    keeps the worker's, as a single-process trainer does); without it the reference semantics
    apply (every fetch resets them to the server's never-updated copy)."""
    cfg = PSConfig(model="resnet18", mode="sync", workers=1, lr=args.lr, batch_size=args.batch, epochs=10 ** 6,
                   train_samples=args.train, eval_every=0, verbose=0, dtype=dtype, codec=codec,
                   bn_sync=bn_sync).validate()
    model, lay, arena, counters = build_state(cfg)
    srv = ParameterServer(cfg, lay, arena.clone(), counters, device=DEV, total_workers=1, log=_noop)
    comp = make_compute(model, lay, args.batch, DEV, "resnet18", _wire_dtype(cfg), seed=0, use_graph=True,
                        dtype=dtype)
    wk = Worker(cfg, comp, make_local_channel(cfg, srv, lay, DEV), train, test, worker_name="w0", rank=0, log=_noop,
                requested_id=0)
    wk.connect_to_server()
    wk.setup_data()
    loss = torch.zeros(args.steps, dtype=torch.float64, device=DEV)
    corr = torch.zeros(args.steps, dtype=torch.int64, device=DEV)
    t0 = time.time()
    step, ep = 0, 0
    while step < args.steps:
        batches = wk.sampler.epoch_indices(ep)
        for b, idx in enumerate(batches):
            if step >= args.steps:
                break
            wk.fetch_parameters()
            wk.train_local_batch(idx)
            wk.window_push(b, len(batches), 1)
            ls, c = comp.step_stats()
            loss[step] = ls / args.batch
            corr[step] = c
            step += 1
        ep += 1
    wk.fetch_parameters()
    torch.cuda.synchronize()
    dt = time.time() - t0
    acc = comp.evaluate(test)
    return {"loss": loss.cpu().tolist(), "train_acc": (corr.double() / args.batch * 100).cpu().tolist(),
            "test_acc": acc, "seconds": dt, "global_steps": srv.core.global_step}


def run_torch(args, train, test, init_seed: int):
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    cfg = PSConfig(model="resnet18", seed=init_seed).validate()
    model, _, _, _ = build_state(cfg)
    net = copy.deepcopy(model).to(DEV).float().train()
    B = args.batch
    x0 = torch.zeros(B, 32, 32, 4, dtype=torch.float32, device=DEV)
    lab = torch.zeros(B, dtype=torch.int32, device=DEV)
    loss_h = torch.zeros(args.steps, dtype=torch.float64, device=DEV)
    corr_h = torch.zeros(args.steps, dtype=torch.int64, device=DEV)
    t0 = time.time()
    for step, idx in enumerate(batches_for(args)):
        meta = torch.tensor(list(idx) + [step], dtype=torch.int32).to(DEV)
        K.augment(train.images, train.labels, meta[:B], x0, lab, B, 32, 32, 4, ENGINE_SEED, meta[B:], True,
                  CIFAR_MEAN, CIFAR_STD)
        x = x0[..., :3].permute(0, 3, 1, 2).contiguous()
        out = net(x)
        loss = F.cross_entropy(out, lab.long())
        net.zero_grad(set_to_none=False)
        loss.backward()
        with torch.no_grad():
            for p in net.parameters():
                p.sub_(p.grad, alpha=args.lr)
            loss_h[step] = loss.double()
            corr_h[step] = (out.argmax(1) == lab.long()).sum()
    torch.cuda.synchronize()
    dt = time.time() - t0
    net.eval()
    correct = 0
    n = len(test)
    with torch.no_grad():
        for s in range(0, n, B):
            idx = (np.arange(s, s + B) % n).tolist()
            meta = torch.tensor(idx + [0], dtype=torch.int32).to(DEV)
            K.augment(test.images, test.labels, meta[:B], x0, lab, B, 32, 32, 4, ENGINE_SEED, meta[B:], False,
                      CIFAR_MEAN, CIFAR_STD)
            pred = net(x0[..., :3].permute(0, 3, 1, 2).contiguous()).argmax(1)
            v = min(B, n - s)
            correct += int((pred[:v] == lab[:v].long()).sum())
    return {"loss": loss_h.cpu().tolist(), "train_acc": (corr_h.double() / B * 100).cpu().tolist(),
            "test_acc": 100.0 * correct / n, "seconds": dt, "global_steps": args.steps}


def run_w4(args, bn_sync: bool):
    """W = 4 sync loopback on the same data (each worker one quarter), reference BN semantics
    (bn_sync False) or --bn-sync; test accuracy of every worker after the last epoch."""
    spw = args.train // 4
    steps_ep = -(-spw // args.batch)
    epochs = max(1, args.steps // steps_ep)
    cfg = PSConfig(model="resnet18", mode="sync", workers=4, lr=args.lr, batch_size=args.batch, epochs=epochs,
                   train_samples=args.train, test_samples=args.test, eval_every=epochs, verbose=0,
                   synthetic_kind="hard", bn_sync=bn_sync).validate()
    import contextlib
    import io

    with contextlib.redirect_stdout(io.StringIO()):  # METRICS_JSON lines of the loopback run
        res = run_local(cfg, log=_noop)
    accs = [w["all_accuracies_percent"][-1] for w in res["workers"]]
    return {"global_steps": res["server"]["global_steps_completed"], "epochs": epochs,
            "worker_test_acc": accs, "last_loss": [w["last_loss"] for w in res["workers"]]}


def smooth(x, w):
    x = np.asarray(x, dtype=np.float64)
    if len(x) < w:
        return x
    c = np.cumsum(np.insert(x, 0, 0.0))
    return (c[w:] - c[:-w]) / w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--train", type=int, default=10000)
    ap.add_argument("--test", type=int, default=2000)
    ap.add_argument("--window", type=int, default=25, help="moving-average window of the compared curves")
    ap.add_argument("--out", default="gpurun_out/convergence")
    ap.add_argument("--skip-w4", action="store_true")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    train = DeviceDataset.synthetic_hard(args.train, device=DEV)
    test = DeviceDataset.synthetic_hard(args.test, device=DEV, offset=10_000_000)
    runs = {}
    for name, fn in (("torch_fp32", lambda: run_torch(args, train, test, 0)),
                     ("torch_fp32_init1", lambda: run_torch(args, train, test, 1)),
                     ("psx_fp32", lambda: run_psx(args, train, test, "fp32", "fp16")),
                     ("psx_fp32_wire32", lambda: run_psx(args, train, test, "fp32", "none")),
                     ("psx_bf16", lambda: run_psx(args, train, test, "bf16", "fp16")),
                     ("psx_fp32_reference_bn", lambda: run_psx(args, train, test, "fp32", "fp16", bn_sync=False))):
        runs[name] = fn()
        r = runs[name]
        print(f"{name:18s} last-100 loss {np.mean(r['loss'][-100:]):.4f} test acc {r['test_acc']:.2f}% "
              f"({r['seconds']:.1f} s)", flush=True)
    ref = smooth(runs["torch_fp32"]["loss"], args.window)
    cmp = {}
    for name, r in runs.items():
        if name == "torch_fp32":
            continue
        s = smooth(r["loss"], args.window)
        cmp[name] = {"max_abs_smoothed_loss_diff": float(np.max(np.abs(s - ref))),
                     "mean_abs_smoothed_loss_diff": float(np.mean(np.abs(s - ref))),
                     "last100_loss_diff": float(np.mean(r["loss"][-100:]) - np.mean(runs["torch_fp32"]["loss"][-100:])),
                     "test_acc_diff_pp": r["test_acc"] - runs["torch_fp32"]["test_acc"]}
        print(f"  vs torch_fp32: {name:18s} {json.dumps(cmp[name])}", flush=True)
    w4 = {}
    if not args.skip_w4:
        for bn in (False, True):
            key = "bn_sync" if bn else "reference_bn_semantics"
            w4[key] = run_w4(args, bn)
            print(f"W=4 {key}: {json.dumps(w4[key])}", flush=True)
    out = {"config": vars(args), "data": "synthetic_hard: 4x4 class prototypes (std 12) + pixel noise (std 64), "
                                          "20% label noise, 100 classes",
           "runs": runs, "vs_torch_fp32": cmp, "w4_sync": w4}
    with open(os.path.join(args.out, "convergence_parity.json"), "w") as f:
        json.dump(out, f)
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        fig, ax = plt.subplots(1, 2, figsize=(12, 4.5))
        for name, r in runs.items():
            s = smooth(r["loss"], args.window)
            ax[0].plot(np.arange(len(s)) + args.window, s, label=name, lw=1.2)
            a = smooth(r["train_acc"], args.window)
            ax[1].plot(np.arange(len(a)) + args.window, a, label=f"{name} (test {r['test_acc']:.1f}%)", lw=1.2)
        ax[0].set_xlabel("step")
        ax[0].set_ylabel(f"train loss ({args.window}-step mean)")
        ax[1].set_xlabel("step")
        ax[1].set_ylabel(f"train accuracy % ({args.window}-step mean)")
        for a in ax:
            a.grid(alpha=0.3)
            a.legend(fontsize=8)
        fig.suptitle(f"ResNet-18, synthetic_hard (20% label noise), batch {args.batch}, lr {args.lr:g}, MI355X")
        fig.tight_layout()
        fig.savefig(os.path.join(args.out, "convergence_parity.png"), dpi=110)
    except Exception as e:  # noqa: BLE001 - the JSON is the artifact; the figure is a convenience
        print(f"plot skipped: {e}")


if __name__ == "__main__":
    main()
