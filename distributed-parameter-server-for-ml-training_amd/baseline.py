"""Single-process baseline trainer (no parameter server) — the reference's
baseline/baseline_training.py (C32) and its summary generator (C33), MI355X-native.

Same recipe as the reference (baseline/baseline_training.py:201-269): ResNet-18 / CIFAR-100,
batch 128, 3 epochs, SGD(lr 0.1, momentum 0.9, weight decay 5e-4) stepped every batch,
MultiStepLR(milestones [10, 15], gamma 0.1) stepped every epoch, train loss/accuracy per epoch,
test accuracy after every epoch, a 2x2 results figure and a results summary.

The step runs on the HIP engine (models/engine.py, one HIP graph per step) and the optimizer
is the fused SGD-momentum kernel (csrc/kernels/optim.hip) applied in place to the fp32 master
arena the engine reads its weights from — no host sync inside an epoch: per-step loss/accuracy
are accumulated on the device and read once per epoch. On a CPU-only host the torch path
(parallel/compute.py TorchCompute) runs the same loop for tests.
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

from .models.layout import ParamLayout
from .models.resnet import MODEL_INPUT, build_model
from .parallel.compute import make_compute
from .utils import metrics as M
from .utils.data import DeviceDataset, EpochSampler


class TrainingMetrics:
    """Per-epoch history + the reference's 2x2 figure (baseline_training.py:97-147)."""

    def __init__(self):
        self.train_losses, self.train_accuracies, self.test_accuracies, self.epoch_times = [], [], [], []
        self.total_time = 0.0

    def add_epoch(self, train_loss, train_acc, test_acc, epoch_time):
        self.train_losses.append(train_loss)
        self.train_accuracies.append(train_acc)
        self.test_accuracies.append(test_acc)
        self.epoch_times.append(epoch_time)
        self.total_time += epoch_time

    def plot_results(self, path: str):
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        fig, ((a1, a2), (a3, a4)) = plt.subplots(2, 2, figsize=(12, 8))
        a1.plot(self.train_losses)
        a1.set(title="Training Loss", xlabel="Epoch", ylabel="Loss")
        a2.plot(self.train_accuracies, label="Train")
        a2.plot(self.test_accuracies, label="Test")
        a2.set(title="Accuracy", xlabel="Epoch", ylabel="Accuracy (%)")
        a2.legend()
        a3.plot(self.epoch_times)
        a3.set(title="Time per Epoch", xlabel="Epoch", ylabel="Time (seconds)")
        avg = sum(self.epoch_times) / max(1, len(self.epoch_times))
        for y, txt in zip((0.8, 0.6, 0.4, 0.2), (f"Final Test Accuracy: {self.test_accuracies[-1]:.2f}%",
                                                 f"Total Training Time: {self.total_time / 60:.1f} minutes",
                                                 f"Avg Time/Epoch: {avg:.1f} seconds",
                                                 f"Epochs Completed: {len(self.epoch_times)}")):
            a4.text(0.1, y, txt, transform=a4.transAxes, fontsize=12)
        a4.set_title("Training Summary")
        a4.axis("off")
        fig.tight_layout()
        fig.savefig(path, dpi=150, bbox_inches="tight")
        plt.close(fig)


class MultiStepLR:
    def __init__(self, lr, milestones=(10, 15), gamma=0.1):
        self.base, self.milestones, self.gamma = lr, sorted(milestones), gamma
        self.epoch = 0

    @property
    def lr(self):
        return self.base * self.gamma ** sum(1 for m in self.milestones if m <= self.epoch)

    def step(self):
        self.epoch += 1


class BaselineTrainer:
    def __init__(self, model_name="resnet18", batch=128, lr=0.1, momentum=0.9, weight_decay=5e-4,
                 milestones=(10, 15), gamma=0.1, device=None, seed=0, use_graph=True, log=print):
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.model_name = model_name
        self.model = build_model(model_name, seed=seed)
        self.layout = ParamLayout.from_module(self.model)
        arena, _ = self.layout.pack(self.model)
        self.compute = make_compute(self.model, self.layout, batch, self.device, model_name, torch.float32, seed=seed,
                                    use_graph=use_graph)
        self.compute.local_arena.copy_(arena.to(self.device))
        self.n = self.layout.param_numel
        self.params = self.compute.local_arena[: self.n]
        self.mom = torch.zeros_like(self.params)
        self.momentum, self.wd = momentum, weight_decay
        self.sched = MultiStepLR(lr, milestones, gamma)
        self.B = batch
        self.seed = seed
        self.log = log
        self._first = True
        self.metrics = TrainingMetrics()

    def _sgd_step(self):
        """optimizer.step(): torch SGD(momentum, weight_decay) on the whole parameter prefix."""
        g = self.compute.grads[: self.n]
        lr = self.sched.lr
        if self.device.type == "cuda":
            from .ops import kernels as K

            K.sgd_apply(self.params, g, lr, momentum=self.momentum, wd=self.wd, buf=self.mom, first=self._first,
                        n=self.n)
        else:
            d = g.float() + self.wd * self.params
            if self._first:
                self.mom.copy_(d)
            else:
                self.mom.mul_(self.momentum).add_(d)
            self.params.sub_(lr * self.mom)
        self._first = False

    def train_epoch(self, train_set, epoch, t_start):
        sampler = EpochSampler(0, len(train_set), self.B, seed=self.seed)
        batches = sampler.epoch_indices(epoch)
        loss_acc = torch.zeros((), dtype=torch.float64, device=self.device)
        corr_acc = torch.zeros((), dtype=torch.int64, device=self.device)
        t_ep = time.time()
        for bi, idx in enumerate(batches):
            self.compute.train_step(train_set, idx)
            self._sgd_step()
            ls, cs = self.compute.step_stats()
            loss_acc += ls.to(self.device)
            corr_acc += cs.to(self.device)
            if bi % 10 == 0 and self.device.type == "cpu":  # progress (reference prints every 10 batches)
                self.log(f"Batch {bi}/{len(batches)}, Loss: {self.compute.last_loss():.4f}, "
                         f"Elapsed: {(time.time() - t_ep) / 60:.1f}min this epoch, "
                         f"{(time.time() - t_start) / 60:.1f}min total")
        seen = len(batches) * self.B
        return float(loss_acc) / seen, 100.0 * float(corr_acc) / seen

    def fit(self, train_set, test_set, epochs=3):
        t0 = time.time()
        for ep in range(epochs):
            self.log(f"\nEpoch {ep + 1}/{epochs}")
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            te = time.time()
            tr_loss, tr_acc = self.train_epoch(train_set, ep, t0)
            test_acc = self.compute.evaluate(test_set) if test_set is not None else 0.0
            self.sched.step()
            dt = time.time() - te
            self.metrics.add_epoch(tr_loss, tr_acc, test_acc, dt)
            self.log(f"Epoch {ep + 1} completed in {dt:.1f}s (Total elapsed: {(time.time() - t0) / 60:.1f}min)")
            self.log(f"Train Loss: {tr_loss:.4f}, Train Acc: {tr_acc:.2f}%, Test Acc: {test_acc:.2f}%")
        return self.metrics


def write_summary(results: dict, out_dir: str):
    """Summary generator (reference baseline/results/generate_summary.py, which writes a
    hard-coded epoch-1 result) — here computed from the run that just finished."""
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "baseline_summary.json"), "w") as f:
        json.dump(results, f, indent=2)
    with open(os.path.join(out_dir, "baseline_summary.txt"), "w") as f:
        f.write("Baseline Results Summary\n========================\n")
        for k, v in results.items():
            f.write(f"{k}: {v}\n")


def main(argv=None):
    ap = argparse.ArgumentParser(description="single-process baseline trainer (no parameter server)")
    ap.add_argument("--model", default="resnet18", choices=["resnet18", "resnet50", "resnet_tiny"])
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--weight-decay", type=float, default=5e-4)
    ap.add_argument("--milestones", default="10,15")
    ap.add_argument("--train-samples", type=int, default=50000)
    ap.add_argument("--test-samples", type=int, default=10000)
    ap.add_argument("--data-dir", default="", help="directory with CIFAR-100 binary train.bin/test.bin")
    ap.add_argument("--out-dir", default="baseline_results")
    ap.add_argument("--no-plot", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    dev = torch.device("cpu" if a.cpu or not torch.cuda.is_available() else "cuda")
    print(f"Using device: {dev}")
    tr = BaselineTrainer(a.model, a.batch_size, a.lr, a.momentum, a.weight_decay,
                         tuple(int(m) for m in a.milestones.split(",") if m), device=dev, seed=a.seed,
                         use_graph=not a.no_graph)
    (_, h, _), classes = MODEL_INPUT[a.model]
    if a.data_dir:
        train = DeviceDataset.cifar_binary(os.path.join(a.data_dir, "train.bin"), a.train_samples, device=dev)
        test = DeviceDataset.cifar_binary(os.path.join(a.data_dir, "test.bin"), a.test_samples, device=dev)
    else:
        train = DeviceDataset.synthetic(a.train_samples, h, classes, seed=a.seed, device=dev)
        test = DeviceDataset.synthetic(a.test_samples, h, classes, seed=a.seed, device=dev, offset=10_000_000)
    print(f"Dataset loaded - Train: {len(train)} samples, Test: {len(test)} samples")
    print(f"Model has {tr.n:,} parameters")
    print("\nStarting baseline training...")
    m = tr.fit(train, test, a.epochs)
    print("\nBaseline training completed!")
    print(f"Total time: {m.total_time / 60:.1f} minutes")
    print(f"Final test accuracy: {m.test_accuracies[-1]:.2f}%")
    os.makedirs(a.out_dir, exist_ok=True)
    if not a.no_plot:
        m.plot_results(os.path.join(a.out_dir, "baseline_results.png"))
    steps = a.epochs * (len(train) // a.batch_size + (len(train) % a.batch_size > 0))
    results = {
        "final_accuracy": m.test_accuracies[-1],
        "total_time_minutes": m.total_time / 60,
        "avg_epoch_time": float(np.mean(m.epoch_times)),
        "model_parameters": tr.n,
        "batch_size": a.batch_size,
        "epochs": a.epochs,
        # psx extensions
        "images_per_second": round(steps * a.batch_size / max(1e-9, sum(m.epoch_times)), 2),
        "train_losses": m.train_losses,
        "train_accuracies": m.train_accuracies,
        "test_accuracies": m.test_accuracies,
        "device": str(dev),
        "data": "cifar-100 binary" if a.data_dir else "synthetic CIFAR-100-shaped",
    }
    print("\nBaseline Results Summary:")
    for k in ("final_accuracy", "total_time_minutes", "avg_epoch_time", "model_parameters", "batch_size", "epochs"):
        print(f"{k}: {results[k]}")
    write_summary(results, a.out_dir)
    M.emit(dict(type="BASELINE_FINAL_METRICS", **{k: v for k, v in results.items()}))
    return results


if __name__ == "__main__":
    main()
