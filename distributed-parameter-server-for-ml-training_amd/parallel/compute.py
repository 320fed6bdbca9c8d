"""Worker compute backends: produce the flat wire gradient of one local batch.

* ``HipCompute``   — the MI355X path: models/engine.py (hand-written CDNA4 kernels), whole step
                     captured in a HIP graph; parameters come from the worker-local fp32 arena.
* ``TorchCompute`` — the CPU reference path (torch nn.Module + autograd), used by the CPU
                     test-suite and for numerics checks. It is never selected on a GPU device.

Both expose the same surface: ``local_arena`` (fetched server state, fp32), ``grads`` (wire
buffer over the trainable-parameter prefix, fp16 codec or fp32), ``train_step(indices)``,
``evaluate(dataset)`` and ``last_loss()``. This replaces the reference's
setup_model/train_local_batch/evaluate_model (src/workers/worker.py:128-138,313-348).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F

from ..models.layout import ParamLayout
from ..models.resnet import MODEL_INPUT


class TorchCompute:
    def __init__(self, model: torch.nn.Module, layout: ParamLayout, batch: int, grad_dtype=torch.float16,
                 mean=(0.5071, 0.4867, 0.4408), std=(0.2675, 0.2565, 0.2761), seed: int = 0):
        self.model = model.cpu()
        self.layout = layout
        self.B = batch
        self.device = torch.device("cpu")
        self.local_arena = torch.zeros(layout.arena_numel, dtype=torch.float32)
        self.grads = torch.zeros(layout.param_numel, dtype=grad_dtype)
        self.mean = torch.tensor(mean).view(1, 3, 1, 1)
        self.std = torch.tensor(std).view(1, 3, 1, 1)
        self._loss = 0.0
        self._step = 0
        self.seed = seed

    # arena <-> module
    def _load_module(self):
        with torch.no_grad():
            sd = self.model.state_dict()
            for name, e in self.layout.entries.items():
                if e.region == "counter":
                    continue
                sd[name].copy_(self.local_arena[e.offset:e.offset + e.numel].view(e.shape))

    def _store_buffers(self):
        with torch.no_grad():
            sd = self.model.state_dict()
            for name, e in self.layout.entries.items():
                if e.region == "buffer":
                    self.local_arena[e.offset:e.offset + e.numel] = sd[name].reshape(-1)

    def _batch(self, dataset, idx, train=True):
        x = dataset.images[torch.as_tensor(idx, dtype=torch.long)].permute(0, 3, 1, 2).float() / 255.0
        if train:
            rng = np.random.default_rng([self.seed, self._step])
            xp = F.pad(x, (4, 4, 4, 4))
            out = torch.empty_like(x)
            for i in range(x.shape[0]):
                dy, dx = rng.integers(0, 9, size=2)
                crop = xp[i, :, dy:dy + x.shape[2], dx:dx + x.shape[3]]
                out[i] = crop.flip(2) if rng.integers(0, 2) else crop
            x = out
        x = (x - self.mean) / self.std
        y = dataset.labels[torch.as_tensor(idx, dtype=torch.long)].long()
        return x, y

    def set_buckets(self, buckets):
        self._nbuckets = len(buckets)

    def train_step(self, dataset, idx, on_bucket=None):
        self._load_module()
        self.model.train()
        self.model.zero_grad(set_to_none=False)
        x, y = self._batch(dataset, idx, train=True)
        out = self.model(x)
        loss = F.cross_entropy(out, y)
        loss.backward()
        self._loss = loss.item()
        self._correct = int((out.argmax(1) == y).sum())
        with torch.no_grad():
            for name, p in self.model.named_parameters():
                e = self.layout.entries[name]
                self.grads[e.offset:e.offset + e.numel] = p.grad.reshape(-1).to(self.grads.dtype)
        self._store_buffers()
        self._step += 1
        if on_bucket is not None:  # eager CPU path: every bucket is final after backward
            for k in range(self._nbuckets):
                on_bucket(k, self.grads)

    def last_loss(self) -> float:
        return self._loss

    def pad_grads(self, n: int):
        """Grow the gradient wire buffer to n elements (zero tail), see HipCompute.pad_grads."""
        if self.grads.numel() < n:
            g = torch.zeros(n, dtype=self.grads.dtype)
            g[: self.grads.numel()].copy_(self.grads)
            self.grads = g

    def step_stats(self):
        """(sum of per-sample losses, #correct) of the last train step."""
        return torch.tensor(self._loss * self.B, dtype=torch.float64), torch.tensor(self._correct)

    @torch.no_grad()
    def evaluate(self, dataset, batch=None) -> float:
        self._load_module()
        self.model.eval()
        b = batch or self.B
        correct = 0
        n = len(dataset)
        for s in range(0, n, b):
            idx = np.arange(s, min(n, s + b))
            x, y = self._batch(dataset, idx, train=False)
            correct += int((self.model(x).argmax(1) == y).sum())
        return 100.0 * correct / max(1, n)


class HipCompute:
    def __init__(self, model: torch.nn.Module, layout: ParamLayout, batch: int, device, model_name="resnet18",
                 grad_dtype=torch.float16, seed: int = 0, use_graph: bool = True, dtype: str = "fp32",
                 deterministic: bool | None = None):
        from ..models.engine import CIFAR_MEAN, CIFAR_STD, IMAGENET_MEAN, IMAGENET_STD, HipResNetEngine

        (c, h, w), _ = MODEL_INPUT.get(model_name, ((3, 32, 32), 100))
        mean, std = (CIFAR_MEAN, CIFAR_STD) if h == 32 else (IMAGENET_MEAN, IMAGENET_STD)
        self.device = torch.device(device)
        self.layout = layout
        self.B = batch
        self.engine = HipResNetEngine(model, layout, batch, device=self.device, grad_dtype=grad_dtype, in_hw=(h, w),
                                      mean=mean, std=std, seed=1234 + seed,
                                      dtype=torch.float32 if dtype == "fp32" else torch.bfloat16,
                                      deterministic=deterministic)
        self.local_arena = torch.zeros(layout.arena_numel, dtype=torch.float32, device=self.device)
        self.grads = self.engine.grads
        self.use_graph = use_graph
        self._dataset = None
        self._step = 0
        # pinned staging ring for [batch indices | step] (one H2D copy per step); a slot is
        # rewritten only after the copy that last read it has run (its event), so the host may
        # run ahead of the device by up to len(ring) steps without racing the DMA
        self._meta_ring = [torch.zeros(batch + 1, dtype=torch.int32).pin_memory() for _ in range(4)]
        self._meta_ev = [None] * len(self._meta_ring)
        self._meta_i = 0
        self.host_wait_s = 0.0

    def _set_batch(self, idx):
        k = self._meta_i % len(self._meta_ring)
        self._meta_i += 1
        if self._meta_ev[k] is not None:
            t0 = time.perf_counter()
            self._meta_ev[k].synchronize()
            self.host_wait_s += time.perf_counter() - t0  # host ahead of the device by len(ring)
        buf = self._meta_ring[k]
        buf[: self.B].copy_(torch.as_tensor(idx, dtype=torch.int32))
        buf[self.B] = self._step
        self.engine.batch_meta.copy_(buf, non_blocking=True)
        ev = self._meta_ev[k] or torch.cuda.Event()
        ev.record()
        self._meta_ev[k] = ev

    def set_buckets(self, buckets):
        self.engine.set_segments([b.keys for b in buckets])

    def use_wire(self, wire, small_from=None):
        """Fetches land in ``wire`` (parallel/codec.py WeightWire) instead of the fp32 local
        arena: every captured step unpacks the conv operands straight from the wire's bf16 image
        and, in the same launch, scatters the fp32 remainder (BN affine, FC, BN running
        statistics) into the local arena. ``small_from``: the server's fp32 arena, when this
        worker shares the server's device and reads the server's own wire (co-located sync
        round) — the remainder is then gathered from it directly and the server need not
        publish it. The local arena's conv-weight region is not used any more."""
        self.wire = wire
        self.engine.set_weight_source(wire.img, scatter=wire.scatter_spec(self.local_arena, small_from))

    def pad_grads(self, n: int):
        """Grow the gradient wire buffer to n elements (zero tail): collectives that split it
        into equal per-rank chunks (the sharded server's reduce-scatter). Invalidates graphs."""
        if self.grads.numel() < n:
            g = torch.zeros(n, dtype=self.grads.dtype, device=self.grads.device)
            g[: self.grads.numel()].copy_(self.grads)
            self.engine.grads = self.grads = g
            self.engine.graph = self.engine.graphs = None

    def train_step(self, dataset, idx, on_bucket=None, round_hooks=None):
        seg = (lambda k: on_bucket(k, self.grads)) if on_bucket is not None else None
        self._set_batch(idx)
        if round_hooks is not None:  # the whole PS round in one graph (parallel/graph_round.py)
            if not self.use_graph:
                self.engine.train_step(self.local_arena, dataset.images, dataset.labels, unpack=True,
                                       on_segment=round_hooks.after_segment)
                round_hooks.finish()
            else:
                if self.engine.graph is None or self._dataset is not dataset:
                    self._dataset = dataset
                    backup = self.local_arena.clone()
                    self.engine.capture(self.local_arena, dataset.images, dataset.labels, unpack=True, warmup=1)
                    self.local_arena.copy_(backup)
                    del backup
                # one graph per backward segment; after each replay the segment's reduce/apply/
                # broadcast is forked onto the communication stream (the compute stream never waits)
                self.engine.step_graph(on_segment=round_hooks.after_segment)
                round_hooks.finish()
            self._step += 1
            return
        if self.use_graph:
            if self.engine.graph is None or self._dataset is not dataset:
                # One-time capture of unpack + augment + fwd + bwd over the fixed local arena
                # (fetches land in it in place). Warm-up/capture side effects on the BN running
                # statistics are undone so the first replay starts from the fetched state.
                self._dataset = dataset
                backup = self.local_arena.clone()
                self.engine.capture(self.local_arena, dataset.images, dataset.labels, unpack=True, warmup=1)
                self.local_arena.copy_(backup)
                del backup
            self.engine.step_graph(on_segment=seg)
        else:
            self.engine.train_step(self.local_arena, dataset.images, dataset.labels, unpack=True, on_segment=seg)
        self._step += 1

    def last_loss(self) -> float:
        return float(self.engine.loss.mean())

    def rewind(self, step: int):
        """Re-enter training at local step ``step`` (sync shrink rollback, parallel/elastic.py):
        the augmentation stream is keyed by the step counter, and the BN statistic shifts came
        from steps the rollback discarded — the next step sums plainly, as a fresh engine's first
        step does (HipResNetEngine.reset_stat_shift)."""
        self._step = int(step)
        self.engine.reset_stat_shift()

    def step_stats(self):
        """Device tensors (sum of per-sample losses, #correct) of the last train step (no sync)."""
        return self.engine.loss.sum(dtype=torch.float64), self.engine.correct.sum(dtype=torch.int64)

    @torch.no_grad()
    def evaluate(self, dataset, batch=None) -> float:
        n = len(dataset)
        B = self.B
        correct = 0
        self.engine.unpack(self.local_arena)
        for s in range(0, n, B):
            idx = np.arange(s, s + B) % n
            self._set_batch(idx)
            self.engine.evaluate_batch(self.local_arena, dataset.images, dataset.labels)
            valid = min(B, n - s)
            if valid == B:
                correct += int(self.engine.correct.item())
            else:  # partial last batch: recount only the valid rows
                logits_ok = self._count_prefix(valid)
                correct += logits_ok
        return 100.0 * correct / max(1, n)

    def _count_prefix(self, valid: int) -> int:
        # re-run the head on the first `valid` samples only
        from ..ops import kernels as K

        sp = self.engine.spec
        self.engine.correct.zero_()
        K.head_fwd_bwd(self.engine.final, valid, self.engine.head_hw, sp.fc_in,
                       self.layout.view(self.local_arena, f"{sp.fc}.weight"),
                       self.layout.view(self.local_arena, f"{sp.fc}.bias"), sp.classes, self.engine.labels,
                       self.engine.pooled, self.engine.dlogits, None, self.engine.loss, self.engine.correct)
        return int(self.engine.correct.item())


def make_compute(model, layout, batch, device, model_name="resnet18", grad_dtype=torch.float16, seed=0,
                 use_graph=True, dtype="fp32", deterministic=None):
    """The worker's local fwd/bwd: the HIP engine on a GPU (compute dtype fp32 or bf16), torch
    fp32 autograd on the CPU (tests)."""
    dev = torch.device(device)
    if dev.type == "cuda":
        return HipCompute(model, layout, batch, dev, model_name, grad_dtype, seed, use_graph, dtype, deterministic)
    return TorchCompute(model, layout, batch, grad_dtype, seed=seed)
