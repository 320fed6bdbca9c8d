"""Datasets, per-worker sharding and epoch sampling.

Reference behaviour (src/workers/worker.py:140-197):
  * CIFAR-100 train set partitioned into contiguous index ranges:
      samples_per_worker = N // W; worker k gets [k*spw, (k+1)*spw), the last worker also takes
      the remainder (worker.py:166-179);
  * shuffled DataLoader per shard, batch_size from the CLI, no drop_last; full 10k test set.

MI355X-native design: the whole uint8 dataset lives in HBM (50000x32x32x3 = 153 MB of 288 GB),
each step gathers its batch and applies crop/flip/normalize in one HIP kernel
(csrc/kernels/data.hip), so there are no DataLoader worker processes and no host->device copy
in the training loop. Sources: a deterministic learnable synthetic CIFAR-shaped set (default; no
network access for the real one) or the official CIFAR-100 *binary* files read by the native
reader (csrc/runtime/cifar_io.cpp). The epoch order is a per-(seed, epoch, shard) permutation;
the final partial batch is filled by wrapping to the start of the permutation, so every worker
runs ceil(shard/B) steps per epoch exactly like the reference DataLoader.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch


def shard_range(worker_id: int, total_workers: int, n: int) -> tuple[int, int]:
    """Contiguous shard of worker ``worker_id`` (reference worker.py:166-179)."""
    if not (0 <= worker_id < total_workers):
        raise ValueError(f"worker_id {worker_id} outside [0, {total_workers})")
    spw = n // total_workers
    start = worker_id * spw
    end = n if worker_id == total_workers - 1 else start + spw
    return start, end


def steps_per_epoch(n_shard: int, batch: int) -> int:
    return -(-n_shard // batch)


class DeviceDataset:
    """uint8 NHWC images + int32 labels resident on one device (or CPU for the test path)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor):
        assert images.dtype == torch.uint8 and images.dim() == 4 and images.shape[-1] == 3
        self.images = images
        self.labels = labels.to(torch.int32)

    def __len__(self):
        return self.images.shape[0]

    @classmethod
    def synthetic(cls, n: int, hw: int = 32, classes: int = 100, seed: int = 0, device="cuda", offset: int = 0):
        dev = torch.device(device)
        imgs = torch.empty(n, hw, hw, 3, dtype=torch.uint8, device=dev)
        labs = torch.empty(n, dtype=torch.int32, device=dev)
        if dev.type == "cuda":
            from ..ops import kernels as K

            K.synth_gen(imgs, labs, n, hw, hw, classes, seed, offset)
        else:
            imgs_np, labs_np = synthetic_numpy(n, hw, classes, seed, offset)
            imgs.copy_(torch.from_numpy(imgs_np))
            labs.copy_(torch.from_numpy(labs_np))
        return cls(imgs, labs)

    @classmethod
    def synthetic_hard(cls, n: int, hw: int = 32, classes: int = 100, seed: int = 0, device="cuda", offset: int = 0,
                       label_noise: float = 0.2):
        """synthetic_hard_numpy, resident on ``device``."""
        imgs, labs = synthetic_hard_numpy(n, hw, classes, seed, offset, label_noise)
        return cls(torch.from_numpy(imgs).to(device), torch.from_numpy(labs).to(device))

    @classmethod
    def cifar_binary(cls, path: str, label_bytes: int = 2, label_index: int = 1, max_records: int = 0,
                     device="cuda"):
        from ..ops._lib import runtime

        rt = runtime()
        n = rt.psx_cifar_count(path.encode(), label_bytes)
        if n <= 0:
            raise FileNotFoundError(f"{path}: not a CIFAR binary file")
        if max_records:
            n = min(n, max_records)
        img = np.empty((n, 32, 32, 3), dtype=np.uint8)
        lab = np.empty((n,), dtype=np.int32)
        got = rt.psx_cifar_read(path.encode(), label_bytes, label_index, img.ctypes.data_as(C.c_void_p),
                                lab.ctypes.data_as(C.c_void_p), n, min(8, os.cpu_count() or 1))
        if got != n:
            raise IOError(f"{path}: read {got} of {n} records")
        return cls(torch.from_numpy(img).to(device), torch.from_numpy(lab).to(device))


def synthetic_hard_numpy(n: int, hw: int = 32, classes: int = 100, seed: int = 0, offset: int = 0,
                         label_noise: float = 0.2, chunk: int = 4096):
    """Class-conditional noise with label noise (convergence studies, ``--synthetic-kind hard``):
    low-contrast 4x4 class prototypes (128 + 12·N(0,1) per cell and channel) under per-pixel
    Gaussian noise of std 64, and a fraction ``label_noise`` of the labels replaced by a uniformly
    drawn class. Not trivially separable, and the label noise caps the attainable accuracy at
    about 1 - label_noise·(1 - 1/classes). The prototypes depend on ``seed`` only, so the train
    set (offset 0) and the test set (another offset) share them."""
    protos = 128.0 + 12.0 * np.random.default_rng([seed, 7]).standard_normal((classes, 4, 4, 3))
    up = np.repeat(np.repeat(protos, hw // 4, axis=1), hw // 4, axis=2).astype(np.float32)
    rng = np.random.default_rng([seed, offset, 1])
    labels = rng.integers(0, classes, size=n)
    imgs = np.empty((n, hw, hw, 3), dtype=np.uint8)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        x = up[labels[s:e]] + 64.0 * rng.standard_normal((e - s, hw, hw, 3), dtype=np.float32)
        imgs[s:e] = np.clip(np.rint(x), 0, 255).astype(np.uint8)
    noisy = rng.random(n) < label_noise
    observed = np.where(noisy, rng.integers(0, classes, size=n), labels).astype(np.int32)
    return imgs, observed


def synthetic_numpy(n: int, hw: int = 32, classes: int = 100, seed: int = 0, offset: int = 0):
    """CPU twin of the synthetic generator (class prototype + noise), for the CPU test path."""
    protos = np.random.default_rng(seed).integers(0, 200, size=(classes, 4, 4, 3)).astype(np.int16)
    rng = np.random.default_rng([seed, offset])
    labels = rng.integers(0, classes, size=n).astype(np.int32)
    up = np.repeat(np.repeat(protos, hw // 4, axis=1), hw // 4, axis=2)
    noise = rng.integers(-32, 32, size=(n, hw, hw, 3)).astype(np.int16)
    imgs = np.clip(up[labels] + noise, 0, 255).astype(np.uint8)
    return imgs, labels


class EpochSampler:
    """Per-epoch shuffled batches of a contiguous shard, padded by wrap-around."""

    def __init__(self, start: int, end: int, batch: int, seed: int = 0, shuffle: bool = True,
                 steps: int | None = None):
        self.start, self.end, self.batch = start, end, batch
        self.seed, self.shuffle = seed, shuffle
        # collective (sync) runs force one common step count for every worker
        self.steps = steps

    def __len__(self):
        return self.steps if self.steps is not None else steps_per_epoch(self.end - self.start, self.batch)

    def epoch_indices(self, epoch: int) -> np.ndarray:
        n = self.end - self.start
        idx = np.arange(self.start, self.end, dtype=np.int32)
        if self.shuffle:
            rng = np.random.default_rng([self.seed, epoch, self.start])
            idx = idx[rng.permutation(n)]
        total = len(self) * self.batch
        if total != n:
            idx = np.resize(idx, total)  # cyclic wrap-around fill of the final batch (or truncation)
        return idx.reshape(len(self), self.batch)
