"""Wire codecs of the PS protocol.

Fetch (server -> worker). The reference ships the full fp32 state_dict on every fetch
(reference: src/parameter_server/server.py:221-223, 44.9 MB for ResNet-18). Two fetch codecs:

* ``fp32``     — the reference payload: the whole fp32 arena (params + BN buffers).
* ``bf16conv`` — (default) exactly the bits a psx worker consumes: conv weights as bf16 (the HIP
  engine rounds every conv weight to bf16 before use, csrc/kernels/optim.hip param_unpack, so a
  worker that receives fp32 and rounds locally computes bit-identical results) plus fp32 for
  every other tensor (BN affine, FC, BN running statistics). 22.5 MB instead of 44.9 MB per
  fetch for ResNet-18, and the worker-side arena is reconstructed exactly (bf16 -> fp32 is exact).

Push (worker -> server): the reference's fp16 cast (worker.py:264-268) is the default wire dtype
of the gradient buffer; top-k sparsification lives in parallel/topk.py.
"""
from __future__ import annotations

import torch


class FetchCodec:
    def __init__(self, layout, kind: str = "bf16conv", device="cpu"):
        if kind not in ("fp32", "bf16conv"):
            raise ValueError(f"unknown fetch codec {kind!r}")
        self.kind = kind
        self.layout = layout
        self.device = torch.device(device)
        n = layout.arena_numel
        if kind == "fp32":
            self.wire = [torch.zeros(n, dtype=torch.float32, device=self.device)]
            return
        conv_mask = torch.zeros(layout.param_numel, dtype=torch.bool)
        for e in layout.entries.values():
            if e.region == "param" and len(e.shape) == 4:
                conv_mask[e.offset:e.offset + e.numel] = True
        keep = torch.cat([torch.nonzero(~conv_mask).flatten(),
                          torch.arange(layout.param_numel, n, dtype=torch.int64)])
        self.small_index = keep.to(self.device)
        self.wire = [torch.zeros(layout.param_numel, dtype=torch.bfloat16, device=self.device),
                     torch.zeros(keep.numel(), dtype=torch.float32, device=self.device)]

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.wire)

    def pack(self, arena: torch.Tensor):
        """server arena -> wire buffers (stream-ordered after the update)."""
        if self.kind == "fp32":
            self.wire[0].copy_(arena)
            return self.wire
        self.wire[0].copy_(arena[: self.layout.param_numel])
        torch.index_select(arena, 0, self.small_index, out=self.wire[1])
        return self.wire

    def unpack(self, local_arena: torch.Tensor, wire=None):
        wire = wire if wire is not None else self.wire
        if self.kind == "fp32":
            if wire[0].data_ptr() != local_arena.data_ptr():
                local_arena.copy_(wire[0])
            return local_arena
        local_arena[: self.layout.param_numel].copy_(wire[0])
        local_arena.index_copy_(0, self.small_index, wire[1])
        return local_arena


def small_index_of(layout) -> torch.Tensor:
    """Arena indices of everything that is not a conv weight: BN affine, FC, BN buffers."""
    conv_mask = torch.zeros(layout.param_numel, dtype=torch.bool)
    for e in layout.entries.values():
        if e.region == "param" and len(e.shape) == 4:
            conv_mask[e.offset:e.offset + e.numel] = True
    return torch.cat([torch.nonzero(~conv_mask).flatten(),
                      torch.arange(layout.param_numel, layout.arena_numel, dtype=torch.int64)])


class WeightWire:
    """The ``bf16conv`` fetch payload as ONE contiguous buffer that the server writes in place
    and the HIP engine reads in place (the sync fast path, see weight_image_enabled):

        buf = [ img: bf16 bits of every trainable parameter (param_numel, 16-byte padded)
              | small: fp32 of the non-conv entries (BN affine, FC, BN running statistics) ]

    * server: the fused SGD apply writes ``img`` in the same pass as the fp32 update
      (csrc/kernels/optim.hip sgd_apply img), ``publish_small`` gathers the fp32 remainder
      once per round — no separate pack kernel, one broadcast per fetch;
    * worker: the captured step scatters ``small`` into its local arena and unpacks the conv
      operands straight from ``img`` (csrc/kernels/optim.hip param_unpack_tiles on bf16), so the
      fp32 conv weights are never materialised on a worker (bf16 is all the engine computes
      with; bit-identical to unpacking the fp32 master copy).

    Same bytes as FetchCodec("bf16conv") (22.5 MB for ResNet-18 vs 44.9 MB fp32)."""

    def __init__(self, layout, device, small_index: torch.Tensor | None = None):
        self.layout = layout
        self.device = torch.device(device)
        n = layout.param_numel
        idx = small_index if small_index is not None else small_index_of(layout)
        self.small_index = idx.to(self.device)
        self.img_bytes = -(-2 * n // 16) * 16
        self.buf = torch.zeros(self.img_bytes + 4 * idx.numel(), dtype=torch.uint8, device=self.device)
        self.img = self.buf[: 2 * n].view(torch.bfloat16)
        self.small = self.buf[self.img_bytes:].view(torch.float32)

    @property
    def nbytes(self) -> int:
        return self.buf.numel()

    def publish_small(self, arena: torch.Tensor):
        torch.index_select(arena, 0, self.small_index, out=self.small)

    def publish_full(self, arena: torch.Tensor):
        """Whole payload from the fp32 arena (initial state, resume, out-of-band updates)."""
        self.img.copy_(arena[: self.layout.param_numel])  # RNE, same bits as the kernels' f2bf
        self.publish_small(arena)

    def consume_small(self, local_arena: torch.Tensor):
        local_arena.index_copy_(0, self.small_index, self.small)

    def scatter_spec(self, local_arena: torch.Tensor, small_from: torch.Tensor | None = None):
        """How the unpack launch scatters the fp32 remainder into ``local_arena``
        (kernels.param_unpack_tiles ``scatter``): from this wire, or gathered straight from the
        server arena ``small_from``."""
        if small_from is not None:
            return (small_from, self.small_index, local_arena, True)
        return (self.small, self.small_index, local_arena, False)

    def to_arena(self, local_arena: torch.Tensor):
        """Materialise the full fp32 state (conv weights exact from bf16) — tests/diagnostics."""
        local_arena[: self.layout.param_numel].copy_(self.img)
        self.consume_small(local_arena)
        return local_arena


def weight_image_enabled(cfg) -> bool:
    """The WeightWire fast path applies to sync rounds that push every batch with a dense
    gradient and the bf16conv fetch codec (the semantics are then exactly those of
    fetch-into-the-local-arena, see WeightWire). PSX_WEIGHT_IMAGE=0 turns it off (A/B)."""
    import os

    return (os.environ.get("PSX_WEIGHT_IMAGE", "1") != "0" and cfg.mode == "sync" and max(1, cfg.sync_steps) == 1
            and cfg.codec in ("fp16", "none") and cfg.fetch_codec == "bf16conv" and not cfg.overlap)
