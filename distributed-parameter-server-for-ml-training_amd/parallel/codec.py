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
