"""Flat parameter arena + name -> offset table, in reference ``state_dict`` terms.

The reference server keeps ``self.parameters = {name: np.ndarray}`` — the full state_dict
(params *and* BN buffers) — and ships it pickled on every fetch (reference:
src/parameter_server/server.py:95-96,221-223). Here that state is one contiguous fp32 arena in
HBM so that a fetch is a single RCCL broadcast / send of one buffer, an update is one fused
kernel over one buffer, and a checkpoint is one device->host copy:

    arena = [ trainable params (named_parameters order) | float buffers (state_dict order) ]
    counters = int64 [num_batches_tracked ...] (host side; never updated by the server)

Because trainable parameters form one prefix, the gradient wire buffer (fp16 codec) is simply
``arena[:param_numel]``-shaped and the server update is a flat elementwise kernel.
``to_state_dict`` / ``from_state_dict`` convert to and from the reference's exact key order,
shapes and dtypes (checkpoint parity, see utils/checkpoint.py).
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np
import torch


@dataclass
class Entry:
    name: str
    shape: tuple
    dtype: str  # "float32" | "int64"
    region: str  # "param" | "buffer" | "counter"
    offset: int  # element offset inside its region (arena for param/buffer, counters array)
    numel: int


@dataclass
class ParamLayout:
    entries: "OrderedDict[str, Entry]" = field(default_factory=OrderedDict)  # state_dict order
    param_numel: int = 0
    buffer_numel: int = 0
    num_counters: int = 0

    @property
    def arena_numel(self) -> int:
        return self.param_numel + self.buffer_numel

    @property
    def param_names(self):
        return [e.name for e in self.entries.values() if e.region == "param"]

    @classmethod
    def from_module(cls, module: torch.nn.Module) -> "ParamLayout":
        sd = module.state_dict()
        pnames = [n for n, _ in module.named_parameters()]
        lay = cls()
        off = 0
        tmp = {}
        for n in pnames:
            t = sd[n]
            tmp[n] = Entry(n, tuple(t.shape), "float32", "param", off, t.numel())
            off += t.numel()
        lay.param_numel = off
        boff, coff = 0, 0
        for n, t in sd.items():
            if n in tmp:
                continue
            if t.dtype == torch.int64:
                tmp[n] = Entry(n, tuple(t.shape), "int64", "counter", coff, max(1, t.numel()))
                coff += max(1, t.numel())
            else:
                tmp[n] = Entry(n, tuple(t.shape), "float32", "buffer", off + boff, t.numel())
                boff += t.numel()
        lay.buffer_numel = boff
        lay.num_counters = coff
        for n in sd.keys():
            lay.entries[n] = tmp[n]
        return lay

    # ------------------------------------------------------------------ conversions
    def pack(self, module_or_sd) -> tuple[torch.Tensor, torch.Tensor]:
        """state_dict (or module) -> (fp32 arena, int64 counters) on CPU."""
        sd = module_or_sd.state_dict() if isinstance(module_or_sd, torch.nn.Module) else module_or_sd
        return self.from_state_dict(sd)

    def from_state_dict(self, sd) -> tuple[torch.Tensor, torch.Tensor]:
        arena = torch.zeros(self.arena_numel, dtype=torch.float32)
        counters = torch.zeros(max(1, self.num_counters), dtype=torch.int64)
        missing = [n for n in self.entries if n not in sd]
        if missing:
            raise KeyError(f"state_dict is missing {len(missing)} entries, e.g. {missing[:3]}")
        for n, e in self.entries.items():
            v = sd[n]
            v = torch.as_tensor(np.asarray(v)) if not torch.is_tensor(v) else v
            if tuple(v.shape) != e.shape:
                raise ValueError(f"{n}: shape {tuple(v.shape)} != layout {e.shape}")
            if e.region == "counter":
                counters[e.offset] = int(v.reshape(-1)[0]) if v.numel() else 0
            else:
                arena[e.offset:e.offset + e.numel] = v.detach().reshape(-1).to(torch.float32).cpu()
        return arena, counters

    def to_state_dict(self, arena: torch.Tensor, counters: torch.Tensor | None = None, as_numpy: bool = False):
        """(arena, counters) -> OrderedDict with the reference's keys, order, shapes and dtypes."""
        arena = arena.detach().cpu()
        out = OrderedDict()
        for n, e in self.entries.items():
            if e.region == "counter":
                val = int(counters[e.offset]) if counters is not None else 0
                t = torch.tensor(val, dtype=torch.int64).reshape(e.shape)
            else:
                t = arena[e.offset:e.offset + e.numel].reshape(e.shape).clone()
            out[n] = t.numpy() if as_numpy else t
        return out

    def view(self, arena: torch.Tensor, name: str) -> torch.Tensor:
        e = self.entries[name]
        if e.region == "counter":
            raise KeyError(f"{name} is a host counter, not in the arena")
        return arena[e.offset:e.offset + e.numel].view(e.shape)

    def offset(self, name: str) -> int:
        return self.entries[name].offset

    def grad_view(self, grads: torch.Tensor, name: str) -> torch.Tensor:
        e = self.entries[name]
        assert e.region == "param", name
        return grads[e.offset:e.offset + e.numel].view(e.shape)

    def summary(self) -> dict:
        return {
            "state_dict_entries": len(self.entries),
            "trainable_tensors": sum(1 for e in self.entries.values() if e.region == "param"),
            "trainable_params": self.param_numel,
            "float_buffer_elems": self.buffer_numel,
            "int64_counters": self.num_counters,
            "arena_bytes_fp32": 4 * self.arena_numel,
            "grad_wire_bytes_fp16": 2 * self.param_numel,
        }
