"""Server checkpoint / resume in the reference's state_dict-keyed layout.

The reference has no checkpointing (listed as future work, reference DEPLOYMENT.md:309); its
de-facto wire layout is the FetchReply payload ``{state_dict_name: ndarray}``
(src/parameter_server/server.py:221-223). A psx checkpoint is that dict plus server state:

    {"format": "psx-ckpt-v1",
     "parameters": OrderedDict{name: tensor}   # keys/order/shapes/dtypes = reference state_dict
     "global_step": int, "mode": str, "total_workers": int, "lr": float,
     "server_optimizer_state": {"momentum": tensor | None}, "config": json str}

Written with torch.save to a temp file + atomic rename; loaded with
``torch.load(weights_only=True)`` (no arbitrary unpickling). ``parameters`` can be fed straight
into ``ResNet18().load_state_dict`` of the reference model.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

FORMAT = "psx-ckpt-v1"


def save(path: str, layout, arena: torch.Tensor, counters: torch.Tensor | None, global_step: int, mode: str,
         total_workers: int, lr: float, momentum_buf: torch.Tensor | None = None, config_json: str = "") -> str:
    sd = layout.to_state_dict(arena, counters)
    obj = {
        "format": FORMAT,
        "parameters": OrderedDict(sd),
        "global_step": int(global_step),
        "mode": mode,
        "total_workers": int(total_workers),
        "lr": float(lr),
        "server_optimizer_state": {"momentum": None if momentum_buf is None else momentum_buf.detach().cpu()},
        "config": config_json,
    }
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)
    return path


def load(path: str) -> dict:
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if obj.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    return obj


def restore(path: str, layout):
    """-> (arena fp32 CPU tensor, counters int64, global_step, momentum or None, full dict)."""
    obj = load(path)
    arena, counters = layout.from_state_dict(obj["parameters"])
    mom = obj.get("server_optimizer_state", {}).get("momentum")
    return arena, counters, int(obj["global_step"]), mom, obj


def latest(ckpt_dir: str) -> str | None:
    if not os.path.isdir(ckpt_dir):
        return None
    cands = [f for f in os.listdir(ckpt_dir) if f.startswith("step_") and f.endswith(".pt")]
    if not cands:
        return None
    cands.sort(key=lambda f: int(f[5:-3]))
    return os.path.join(ckpt_dir, cands[-1])


def path_for(ckpt_dir: str, step: int) -> str:
    return os.path.join(ckpt_dir, f"step_{step:08d}.pt")
