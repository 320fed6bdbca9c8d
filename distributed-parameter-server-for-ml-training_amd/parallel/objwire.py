"""Control-plane object codec: tagged JSON instead of pickle.

The reference ships every message as a pickle over gRPC (src/communication/ps_pb2_grpc.py,
src/parameter_server/server.py:370-393: ``pickle.loads`` of whatever a peer sent), which lets a
peer run code in the receiver. psx's control plane carries only small host values — rank names,
counts, error strings, RCCL unique ids (bytes), ``{rank: id}`` maps, step numbers, the elastic
plan dict — so it encodes them as JSON with three tags and never unpickles:

  bytes   -> {"__b": base64}         (RCCL unique ids)
  tuple   -> {"__t": [items]}
  dict with non-string keys -> {"__d": [[key, value], ...]}

Anything else (objects, sets, tensors) raises TypeError at the sender. Used by the transports'
``all_gather_object`` / ``broadcast_object`` on the gloo control group and on the TCPStore
(parallel/transport.py, parallel/elastic.py).
"""
from __future__ import annotations

import base64
import json

import torch
import torch.distributed as dist


def _enc(o):
    if o is None or isinstance(o, (bool, int, float, str)):
        return o
    if isinstance(o, (bytes, bytearray)):
        return {"__b": base64.b64encode(bytes(o)).decode("ascii")}
    if isinstance(o, tuple):
        return {"__t": [_enc(v) for v in o]}
    if isinstance(o, list):
        return [_enc(v) for v in o]
    if isinstance(o, dict):
        if all(isinstance(k, str) and not k.startswith("__") for k in o):
            return {k: _enc(v) for k, v in o.items()}
        return {"__d": [[_enc(k), _enc(v)] for k, v in o.items()]}
    raise TypeError(f"control-plane value of type {type(o).__name__} is not JSON-encodable")


def _dec(o):
    if isinstance(o, list):
        return [_dec(v) for v in o]
    if isinstance(o, dict):
        if len(o) == 1:
            (k, v), = o.items()
            if k == "__b":
                return base64.b64decode(v)
            if k == "__t":
                return tuple(_dec(x) for x in v)
            if k == "__d":
                return {_dec(a): _dec(b) for a, b in v}
        return {k: _dec(v) for k, v in o.items()}
    return o


def dumps(obj) -> bytes:
    return json.dumps(_enc(obj), separators=(",", ":"), allow_nan=True).encode("utf-8")


def loads(data: bytes):
    return _dec(json.loads(bytes(data).decode("utf-8")))


def all_gather(obj, group, world_size: int) -> list:
    """``dist.all_gather_object`` over ``group`` (a CPU / gloo group) with this codec: lengths,
    then the zero-padded payloads, as uint8 tensors."""
    data = dumps(obj)
    n = torch.tensor([len(data)], dtype=torch.int64)
    lens = [torch.zeros(1, dtype=torch.int64) for _ in range(world_size)]
    dist.all_gather(lens, n, group=group)
    m = max(int(x.item()) for x in lens)
    buf = torch.zeros(m, dtype=torch.uint8)
    buf[: len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    outs = [torch.empty(m, dtype=torch.uint8) for _ in range(world_size)]
    dist.all_gather(outs, buf, group=group)
    return [loads(o[: int(lens[r].item())].numpy().tobytes()) for r, o in enumerate(outs)]


def broadcast(obj, group, src: int = 0, rank: int = 0):
    """``dist.broadcast_object_list([obj])[0]`` over ``group`` with this codec (``rank`` is the
    caller's rank in the group's numbering; ``obj`` is read on ``src`` only)."""
    data = dumps(obj) if rank == src else b""
    n = torch.tensor([len(data)], dtype=torch.int64)
    dist.broadcast(n, src=src, group=group)
    buf = torch.empty(int(n.item()), dtype=torch.uint8)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    dist.broadcast(buf, src=src, group=group)
    return loads(buf.numpy().tobytes())
