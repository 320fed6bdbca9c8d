"""Data plane: bulk tensor movement between the parameter server (rank 0) and the workers.

Replaces the reference's gRPC + pickle transport (reference: src/communication/ps_pb2_grpc.py:28-121,
src/parameter_server/server.py:370-393, src/workers/worker.py:199-311):

  reference RPC               payload                          here (one process per GPU)
  PushGradrients  (sync)      pickled fp16 dict, 22.4 MB       RCCL reduce(sum) of the flat fp16
                                                               wire buffer to rank 0
  FetchParameters (sync)      pickled fp32 state_dict, 44.9 MB RCCL broadcast of the flat fp32 arena
  PushGradrients  (async)     same                             RCCL send(worker -> 0) into a
                                                               per-worker staging slot
  FetchParameters (async)     same                             RCCL send(0 -> worker) of a
                                                               per-worker snapshot of the arena

``DistTransport`` is torch.distributed with backend "nccl" (= RCCL over xGMI on ROCm) for
device tensors, or "gloo" for the CPU test path — the same code drives both. A gloo side group
carries small host-side collectives (registration names, metrics gathering).
``LocalTransport`` is the single-process (1 GPU, server + workers co-located) loopback.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class LocalTransport:
    rank = 0
    world_size = 1
    is_distributed = False

    def __init__(self, device):
        self.device = torch.device(device)

    def reduce_sum_to_server(self, t):
        return t

    def broadcast_from_server(self, t):
        return t

    def gather_to_server(self, t):
        return [t]

    def gather_from_workers(self, t, bufs):
        """No remote ranks in a single process."""
        assert not bufs
        return bufs

    def reduce_scatter_sum(self, t, out):
        out.copy_(t[: out.numel()])
        return out

    def all_gather_into(self, buf, chunk: int):
        return buf

    def exchange_chunks(self, t, chunk: int, bufs):
        assert not bufs
        return bufs

    def gather_async(self, t, bufs):
        assert not bufs
        return _Works([])

    def isend(self, t, dst):
        raise RuntimeError("LocalTransport has no peers")

    irecv = isend

    def barrier(self):
        pass

    def all_gather_object(self, obj):
        return [obj]

    def broadcast_object(self, obj):
        return obj

    def close(self):
        pass


class _Works:
    """Several point-to-point works as one (wait = all)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True

    def is_completed(self) -> bool:
        return all(w.is_completed() for w in self.works)


class DistTransport:
    is_distributed = True

    def __init__(self, backend: str | None = None, device=None, timeout_s: float = 600.0):
        if not dist.is_initialized():
            if backend is None:
                # PSX_DIST_BACKEND=gloo: the torch group on gloo even with GPUs (several ranks
                # sharing one GPU in tests, where RCCL would refuse the duplicate device)
                backend = os.environ.get("PSX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = torch.device(device)
            attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
            if os.environ.get("WORLD_SIZE", "1") == "1" and os.environ.get("PSX_WORLD1_TCP") != "1":
                # a world of one rank needs no rendezvous: an in-process store, so no TCP port can
                # collide with another process on the box (EADDRINUSE seen once on a GPU box)
                kw.update(store=dist.HashStore(), rank=0, world_size=1)
            elif attempt and os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True":
                # restarted group on the agent's long-lived store (static rendezvous): namespace
                # this attempt's keys, or ranks would read the dead attempt's peer addresses
                base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                                     int(os.environ["WORLD_SIZE"]), is_master=False,
                                     timeout=datetime.timedelta(seconds=timeout_s))
                kw.update(store=dist.PrefixStore(f"psx/attempt{attempt}", base), rank=int(os.environ["RANK"]),
                          world_size=int(os.environ["WORLD_SIZE"]))
            dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
        self.backend = dist.get_backend()
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        # host-side control collectives always go through gloo
        self.ctrl = dist.new_group(backend="gloo") if self.backend != "gloo" else dist.group.WORLD

    # ---- sync mode collectives (bulk, device tensors)
    def reduce_sum_to_server(self, t):
        dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        return t

    def broadcast_from_server(self, t):
        dist.broadcast(t, src=0)
        return t

    def reduce_scatter_sum(self, t, out):
        """Sharded server push: out = sum over ranks of this rank's slice of t (t.numel() ==
        world * out.numel()). gloo has no reduce-scatter: all-reduce + slice there."""
        if self.backend == "gloo":
            tmp = t.clone()
            dist.all_reduce(tmp, op=dist.ReduceOp.SUM)
            out.copy_(tmp[self.rank * out.numel():(self.rank + 1) * out.numel()])
            return out
        dist.reduce_scatter_tensor(out, t, op=dist.ReduceOp.SUM)
        return out

    def all_gather_into(self, buf, chunk: int):
        """Sharded server fetch: buf[r*chunk:(r+1)*chunk] of rank r reaches every rank, in place."""
        if buf.element_size() == 2:  # a pure copy: move the bits as int32 pairs (gloo has no 16-bit ints)
            assert chunk % 2 == 0 and buf.numel() % 2 == 0
            buf, chunk = buf.view(torch.int32), chunk // 2
        mine = buf[self.rank * chunk:(self.rank + 1) * chunk]
        if self.backend == "gloo":
            parts = list(buf[: chunk * self.world_size].split(chunk))
            dist.all_gather(parts, mine.clone())
            return buf
        dist.all_gather_into_tensor(buf[: chunk * self.world_size], mine)
        return buf

    def exchange_chunks(self, t, chunk: int, bufs):
        """All-to-all of equal chunks: rank r sends t[p*chunk:(p+1)*chunk] to every rank p != r
        and receives rank p's chunk r into bufs[p] (sharded server push)."""
        r = self.rank
        works = []
        for p in range(self.world_size):
            if p == r:
                continue
            if p < r:  # deterministic pairing order on both ends
                works.append(dist.irecv(bufs[p], src=p))
                works.append(dist.isend(t[p * chunk:(p + 1) * chunk].contiguous(), dst=p))
            else:
                works.append(dist.isend(t[p * chunk:(p + 1) * chunk].contiguous(), dst=p))
                works.append(dist.irecv(bufs[p], src=p))
        for w in works:
            w.wait()
        return bufs

    def gather_to_server(self, t):
        """Equal-size tensors of every rank -> list on rank 0 (RCCL gather: point-to-point
        sends into rank 0; used for top-k payloads, which cannot be reduced)."""
        if self.rank == 0:
            out = [t] + [torch.empty_like(t) for _ in range(self.world_size - 1)]
            dist.gather(t, gather_list=out, dst=0)
            return out
        dist.gather(t, gather_list=None, dst=0)
        return None

    def gather_from_workers(self, t, bufs):
        """Sync push with fp32 aggregation on the server: rank r > 0 sends its wire ``t`` to rank
        0, which receives it into ``bufs[r]`` (preallocated, one per remote rank) — point-to-point
        transfers that all run at once (each worker on its own xGMI link). Rank 0's own wire
        stays where it is. The server then sums the wires in fp32 (kernels.sgd_apply_multi)."""
        if self.rank == 0:
            works = [dist.irecv(b, src=r) for r, b in sorted(bufs.items())]
            for w in works:
                w.wait()
            return bufs
        dist.send(t, dst=0)
        return None

    # ---- bucketed (overlapped) sync round: non-blocking; RCCL runs on its own stream ordered
    # after the caller's stream at issue time, work.wait() orders the caller's stream after it
    def gather_async(self, t, bufs):
        """Non-blocking gather_from_workers (one bucket of the overlapped round)."""
        if self.rank == 0:
            return _Works([dist.irecv(b, src=r) for r, b in sorted(bufs.items())])
        return _Works([dist.isend(t, dst=0)])

    def reduce_async(self, t):
        return dist.reduce(t, dst=0, op=dist.ReduceOp.SUM, async_op=True)

    def broadcast_async(self, t):
        return dist.broadcast(t, src=0, async_op=True)

    # ---- async mode point-to-point (bulk)
    def isend(self, t, dst: int):
        return dist.isend(t, dst=dst)

    def irecv(self, t, src: int):
        return dist.irecv(t, src=src)

    def completed(self, work) -> bool:
        """Non-blocking completion test of a p2p work. RCCL works are polled through their HIP
        event; gloo works only complete inside wait(), so they are waited for (the payload is
        already in flight when the server polls, see ParameterServer.serve_async)."""
        if self.backend == "gloo":
            work.wait()
            return True
        if work.is_completed():
            work.wait()  # orders the caller's stream after the RCCL stream (no host block)
            return True
        return False

    # ---- degraded mode: the job goes on without ranks the async server dropped
    degraded = ()

    def degrade(self, dead, tag: str):
        """Ranks ``dead`` (async workers the server dropped: crashed, hung) will never join another
        collective: from here on the host control operations run among the live ranks on the
        rendezvous store (a gloo / RCCL collective would wait for the dead ranks forever), and
        close() aborts communicators instead of destroying them."""
        self.degraded = tuple(sorted(set(int(r) for r in dead)))
        self._dtag, self._dseq = tag, 0

    def _live(self):
        return [r for r in range(self.world_size) if r not in self.degraded]

    @staticmethod
    def _store():
        from torch.distributed import distributed_c10d as c10d

        return c10d._get_default_store()

    def _dkey(self, what: str) -> str:
        self._dseq += 1
        return f"psx/{self._dtag}/{what}{self._dseq}"

    def _store_gather(self, obj):
        from . import objwire

        key, st = self._dkey("obj"), self._store()
        st.set(f"{key}/{self.rank}", objwire.dumps(obj))
        if self.rank in self.degraded:
            return [obj if r == self.rank else None for r in range(self.world_size)]
        live = self._live()
        st.wait([f"{key}/{r}" for r in live])
        return [objwire.loads(st.get(f"{key}/{r}")) if r in live else None for r in range(self.world_size)]

    # ---- host control
    def barrier(self):
        if self.degraded:
            self._store_gather(None)  # every live rank's key present = everyone arrived
            return
        dist.barrier(group=self.ctrl)

    def all_gather_object(self, obj):
        if self.degraded:
            return self._store_gather(obj)
        from . import objwire  # JSON, never pickle (objwire.py)

        return objwire.all_gather(obj, self.ctrl, self.world_size)

    def broadcast_object(self, obj):
        if self.degraded:
            return self._store_gather(obj if self.rank == 0 else None)[0]
        from . import objwire

        return objwire.broadcast(obj, self.ctrl, src=0, rank=self.rank)

    def close(self):
        if dist.is_initialized():
            if self.degraded:
                # the store lives in rank 0's process: rank 0 leaves last (the others only check in)
                key, st = self._dkey("close"), self._store()
                try:
                    st.set(f"{key}/{self.rank}", b"1")
                    if self.rank == 0:
                        st.wait([f"{key}/{r}" for r in self._live() if r != 0])
                except Exception:
                    pass
            else:
                try:
                    dist.barrier(group=self.ctrl)
                except Exception:
                    pass
            dist.destroy_process_group()


def env_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torchrun-style environment (defaults: single process)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local
