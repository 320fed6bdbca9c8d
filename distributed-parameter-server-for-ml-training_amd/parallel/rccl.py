"""Native RCCL transport: every bulk tensor of the PS protocol on psx's own communicators.

``RcclTransport`` keeps DistTransport's torch.distributed group for host control only (gloo:
registration names, barriers, metrics, the unique ids) and moves every bulk tensor through
psx's RCCL communicators (csrc/comm/rccl_comm.cpp):

  reference RPC (src/communication/ps.proto:4-19)   here
  PushGradrients (sync)   pickled fp16 dict         grouped ncclSend/ncclRecv gather of the wires
                                                    to rank 0 (fp32 sum there), or ncclReduce
  FetchParameters (sync)  pickled fp32 state_dict   ncclBroadcast(rank 0) of the weight wire
  (top-k payloads)        -                         grouped ncclSend/ncclRecv gather to rank 0
  PushGradrients (async)  pickled fp16 dict         ncclSend worker -> server on the pair's
  FetchParameters (async) pickled fp32 state_dict   communicator / ncclSend server -> worker

Async point-to-point runs on one 2-rank communicator per (server, worker) pair (``open_pairs``)
with its own HIP stream on each side, so the transfers of different workers never queue behind
each other: with 7 workers the server's 7 xGMI links carry 7 pushes at once (the reference's
20-thread gRPC pool, server.py:380-383, serves concurrent RPCs).

Each collective is enqueued on the caller's current HIP stream — the worker's compute stream —
so a round needs no cross-stream event and no host wait (torch.distributed runs RCCL on an
internal stream and joins it with events on every call). The bucketed overlap channel still gets
non-blocking collectives: they run on one communication stream that first waits on the compute
stream, and return a ``NativeWork`` whose ``wait()`` joins the caller's stream to it.

Bootstrap: rank 0 draws the RCCL unique id, the gloo control group broadcasts it, every rank
calls ncclCommInitRank on its own GPU. The library RCCL is bound to is the one PyTorch loaded
(torch/lib/librccl.so), so the process runs one RCCL instance.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from ..ops._lib import comm
from .transport import DistTransport

DTYPES = {torch.uint8: (0, 1), torch.float16: (1, 2), torch.float32: (2, 4), torch.bfloat16: (3, 2),
          torch.int32: (4, 4)}


class RcclError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc != 0:
        msg = comm().psx_comm_error_string(rc)
        raise RcclError(f"{what}: RCCL error {rc} ({msg.decode() if msg else '?'})")


def torch_rccl_path() -> str:
    """librccl.so of the PyTorch build in use (bundled in torch/lib), else ROCm's
    (PSX_RCCL_LIB overrides)."""
    if os.environ.get("PSX_RCCL_LIB"):
        return os.environ["PSX_RCCL_LIB"]
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if os.path.exists(p):
        return p
    return "/opt/rocm/lib/librccl.so"


def _dt(t: torch.Tensor):
    try:
        return DTYPES[t.dtype]
    except KeyError:
        raise RcclError(f"dtype {t.dtype} not supported by the native transport") from None


def _stream(s=None) -> int:
    return (s if s is not None else torch.cuda.current_stream()).cuda_stream


class NativeComm:
    """One RCCL communicator over all ranks of the job (C handle + the device it lives on)."""

    def __init__(self, rank: int, world: int, device: torch.device, broadcast_object, all_gather_object=None):
        # every rank loads the library (and rank 0 draws the id) BEFORE anyone enters the
        # collective ncclCommInitRank: with all_gather_object the ranks agree first, so a rank
        # that cannot bind RCCL fails the job everywhere instead of leaving the others blocked
        uid, err = None, ""
        try:
            lib = comm()
            _check(lib.psx_comm_load(torch_rccl_path().encode()), "psx_comm_load")
            if rank == 0:
                buf = C.create_string_buffer(lib.psx_comm_id_bytes())
                _check(lib.psx_comm_unique_id(buf), "ncclGetUniqueId")
                uid = buf.raw
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = f"rank {rank}: {e}"
        if all_gather_object is not None:
            errs = [x for x in all_gather_object(err) if x]
            if errs:
                raise RcclError("native communicator unavailable: " + "; ".join(errs))
        elif err:
            raise RcclError(err)
        uid = broadcast_object(uid)
        self._init(uid, world, rank, device)

    def _init(self, uid: bytes, world: int, rank: int, device):
        h = C.c_void_p()
        self.device = torch.device(device)
        _check(comm().psx_comm_init(uid, world, rank, self.device.index or 0, C.byref(h)), "ncclCommInitRank")
        self.h = h
        self.rank, self.world = rank, world
        # in-place reduce / all-reduce / broadcast over one rank are identities: skipped (RCCL
        # still moved the 45 MB fetch and the 22 MB wire through a self-copy each, ~28 us per
        # N = 1 step). PSX_COMM_SELF=1 issues them anyway (tests of the RCCL call path).
        self.identity = world == 1 and os.environ.get("PSX_COMM_SELF", "0") != "1"

    @classmethod
    def from_id(cls, uid: bytes, world: int, rank: int, device) -> "NativeComm":
        """A communicator over an id drawn by ``new_id`` (library already loaded)."""
        c = cls.__new__(cls)
        c._init(uid, world, rank, device)
        return c

    @staticmethod
    def new_id() -> bytes:
        lib = comm()
        buf = C.create_string_buffer(lib.psx_comm_id_bytes())
        _check(lib.psx_comm_unique_id(buf), "ncclGetUniqueId")
        return buf.raw

    def reduce_sum(self, t: torch.Tensor, root: int = 0, stream=None):
        if self.identity:
            return
        code, _ = _dt(t)
        _check(comm().psx_comm_reduce_sum(self.h, t.data_ptr(), t.data_ptr(), t.numel(), code, root, _stream(stream)),
               "ncclReduce")

    def all_reduce_sum(self, t: torch.Tensor, stream=None):
        if self.identity:
            return
        code, _ = _dt(t)
        _check(comm().psx_comm_all_reduce_sum(self.h, t.data_ptr(), t.data_ptr(), t.numel(), code, _stream(stream)),
               "ncclAllReduce")

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None):
        if self.identity:
            return
        code, _ = _dt(t)
        _check(comm().psx_comm_broadcast(self.h, t.data_ptr(), t.numel(), code, root, _stream(stream)), "ncclBroadcast")

    def reduce_scatter_sum(self, t: torch.Tensor, out: torch.Tensor, stream=None):
        """out (numel/world) = sum over ranks of this rank's slice of t (out may be that slice)."""
        code, _ = _dt(t)
        assert t.numel() == out.numel() * self.world and t.dtype == out.dtype
        _check(comm().psx_comm_reduce_scatter_sum(self.h, t.data_ptr(), out.data_ptr(), out.numel(), code,
                                                  _stream(stream)), "ncclReduceScatter")

    def all_gather(self, t: torch.Tensor, out: torch.Tensor, stream=None):
        """out[r*numel:(r+1)*numel] = rank r's t on every rank (t may be this rank's slice of out)."""
        code, _ = _dt(t)
        assert out.numel() == t.numel() * self.world and t.dtype == out.dtype
        _check(comm().psx_comm_all_gather(self.h, t.data_ptr(), out.data_ptr(), t.numel(), code, _stream(stream)),
               "ncclAllGather")

    def gather(self, t: torch.Tensor, out: torch.Tensor | None, root: int = 0, stream=None):
        """Equal-size tensors of every rank -> ``out`` ([world * numel], root only)."""
        code, esz = _dt(t)
        _check(comm().psx_comm_gather(self.h, t.data_ptr(), out.data_ptr() if out is not None else None, t.numel(),
                                      code, esz, root, self.rank, self.world, _stream(stream)), "gather")

    def send(self, t: torch.Tensor, peer: int, stream=None):
        code, _ = _dt(t)
        _check(comm().psx_comm_send(self.h, t.data_ptr(), t.numel(), code, peer, _stream(stream)), "ncclSend")

    def recv(self, t: torch.Tensor, peer: int, stream=None):
        code, _ = _dt(t)
        _check(comm().psx_comm_recv(self.h, t.data_ptr(), t.numel(), code, peer, _stream(stream)), "ncclRecv")

    def async_error(self) -> int:
        return comm().psx_comm_async_error(self.h) if self.h else 0

    def count(self) -> int:
        """Ranks of the communicator as RCCL reports them (ncclCommCount); -1 if unavailable."""
        n = C.c_int(-1)
        if not self.h or comm().psx_comm_count(self.h, C.byref(n)) != 0:
            return -1
        return int(n.value)

    def destroy(self, abort: bool = False):
        if self.h:
            (comm().psx_comm_abort if abort else comm().psx_comm_destroy)(self.h)
            self.h = None


class NativeWork:
    """Completion of an operation issued on the communication stream (torch Work look-alike)."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        return True

    def is_completed(self) -> bool:
        return self.event.query()


class RcclTransport(DistTransport):
    """DistTransport whose sync-round bulk tensors go through the native communicator."""

    native = True

    def __init__(self, backend: str | None = None, device=None, timeout_s: float = 600.0):
        super().__init__(backend=backend, device=device, timeout_s=timeout_s)
        if self.device.type != "cuda":
            raise RcclError("RcclTransport needs a HIP device")
        self.comm = NativeComm(self.rank, self.world_size, self.device, self.broadcast_object,
                               self.all_gather_object)
        self._cstream = torch.cuda.Stream(device=self.device)
        self._pairs = {}    # peer rank -> (communicator, peer's rank in it)
        self._pstream = {}  # peer rank -> HIP stream of the async point-to-point with that peer

    # ---- async mode point-to-point: one communicator + stream per (server, worker) pair
    def open_pairs(self, peers=None):
        """Collective over all ranks: a 2-rank communicator {0, r} for every rank r in ``peers``
        (default: every rank > 0). Rank 0 draws the ids; the ranks initialise in rank order on
        rank 0 (each worker only waits for its own pair). PSX_PAIR_COMMS=0 keeps everything on
        the job communicator. World 2 gets its own pair as well: the async server aborts a dropped
        worker's pair communicator, which must never be the job communicator."""
        peers = sorted(peers) if peers is not None else list(range(1, self.world_size))
        if os.environ.get("PSX_PAIR_COMMS", "1") == "0" or self.world_size < 2:
            return
        ids = self.broadcast_object({r: NativeComm.new_id() for r in peers} if self.rank == 0 else None)
        if self.rank == 0:
            for r in peers:
                self._pairs[r] = (NativeComm.from_id(ids[r], 2, 0, self.device), 1)
        elif self.rank in ids:
            self._pairs[0] = (NativeComm.from_id(ids[self.rank], 2, 1, self.device), 0)

    def p2p(self, peer: int):
        """(communicator, peer rank in it) carrying this rank's point-to-point with ``peer``."""
        return self._pairs.get(peer, (self.comm, peer))

    def _p2p_stream(self, peer: int):
        s = self._pstream.get(peer)
        if s is None:
            s = self._pstream[peer] = torch.cuda.Stream(device=self.device)
        return s

    def _p2p(self, t, peer: int, send: bool):
        c, p = self.p2p(peer)
        s = self._p2p_stream(peer)
        s.wait_stream(torch.cuda.current_stream())
        (c.send if send else c.recv)(t, p, stream=s)
        ev = torch.cuda.Event()
        ev.record(s)
        t.record_stream(s)
        return NativeWork(ev)

    def isend(self, t, dst: int):
        """Non-blocking send on the pair's stream; ``completed`` / ``wait()`` joins the caller's
        stream to it (the tensor must stay unmodified until then)."""
        return self._p2p(t, dst, True)

    def irecv(self, t, src: int):
        return self._p2p(t, src, False)

    # ---- sync mode collectives: in stream order on the caller's stream
    def reduce_sum_to_server(self, t):
        self.comm.reduce_sum(t, 0)
        return t

    def broadcast_from_server(self, t):
        self.comm.broadcast(t, 0)
        return t

    def gather_to_server(self, t):
        if self.rank == 0:
            flat = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
            self.comm.gather(t, flat, 0)
            return list(flat.view(self.world_size, t.numel()).unbind(0))
        self.comm.gather(t, None, 0)
        return None

    def gather_from_workers(self, t, bufs):
        """DistTransport.gather_from_workers on the native communicator: one group of
        ncclRecv (rank 0, one per remote rank, concurrent over the xGMI links) / one ncclSend
        (workers), in stream order on the caller's stream."""
        lib = comm()
        if self.rank == 0:
            _check(lib.psx_comm_group_start(), "ncclGroupStart")
            try:
                for r, b in sorted(bufs.items()):
                    self.comm.recv(b, r)
            finally:
                _check(lib.psx_comm_group_end(), "ncclGroupEnd")
            return bufs
        self.comm.send(t, 0)
        return None

    # ---- sharded server (parallel/sharded.py)
    def exchange_chunks(self, t, chunk: int, bufs):
        """All-to-all of the wire chunks in one group of ncclSend/ncclRecv (every link busy at
        once), on the caller's stream."""
        lib = comm()
        _check(lib.psx_comm_group_start(), "ncclGroupStart")
        try:
            for p in range(self.world_size):
                if p != self.rank:
                    self.comm.send(t[p * chunk:(p + 1) * chunk], p)
                    self.comm.recv(bufs[p], p)
        finally:
            _check(lib.psx_comm_group_end(), "ncclGroupEnd")
        return bufs

    def reduce_scatter_sum(self, t, out):
        self.comm.reduce_scatter_sum(t, out)
        return out

    def all_gather_into(self, buf, chunk: int):
        self.comm.all_gather(buf[self.rank * chunk:(self.rank + 1) * chunk], buf[: chunk * self.world_size])
        return buf

    # ---- bucketed (overlapped) round: non-blocking on the communication stream
    def _on_comm_stream(self, fn):
        cur = torch.cuda.current_stream()
        self._cstream.wait_stream(cur)
        with torch.cuda.stream(self._cstream):
            fn(self._cstream)
            ev = torch.cuda.Event()
            ev.record(self._cstream)
        return NativeWork(ev)

    def reduce_async(self, t):
        return self._on_comm_stream(lambda s: self.comm.reduce_sum(t, 0, stream=s))

    def gather_async(self, t, bufs):
        """gather_from_workers on the communication stream (one bucket of the overlapped round):
        one group of ncclRecv on rank 0 (every worker's link at once) / one ncclSend."""
        def fn(s):
            lib = comm()
            if self.rank != 0:
                self.comm.send(t, 0, stream=s)
                return
            _check(lib.psx_comm_group_start(), "ncclGroupStart")
            try:
                for r, b in sorted(bufs.items()):
                    self.comm.recv(b, r, stream=s)
            finally:
                _check(lib.psx_comm_group_end(), "ncclGroupEnd")

        return self._on_comm_stream(fn)

    def broadcast_async(self, t):
        return self._on_comm_stream(lambda s: self.comm.broadcast(t, 0, stream=s))

    def completed(self, work) -> bool:
        if isinstance(work, NativeWork):
            if work.is_completed():
                work.wait()
                return True
            return False
        return super().completed(work)

    def close(self):
        """With dead ranks (``degraded``) their pair communicators and the job communicator are
        aborted, not destroyed: a destroy waits for peers that will never come."""
        try:
            torch.cuda.synchronize(self.device)
        finally:
            dead = set(self.degraded)
            for peer, (c, _) in self._pairs.items():
                c.destroy(abort=peer in dead or (self.rank in dead))
            self._pairs = {}
            self.comm.destroy(abort=bool(dead))
            super().close()


def make_transport(device=None):
    """RcclTransport on MI355X (PSX_TRANSPORT=native, the default), torch.distributed otherwise
    (PSX_TRANSPORT=torch, or no GPU: the gloo CPU path)."""
    dev = torch.device(device) if device is not None else None
    kind = os.environ.get("PSX_TRANSPORT", "native")
    if kind == "native" and dev is not None and dev.type == "cuda":
        try:
            return RcclTransport(device=dev)
        except RcclError as e:
            # every rank raised the same collective verdict (NativeComm): all fall back together
            import sys

            print(f"[psx] {e}; falling back to torch.distributed (PSX_TRANSPORT=torch)", file=sys.stderr)
            if torch.distributed.is_initialized():
                return DistTransport(device=device)  # reuses the initialised default group
            raise
    return DistTransport(device=device)
