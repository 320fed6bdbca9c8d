"""Async parameter server on the native event loop (csrc/server/event_loop.cpp).

The async server role of rank 0 — mailbox control, RCCL point-to-point receive of pushed
gradients and send of fetch snapshots, staleness decisions, the fused SGD apply, heartbeat
timeouts, checkpoint triggers — runs in one C++ thread on HIP streams (one communication stream
and one 2-rank communicator per worker, one update stream); see the C++ file for the ordering
rules. Python only starts it, serves the co-located worker's calls through it, writes the
checkpoints it asks for, and joins it. It is THE async server of MI355X jobs on the native
transport (PSX_NATIVE_LOOP=0 selects ParameterServer.serve_async, the Python loop, which stays
the CPU/gloo path and serves the configurations below).

Remote workers use ``NativeAsyncChannel``: control requests on the shared-memory mailbox as
before, tensors by ncclSend/ncclRecv on their pair communicator (parallel/rccl.py open_pairs),
posted on a communication stream ordered after the worker's compute stream by events.

Scope: dense fp16/fp32 gradients; SGD with the server's momentum / weight decay; fetch payload
bf16conv or fp32; checkpoints. Not covered (Python loop): top-k payloads, --bn-sync.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from .. import NATIVE_DIR
from ..ops._lib import comm, kernels, runtime
from . import control as CP
from .codec import small_index_of
from .worker import AsyncChannel

vp, i32, i64, f32, f64 = C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_double


CKPT_CB = C.CFUNCTYPE(i32, C.c_longlong)


class LoopCfg(C.Structure):
    """csrc/server/event_loop.cpp PsxLoopCfg."""
    _fields_ = [("mbox", vp), ("core", vp), ("comms", vp), ("comm_peer", vp), ("arena", vp), ("small_idx", vp),
                ("remote_rank", vp), ("n_params", i64), ("small_n", i64), ("arena_numel", i64), ("lr", f32),
                ("momentum", f32), ("weight_decay", f32), ("device", i32), ("grad_fp16", i32), ("max_wid", i32),
                ("expected", i32), ("fetch_fp32", i32), ("mom_first", i32), ("mom_buf", vp),
                ("heartbeat_timeout", f64), ("poll_s", f64), ("upd_stream", vp), ("own_upd_stream", i32),
                ("ckpt_every", C.c_longlong), ("ckpt_cb", CKPT_CB), ("comm_owned", vp), ("transfer_timeout", f64),
                ("stall_timeout", f64)]


_SIGS = {
    "psx_loop_cfg_size": (i32, []),
    "psx_loop_create": (vp, [C.POINTER(LoopCfg), C.c_char_p, C.c_char_p]),
    "psx_loop_start": (i32, [vp]),
    "psx_loop_join": (i32, [vp]),
    "psx_loop_applies": (C.c_longlong, [vp]),
    "psx_loop_dropped": (i32, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), i32]),
    "psx_loop_local_push": (i32, [vp, i32, vp, C.c_longlong, vp, C.POINTER(C.c_longlong)]),
    "psx_loop_local_fetch": (C.c_longlong, [vp, i32, vp, vp]),
    "psx_loop_local_done": (i32, [vp, i32]),
    "psx_loop_destroy": (None, [vp]),
}


def _lib():
    lib = comm()
    if not getattr(lib, "_psx_loop_declared", False):
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        lib._psx_loop_declared = True
        if lib.psx_loop_cfg_size() != C.sizeof(LoopCfg):
            raise RuntimeError("PsxLoopCfg layout mismatch between csrc/server/event_loop.cpp and native_loop.py")
    return lib


def native_loop_enabled(cfg, transport) -> bool:
    """Default for async jobs on the native transport (PSX_NATIVE_LOOP=0: the Python loop)."""
    return (os.environ.get("PSX_NATIVE_LOOP", "1") == "1" and getattr(transport, "native", False)
            and cfg.codec in ("fp16", "none") and not cfg.bn_sync)


class NativeServerLoop:
    """Rank 0: the server event loop thread (C++)."""

    def __init__(self, server, transport, mbox, rank_of_wid: dict, expected: int, poll_s: float = 0.0005,
                 update_stream: torch.cuda.Stream | None = None):
        """rank_of_wid: worker id -> transport rank of the remote workers (transport None: local
        workers only). update_stream: the co-located worker's compute stream (its pushes/fetches
        are then in plain stream order with the loop's updates); None = the loop creates its own."""
        self.server = server
        self.t = transport
        self.rank_of_wid = dict(rank_of_wid)
        lay = server.layout
        cfg = server.cfg
        self.small_idx = small_index_of(lay).to(server.device)
        max_wid = max([expected] + [w + 1 for w in rank_of_wid])
        self.max_wid = max_wid
        self.remote = (C.c_int * max_wid)(*([-1] * max_wid))
        self.comms = (vp * max_wid)()
        self.peer = (C.c_int * max_wid)(*([-1] * max_wid))
        # 1: the worker's communicator is its own 2-rank pair (abortable when it is dropped);
        # 0: a shared one (PSX_PAIR_COMMS=0), never aborted by the loop
        self.owned = (C.c_int * max_wid)(*([0] * max_wid))
        pairs = getattr(transport, "_pairs", {}) if transport is not None else {}
        for w, r in rank_of_wid.items():
            self.remote[w] = r
            c, p = transport.p2p(r)  # the worker's pair communicator (parallel/rccl.py open_pairs)
            self.comms[w], self.peer[w] = c.h.value, p
            self.owned[w] = int(r in pairs)
        self.dropped = []          # [(worker id, pair communicator aborted)] after join
        self.dropped_ranks = []
        dev = server.device.index or 0
        mom = server.momentum_buf if cfg.momentum else None
        self._ckpt = CKPT_CB(self._checkpoint)  # kept alive with the loop
        self.cfg = LoopCfg(mbox=mbox._h if mbox is not None else None, core=server.core._h,
                           comms=C.cast(self.comms, vp), comm_peer=C.cast(self.peer, vp),
                           arena=server.arena.data_ptr(), small_idx=self.small_idx.data_ptr(),
                           remote_rank=C.cast(self.remote, vp), n_params=lay.param_numel,
                           small_n=self.small_idx.numel(), arena_numel=lay.arena_numel, lr=float(server.lr),
                           momentum=float(cfg.momentum or 0.0), weight_decay=float(cfg.weight_decay or 0.0),
                           device=dev, grad_fp16=int(cfg.codec == "fp16"), max_wid=max_wid, expected=expected,
                           fetch_fp32=int(cfg.fetch_codec == "fp32"), mom_first=int(server._mom_first),
                           mom_buf=mom.data_ptr() if mom is not None else None,
                           heartbeat_timeout=float(cfg.heartbeat_timeout or 0.0), poll_s=poll_s,
                           upd_stream=update_stream.cuda_stream if update_stream is not None else None,
                           own_upd_stream=int(update_stream is None),
                           ckpt_every=int(cfg.ckpt_every or 0) if cfg.ckpt_dir else 0, ckpt_cb=self._ckpt,
                           comm_owned=C.cast(self.owned, vp), transfer_timeout=float(cfg.transfer_timeout or 0.0),
                           stall_timeout=float(cfg.stall_timeout or 0.0))
        kernels()  # both libraries are loaded (the loop binds their entry points by path)
        runtime()
        self.h = _lib().psx_loop_create(C.byref(self.cfg), os.path.join(NATIVE_DIR, "libpsx_runtime.so").encode(),
                                        os.path.join(NATIVE_DIR, "libpsx_kernels.so").encode())
        if not self.h:
            raise RuntimeError("psx_loop_create failed")
        torch.cuda.synchronize(server.device)  # the arena is final before the loop reads it
        _lib().psx_loop_start(self.h)

    def _checkpoint(self, global_step: int) -> int:
        """Called on the loop thread once the update stream has finished the apply that reached
        ``global_step`` (a multiple of --ckpt-every)."""
        try:
            with torch.cuda.device(self.server.device):
                self.server.maybe_checkpoint()
            return 0
        except Exception as e:  # noqa: BLE001 - reported, the loop ends with an error
            import sys

            print(f"[psx native loop] checkpoint at step {global_step} failed: {e}", file=sys.stderr, flush=True)
            return 1

    def join(self):
        if self.h is None:
            return 0
        rc = _lib().psx_loop_join(self.h)
        ids, ab = (C.c_int * self.max_wid)(), (C.c_int * self.max_wid)()
        n = _lib().psx_loop_dropped(self.h, ids, ab, self.max_wid)
        self.dropped = [(int(ids[i]), bool(ab[i])) for i in range(min(n, self.max_wid))]
        for w, aborted in self.dropped:
            r = self.rank_of_wid.get(w)
            if r is None:
                continue
            self.dropped_ranks.append(r)
            if aborted:  # ncclCommAbort freed it: the transport must not destroy it again
                self.t.p2p(r)[0].h = None
        self.server.dropped_workers = sorted(w for w, _ in self.dropped)
        s = self.server
        applies = int(_lib().psx_loop_applies(self.h))
        s._mom_first = s._mom_first and not applies
        if applies:  # the loop fed each apply's device time to the core (event_loop.cpp read_timings)
            s.update_time_source = "device events around the apply kernels (native loop)"
        s.bytes_pushed = int(s.core.metrics().get("gradients_processed", 0)) * s.n * (2 if s.cfg.codec == "fp16" else 4)
        _lib().psx_loop_destroy(self.h)
        self.h = None
        if rc:
            raise RuntimeError(f"native server loop ended with error {rc}")
        return rc


class NativeLocalChannel:
    """Rank 0's co-located worker: requests served by the loop thread, in stream order."""

    def __init__(self, server, loop: NativeServerLoop):
        self.server, self.loop = server, loop

    def register(self, name, requested_id=-1):
        return self.server.register_worker(name, requested_id)

    def fetch(self, worker_id, local_arena):
        gs = _lib().psx_loop_local_fetch(self.loop.h, worker_id, local_arena.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
        if gs < 0:
            raise RuntimeError(f"native local fetch failed ({gs})")
        return gs

    def push(self, worker_id, grads, local_step, buffers=None):
        out = (C.c_longlong * 3)()
        rc = _lib().psx_loop_local_push(self.loop.h, worker_id, grads.data_ptr(), int(local_step),
                                        torch.cuda.current_stream().cuda_stream, out)
        if rc:
            raise RuntimeError(f"native local push failed ({rc})")
        self.last_staleness = int(out[1])
        return bool(out[0])

    def finished(self, worker_id):
        _lib().psx_loop_local_done(self.loop.h, worker_id)


class NativeAsyncChannel(AsyncChannel):
    """Remote worker: mailbox control, tensors over the native communicator (rank 0 = server)."""

    def __init__(self, transport, mbox, rank, codec):
        super().__init__(transport, mbox, rank, codec=codec)
        self.cs = torch.cuda.Stream(device=transport.device)
        self.comm, self.server_peer = transport.p2p(0)  # the pair communicator with the server

    def _fork(self):
        self.cs.wait_stream(torch.cuda.current_stream())
        return torch.cuda.stream(self.cs)

    crash_in_push = False  # --fault-inject crash_in_push (Worker.run_training)

    def _dropped(self, r):
        """R_DROPPED: the server no longer serves this worker. The transfer this call posted has
        no partner any more: abort the pair communicator (that is what ends a posted RCCL kernel)
        and end the training loop."""
        if r.type != CP.R_DROPPED:
            return
        pairs = getattr(self.t, "_pairs", {})
        if 0 in pairs and self.comm.h:
            self.comm.destroy(abort=True)
        raise CP.WorkerDropped(f"worker rank {self.rank}: dropped by the parameter server")

    def fetch(self, worker_id, local_arena):
        self.mbox.send(CP.Msg(CP.FETCH, self.rank, worker_id))
        with self._fork():
            for b in self.codec.wire:  # bf16 image + fp32 remainder, or the fp32 arena (server send order)
                self.comm.recv(b, self.server_peer, stream=self.cs)
        r = self.mbox.wait_reply(self.rank)
        self._dropped(r)
        torch.cuda.current_stream().wait_stream(self.cs)
        self.codec.unpack(local_arena)
        return r.c

    def push(self, worker_id, grads, local_step, buffers=None):
        if buffers is not None:
            raise RuntimeError("the native server loop does not take BN buffers (--bn-sync)")
        self.mbox.send(CP.Msg(CP.PUSH, self.rank, worker_id, 0, local_step))
        if self.crash_in_push:  # the server has posted its receive; this process dies before sending
            import sys

            print(f"fault injected: worker rank {self.rank} crashes inside a push", file=sys.stderr, flush=True)
            os._exit(17)
        with self._fork():
            self.comm.send(grads, self.server_peer, stream=self.cs)
        r = self.mbox.wait_reply(self.rank)
        self._dropped(r)
        torch.cuda.current_stream().wait_stream(self.cs)  # the gradient buffer is reusable
        self.last_staleness = r.d
        return bool(r.b)

