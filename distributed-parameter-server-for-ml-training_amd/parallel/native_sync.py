"""Sync rounds of the dedicated server rank in native code (csrc/server/sync_loop.cpp).

Rank 0 of the reference's 1 server + N-1 workers layout has no training of its own: every round
it broadcasts the state, receives the workers' gradients, averages them in fp32 and applies SGD
(reference: src/parameter_server/server.py:264-288 sync handler, :145-169 averaging, :126-143
apply, :213-230 fetch). ``NativeSyncServer.run(rounds)`` executes ALL of the job's rounds in one
native call on the server's HIP streams — the collective sequence of the workers' sync channel
(serial round: parallel/worker.py SyncCollectiveChannel; overlapped round:
parallel/overlap.py OverlapSyncChannel), the fused fp32 aggregation + SGD kernel
(``psx_sgd_apply_multi``), the native core's barrier bookkeeping and the checkpoint hook — so
no Python runs per round on the server. The liveness watchdog (parallel/liveness.py) follows
the rounds' device completion through ``psx_sync_progress``.

Scope (otherwise the Python channel runs the server side, PSX_NATIVE_SYNC=0 forces it): sync
mode, dedicated topology on the native transport, dense fp16 / fp32 gradient wire, fetch payload
fp32 or bf16conv (WeightWire / BucketWire), no --bn-sync.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from .. import NATIVE_DIR
from ..ops._lib import comm, kernels, runtime

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_long, C.c_float
CKPT_CB = C.CFUNCTYPE(i32, C.c_longlong)


class SyncBucket(C.Structure):
    """csrc/server/sync_loop.cpp PsxSyncBucket."""
    _fields_ = [("lo", i64), ("hi", i64), ("seg", vp), ("seg_bytes", i64), ("small", vp), ("nsmall", i64),
                ("seg_small", vp)]


class SyncCfg(C.Structure):
    """csrc/server/sync_loop.cpp PsxSyncCfg."""
    _fields_ = [("comm", vp), ("core", vp), ("arena", vp), ("n_params", i64), ("arena_numel", i64),
                ("nworkers", i32), ("members", vp), ("gbufs", vp), ("grad_fp16", i32), ("lr", f32),
                ("momentum", f32), ("weight_decay", f32), ("mom_buf", vp), ("mom_first", i32), ("image", i32),
                ("wire_buf", vp), ("wire_bytes", i64), ("wire_img", vp), ("small_idx", vp), ("small_n", i64),
                ("wire_small", vp), ("nbuckets", i32), ("buckets", vp), ("full_wire", vp), ("full_wire_bytes", i64),
                ("primed", i32), ("upd_stream", vp), ("comm_stream", vp), ("ckpt_every", C.c_longlong),
                ("ckpt_cb", CKPT_CB), ("snap", vp), ("snap_mom", vp)]


_SIGS = {
    "psx_sync_cfg_size": (i32, []),
    "psx_sync_bucket_size": (i32, []),
    "psx_sync_create": (vp, [C.POINTER(SyncCfg), C.c_char_p, C.c_char_p]),
    "psx_sync_run": (i32, [vp, C.c_longlong]),
    "psx_sync_drain": (i32, [vp]),
    "psx_sync_progress": (None, [vp, C.POINTER(C.c_longlong)]),
    "psx_sync_phase_us": (None, [vp, C.POINTER(C.c_double)]),
    "psx_sync_mom_first": (i32, [vp]),
    "psx_sync_primed": (i32, [vp]),
    "psx_sync_abort": (C.c_longlong, [vp]),
    "psx_sync_rollback": (C.c_longlong, [vp]),
    "psx_sync_destroy": (None, [vp]),
}


def _lib():
    lib = comm()
    if not getattr(lib, "_psx_sync_declared", False):
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        lib._psx_sync_declared = True
        if lib.psx_sync_cfg_size() != C.sizeof(SyncCfg) or lib.psx_sync_bucket_size() != C.sizeof(SyncBucket):
            raise RuntimeError("PsxSyncCfg / PsxSyncBucket layout mismatch between sync_loop.cpp and native_sync.py")
    return lib


class NativeSyncError(RuntimeError):
    """psx_sync_run's error code (csrc/server/sync_loop.cpp): -60 a communicator call failed,
    -65 the run stopped because the watchdog aborted the communicator — the two that mean 'the
    communicator is gone' (parallel/elastic.py lost_error). -50 HIP error, -61 apply kernel,
    -62 round incomplete on the core, -63 checkpoint callback, -64 small-tensor gather: job
    failures that a shrink would only repeat — unless this server's abort() ran: the watchdog's
    communicator abort then usually surfaces first as a HIP error of the blocked loop thread
    (-50 / -61; the first error wins in the loop), and the run is a lost communicator all the same."""

    LOST = (-60, -65)

    def __init__(self, rc: int, aborted: bool = False):
        self.rc = int(rc)
        self.aborted = bool(aborted)
        super().__init__(f"native sync server failed ({self.rc}{', aborted' if self.aborted else ''})")

    @property
    def comm_lost(self) -> bool:
        return self.rc in self.LOST or self.aborted


def native_sync_enabled(cfg, transport, chan, server, rank: int) -> bool:
    """The dedicated server rank's rounds in native code (default; PSX_NATIVE_SYNC=0: Python)."""
    from .overlap import OverlapSyncChannel
    from .worker import SyncCollectiveChannel

    if not (os.environ.get("PSX_NATIVE_SYNC", "1") == "1" and rank == 0 and server is not None
            and getattr(transport, "native", False) and getattr(transport, "world_size", 1) > 1
            and cfg.mode == "sync" and cfg.topology == "dedicated" and cfg.codec in ("fp16", "none")
            and not cfg.bn_sync and type(chan) in (SyncCollectiveChannel, OverlapSyncChannel)
            and not getattr(chan, "root_worker", True) and getattr(chan, "agg_mode", "gather") == "gather"):
        return False
    if type(chan) is SyncCollectiveChannel and not chan.image:
        # serial_round broadcasts the whole fp32 arena as ONE F32 broadcast: only the raw fp32
        # fetch payload matches the workers' collective sequence (a FetchCodec packs several
        # broadcasts of other dtypes, e.g. bf16conv with --sync-steps > 1 or PSX_WEIGHT_IMAGE=0)
        codec = getattr(chan, "codec", None)
        return codec is None or codec.kind == "fp32"
    return True


class NativeSyncServer:
    """The dedicated server rank's side of a sync channel ``chan``, run natively."""

    def __init__(self, server, transport, chan, elastic: bool = False):
        self.server, self.t, self.chan = server, transport, chan
        self.gs0 = server.core.global_step  # the core's step when this loop took over
        cfg = server.cfg
        dev = server.device
        W = len(chan.members)
        if W != transport.world_size - 1:
            raise ValueError("native sync server: dedicated topology (world = workers + 1)")
        wire_dt = torch.float16 if cfg.codec == "fp16" else torch.float32
        if chan._gbufs is None:
            chan._gbufs = {r: torch.empty(server.n, dtype=wire_dt, device=dev) for r in range(1, transport.world_size)}
        self.gbufs = [chan._gbufs[r] for r in range(1, transport.world_size)]
        self._gptrs = (vp * W)(*[g.data_ptr() for g in self.gbufs])
        self._members = (C.c_int * W)(*chan.members)
        self._ckpt = CKPT_CB(self._checkpoint)
        overlap = bool(getattr(chan, "overlap", False))
        c = SyncCfg(comm=transport.comm.h.value, core=server.core._h, arena=server.arena.data_ptr(),
                    n_params=server.n, arena_numel=server.arena.numel(), nworkers=W,
                    members=C.cast(self._members, vp), gbufs=C.cast(self._gptrs, vp), grad_fp16=int(cfg.codec == "fp16"),
                    lr=float(server.lr), momentum=float(cfg.momentum or 0.0), weight_decay=float(cfg.weight_decay or 0.0),
                    mom_buf=server.momentum_buf.data_ptr() if (cfg.momentum and server.momentum_buf is not None) else None,
                    mom_first=int(server._mom_first),
                    upd_stream=torch.cuda.current_stream(dev).cuda_stream,
                    ckpt_every=int(cfg.ckpt_every or 0) if cfg.ckpt_dir else 0, ckpt_cb=self._ckpt)
        self.keep = []
        if elastic:  # parallel/elastic.py: a snapshot of every in-flight round's starting state
            self.snap = torch.empty(3 * server.arena.numel(), dtype=torch.float32, device=dev)
            c.snap = self.snap.data_ptr()
            if cfg.momentum and server.momentum_buf is not None:
                self.snap_mom = torch.empty(3 * server.n, dtype=torch.float32, device=dev)
                c.snap_mom = self.snap_mom.data_ptr()
        if overlap:
            wire = chan.wire
            bks = []
            for k, b in enumerate(chan.buckets):
                lo_b, hi_b, small, main, nsmall = wire.segs[k]
                base = wire.buf.data_ptr() + lo_b
                if small is not None:
                    self.keep.append(small)
                    bks.append(SyncBucket(b.lo, b.hi, base, hi_b - lo_b, small.data_ptr(), small.numel(), base + main))
                else:
                    bks.append(SyncBucket(b.lo, b.hi, base, hi_b - lo_b, None, 0, None))
            self._buckets = (SyncBucket * len(bks))(*bks)
            c.nbuckets = len(bks)
            c.buckets = C.cast(self._buckets, vp)
            c.full_wire, c.full_wire_bytes = wire.buf.data_ptr(), wire.buf.numel()
            c.primed = int(bool(chan._inflight))
            c.comm_stream = transport._cstream.cuda_stream
        elif chan.image:
            w = server.wire_for_fetch()  # image current (republished if an out-of-band update staled it)
            c.image = 1
            c.wire_buf, c.wire_bytes = w.buf.data_ptr(), w.buf.numel()
            c.wire_img = w.img.data_ptr()
            c.small_idx, c.small_n, c.wire_small = w.small_index.data_ptr(), w.small_index.numel(), w.small.data_ptr()
        self.cfg = c
        self.overlap = overlap
        self._aborted = False  # abort() ran (watchdog): any failure of the run is a lost communicator
        self.wire_bytes = (chan.wire.nbytes if overlap else (c.wire_bytes if c.image else server.arena.numel() * 4))
        kernels()  # both libraries loaded (bound by path)
        runtime()
        self.h = _lib().psx_sync_create(C.byref(c), os.path.join(NATIVE_DIR, "libpsx_runtime.so").encode(),
                                        os.path.join(NATIVE_DIR, "libpsx_kernels.so").encode())
        if not self.h:
            raise RuntimeError("psx_sync_create failed")

    def _checkpoint(self, global_step: int) -> int:
        try:
            with torch.cuda.device(self.server.device):
                self.server.maybe_checkpoint()
            return 0
        except Exception as e:  # noqa: BLE001 - reported, the run ends with an error
            import sys

            print(f"[psx native sync] checkpoint at step {global_step} failed: {e}", file=sys.stderr, flush=True)
            return 1

    def progress(self):
        out = (C.c_longlong * 2)()
        _lib().psx_sync_progress(self.h, out)
        return int(out[0]), int(out[1])

    def phase_totals(self) -> tuple[int, float, float, float]:
        """(rounds retired, gather us, apply us, broadcast us): device time summed over the loop's
        retired rounds (csrc/server/sync_loop.cpp psx_sync_phase_us). The gather range spans the
        receives' post to the last worker's wire landing, so it holds the workers' step."""
        out = (C.c_double * 4)()
        _lib().psx_sync_phase_us(self.h, out)
        return int(out[0]), float(out[1]), float(out[2]), float(out[3])

    def run(self, rounds: int, watchdog=None):
        """All ``rounds`` rounds of the job; returns when their device work is done."""
        if rounds <= 0:
            return
        if self.overlap and not self.cfg.primed:  # the first round's whole-wire fetch
            w = self.chan.wire
            for k in range(len(self.chan.buckets)):
                w.pack(self.server.arena, k)
            w.pack_buffers(self.server.arena)
        if watchdog is not None:
            watchdog.follow(self.progress)
        try:
            rc = _lib().psx_sync_run(self.h, int(rounds))
            rc = _lib().psx_sync_drain(self.h) or rc
        finally:
            if watchdog is not None:
                watchdog.follow(None)
        s, W = self.server, len(self.chan.members)
        s._mom_first = bool(_lib().psx_sync_mom_first(self.h))
        s.update_time_source = "device events around the apply kernels (native sync loop)"
        s.bytes_pushed += rounds * W * s.n * (2 if s.cfg.codec == "fp16" else 4)
        s.bytes_fetched += rounds * self.wire_bytes * max(0, W - 1)
        if self.overlap:
            self.cfg.primed = _lib().psx_sync_primed(self.h)  # later runs skip the host re-pack
            self.chan._inflight = bool(self.cfg.primed)
            self.chan._have_buffers = True
        if rc:
            raise NativeSyncError(rc, aborted=self._aborted)

    def abort(self) -> int:
        """Liveness watchdog thread: freeze the good-round count, stop issuing, abort the
        communicator (csrc/server/sync_loop.cpp psx_sync_abort)."""
        self._aborted = True
        return int(_lib().psx_sync_abort(self.h))

    def rollback(self) -> int:
        """After a failed / aborted run: the arena back at the start of the first round not known
        good; the core's step rolled back to it. Returns the core's global step kept."""
        g = int(_lib().psx_sync_rollback(self.h))
        if g < 0:
            raise RuntimeError(f"native sync rollback failed ({g})")
        self._aborted = False
        s = self.server
        s._mom_first = bool(_lib().psx_sync_mom_first(self.h))
        s.core.rollback_to(self.gs0 + g)
        s._wire_stale = s.wire is not None  # the fetch image no longer matches the arena
        return self.gs0 + g

    def close(self):
        if self.h:
            _lib().psx_sync_destroy(self.h)
            self.h = None
