"""Backward-overlapped synchronous PS round (bucketed reduce -> apply -> broadcast).

The reference's sync round is strictly serial per worker: fetch the whole state, compute,
push the whole gradient, and the server applies once every worker has pushed (reference:
src/workers/worker.py:365-377, src/parameter_server/server.py:264-288). Here the same round is
pipelined over gradient *buckets* so the xGMI traffic hides under the backward pass:

* the flat gradient arena is cut into contiguous buckets in backward order (``plan_buckets``):
  for ResNet-18 with the default 2M-element target that is [fc + layer4.1] 4.8M,
  [layer4.0] 3.7M, [layer3.*] 2.1M, [layer2.*, layer1.*, stem] 0.7M;
* the worker's step is captured as one HIP graph per bucket (models/engine.py set_segments);
  after a segment is enqueued the bucket's RCCL reduce(sum -> rank 0) is issued
  asynchronously — RCCL runs on its own stream, ordered after the segment by an event, while
  the compute stream goes on with the next segment;
* rank 0 (the parameter server) applies the fused SGD update to exactly that slice of the
  master arena, packs it into the bucket's fetch wire segment and broadcasts it — still while
  the workers run the rest of their backward. The apply of bucket k is enqueued on the
  compute stream right *after* segment k+1, by which time its reduce has long finished, so
  the only cross-stream dependencies are already-satisfied events (no side stream, no extra
  hop on the critical path);
* each bucket's wire segment is self-contained (``BucketWire``: bf16 conv weights + the fp32
  BN/FC entries of that bucket), BN running statistics travel once (first fetch) unless
  ``--bn-sync`` changes them every round; the next ``fetch`` only waits for the in-flight
  broadcasts and unpacks.

Semantics are exactly the sync PS round (all W gradients averaged, one SGD step, everyone
fetches the new state), only the communication is overlapped; only the last, smallest bucket
(the stem end of the network) is exposed. Enabled when every batch is pushed (sync_steps 1).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .worker import SyncCollectiveChannel


def unit_key(name: str) -> str:
    """Backward unit a parameter belongs to: 'layer<i>.<j>' (residual block), 'fc' or 'stem'."""
    parts = name.split(".")
    if parts[0].startswith("layer") and len(parts) > 2:
        return ".".join(parts[:2])
    if parts[0] == "fc":
        return "fc"
    return "stem"


@dataclass
class Bucket:
    keys: list
    lo: int
    hi: int

    @property
    def numel(self) -> int:
        return self.hi - self.lo


def plan_buckets(layout, target_elems: int = 2 << 20) -> list:
    """Group backward units (in backward order) into contiguous arena ranges of >= target."""
    units = []  # (key, lo, hi) in arena order
    for name, e in layout.entries.items():
        if e.region != "param":
            continue
        k = unit_key(name)
        if units and units[-1][0] == k and units[-1][2] == e.offset:
            units[-1][2] = e.offset + e.numel
        else:
            if any(u[0] == k for u in units):
                raise ValueError(f"parameters of unit {k!r} are not contiguous in the arena")
            units.append([k, e.offset, e.offset + e.numel])
    buckets, keys, hi = [], [], None
    for k, lo, h in reversed(units):
        keys.append(k)
        hi = h if hi is None else hi
        if hi - lo >= target_elems:
            buckets.append(Bucket(keys, lo, hi))
            keys, hi = [], None
    if keys:
        buckets.append(Bucket(keys, units[0][1], hi))
    assert buckets[0].hi == layout.param_numel and buckets[-1].lo == 0
    return buckets


class BucketWire:
    """Fetch wire format of the overlapped round: one byte buffer, one segment per bucket
    (+ one segment for the BN running statistics).

    ``bf16conv``: segment k = [bf16 of params[lo:hi] | fp32 of the non-conv params in lo:hi];
    bf16 -> fp32 is exact and the HIP engine rounds conv weights to bf16 anyway, so a worker
    reconstructs exactly the state it computes with (see parallel/codec.py).
    ``fp32``: segment k = fp32 params[lo:hi] (the reference payload, split)."""

    def __init__(self, layout, kind, buckets, device):
        self.layout, self.kind, self.buckets = layout, kind, buckets
        dev = torch.device(device)
        conv = torch.zeros(layout.param_numel, dtype=torch.bool)
        for e in layout.entries.values():
            if e.region == "param" and len(e.shape) == 4:
                conv[e.offset:e.offset + e.numel] = True
        self.segs = []  # (byte_lo, byte_hi, small_index or None, bf16/fp32 bytes, small bytes)
        off = 0
        for b in buckets:
            if kind == "fp32":
                main, small = 4 * b.numel, None
                nsmall = 0
            else:
                main = -(-2 * b.numel // 16) * 16
                small = (torch.nonzero(~conv[b.lo:b.hi]).flatten() + b.lo).to(dev)
                nsmall = 4 * small.numel()
            n = -(-(main + nsmall) // 16) * 16
            self.segs.append((off, off + n, small, main, nsmall))
            off += n
        self.buf_lo, self.buf_hi = off, off + 4 * layout.buffer_numel
        self.buf = torch.zeros(max(16, self.buf_hi), dtype=torch.uint8, device=dev)
        self.nbytes = off  # per-round payload (buffers excluded)

    def segment(self, k):
        lo, hi = self.segs[k][:2]
        return self.buf[lo:hi]

    def buffers_segment(self):
        return self.buf[self.buf_lo:self.buf_hi]

    def _views(self, k):
        lo, hi, small, main, nsmall = self.segs[k]
        b = self.buckets[k]
        if self.kind == "fp32":
            return self.buf[lo:lo + main].view(torch.float32), None, None
        return (self.buf[lo:lo + 2 * b.numel].view(torch.bfloat16), small,
                self.buf[lo + main:lo + main + nsmall].view(torch.float32))

    def pack(self, arena, k):
        b = self.buckets[k]
        main, small, sv = self._views(k)
        main.copy_(arena[b.lo:b.hi])
        if small is not None:
            torch.index_select(arena, 0, small, out=sv)

    def unpack(self, local_arena, k):
        b = self.buckets[k]
        main, small, sv = self._views(k)
        local_arena[b.lo:b.hi].copy_(main)
        if small is not None:
            local_arena.index_copy_(0, small, sv)

    def pack_buffers(self, arena):
        self.buffers_segment().view(torch.float32).copy_(arena[self.layout.param_numel:])

    def unpack_buffers(self, local_arena):
        local_arena[self.layout.param_numel:].copy_(self.buffers_segment().view(torch.float32))


class OverlapSyncChannel(SyncCollectiveChannel):
    """Sync-mode channel whose push is streamed bucket by bucket during the backward pass.

    Every rank issues the same collectives in the same order:
    push(b0), push(b1), bcast(b0), push(b2), bcast(b1), ..., bcast(b_last),
    [reduce(BN buffers), bcast(BN buffers)  -- --bn-sync only].
    push(b) = the workers' wire slices gathered to rank 0 by point-to-point (default, every
    worker on its own link) and summed there in fp32 in worker order by the range apply
    (server.apply_range_sources) — the serial round's aggregation; PSX_SYNC_AGG=reduce: an RCCL
    sum-reduce of the slice (wire-dtype arithmetic at every hop).
    """

    overlap = True

    def __init__(self, transport, server=None, members=None, codec=None, buckets=None, device="cpu",
                 root_worker=True):
        super().__init__(transport, server, members, codec, root_worker=root_worker)
        if codec is None:
            raise ValueError("OverlapSyncChannel needs a FetchCodec (its kind selects the wire format)")
        self.buckets = buckets
        self.device = torch.device(device)
        self.wire = BucketWire(codec.layout, codec.kind, buckets, self.device)
        self._works = []
        self._red = {}       # bucket -> (reduce work, grads) not yet applied/broadcast
        self._streamed = 0
        self._inflight = False
        self._have_buffers = False
        self._weight = 1.0 / max(1, len(self.members))

    # ---------------------------------------------------------------- round pieces
    def _finish_bucket(self, k):
        """Apply (rank 0) and broadcast bucket k, whose reduce was issued earlier."""
        w, grads = self._red.pop(k)
        b = self.buckets[k]
        if self.server is not None:
            w.wait()  # compute stream waits for the (normally already finished) reduce / gather
            t0 = self.server._time_begin()  # device time of this range's apply (summed per round)
            if self._gather():
                srcs = ([grads] if self.root_worker else []) + [self._gbufs[r] for r in sorted(self._gbufs)]
                self.server.apply_range_sources(srcs, self._weight, b.lo, b.hi)
            else:
                self.server.apply_range(grads[b.lo:b.hi], self._weight, b.lo, b.hi)
            self.server._time_end(t0)
            self.wire.pack(self.server.arena, k)
        else:
            self._works.append(w)
        self._works.append(self.t.broadcast_async(self.wire.segment(k)))

    def _gather(self) -> bool:
        return self.agg_mode == "gather" and getattr(self.t, "world_size", 1) > 1

    def push_bucket(self, k: int, grads: torch.Tensor):
        """Called right after backward segment k has been enqueued on the compute stream."""
        b = self.buckets[k]
        if self._gather():
            if self.server is not None and self._gbufs is None:
                self._gbufs = {r: torch.empty_like(grads) for r in range(1, self.t.world_size)}
            bufs = {r: g[b.lo:b.hi] for r, g in self._gbufs.items()} if self.server is not None else None
            self._red[k] = (self.t.gather_async(grads[b.lo:b.hi], bufs), grads)
        else:
            self._red[k] = (self.t.reduce_async(grads[b.lo:b.hi]), grads)
        if k > 0:
            self._finish_bucket(k - 1)
        self._streamed += 1

    def _push(self, worker_id, grads, local_step, buffers=None):
        if self._streamed == 0:  # nothing streamed (dedicated server rank): issue every bucket now
            for k in range(len(self.buckets)):
                self.push_bucket(k, grads)
        assert self._streamed == len(self.buckets), (self._streamed, len(self.buckets))
        self._streamed = 0
        self._finish_bucket(len(self.buckets) - 1)
        if buffers is not None:
            wb = self.t.reduce_async(buffers)
            if self.server is not None:
                wb.wait()
                self.server.set_buffers_from_sum(buffers, len(self.members))
                self.wire.pack_buffers(self.server.arena)
            else:
                self._works.append(wb)
            self._works.append(self.t.broadcast_async(self.wire.buffers_segment()))
        if self.server is not None:
            for w in self.members:
                res = self.server.core.on_push(w, local_step)
            assert res.apply, "sync round did not complete on the server core"
            self.server.bytes_pushed += len(self.members) * self.server.n * grads.element_size()
            self.server.finish_round_apply()
            self.server.maybe_checkpoint()
        else:
            self._gs = getattr(self, "_gs", 0) + 1
        self._inflight = True
        return True

    def _full_fetch(self, local_arena):
        """First round: the whole state, all segments + BN statistics in one broadcast."""
        if self.server is not None:
            for k in range(len(self.buckets)):
                self.wire.pack(self.server.arena, k)
            self.wire.pack_buffers(self.server.arena)
        self.t.broadcast_from_server(self.wire.buf)
        self._have_buffers = True
        return self._complete(local_arena, wait=False)

    def _complete(self, local_arena, wait=True):
        if wait:
            for w in self._works:
                w.wait()  # compute stream waits for the RCCL stream (host wait on gloo)
        self._works = []
        self._inflight = False
        if self.server is not None:
            for w in self.members:
                self.server.core.on_fetch(w)
            self.server.bytes_fetched += self.wire.nbytes * max(0, len(self.members) - 1)
            if local_arena is not None and local_arena.data_ptr() != self.server.arena.data_ptr():
                local_arena.copy_(self.server.arena)
            return self.server.core.global_step
        if local_arena is not None:
            for k in range(len(self.buckets)):
                self.wire.unpack(local_arena, k)
            self.wire.unpack_buffers(local_arena)  # parity: fetched running stats overwrite local ones
        return self._gs_after_fetch()

    def _fetch(self, worker_id, local_arena):
        if not self._inflight:
            return self._full_fetch(local_arena)
        return self._complete(local_arena)

    def _round_event(self):
        """The round's gathers / broadcasts run on the transport's communication stream, which
        the compute stream only waits for at the next fetch: the watchdog event is the last
        outstanding work's (recorded on that stream after every collective of the round)."""
        ev = getattr(self._works[-1], "event", None) if self._works else None
        return ev if isinstance(ev, torch.cuda.Event) else super()._round_event()

    def drain(self):
        """Finish an in-flight round without consuming it (end of training)."""
        for w in self._works:
            w.wait()
        self._works = []
        self._inflight = False

    def finished(self, worker_id):
        self.drain()
