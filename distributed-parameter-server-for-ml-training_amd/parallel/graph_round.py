"""The synchronous PS round with its communication overlapped on a second HIP stream.

The reference's sync round is strictly serial per worker: fetch the whole state, compute, push
the whole gradient, then the server applies once every worker has pushed (reference:
src/workers/worker.py:365-377, src/parameter_server/server.py:264-288). Here the worker's step
is captured as one HIP graph per gradient bucket (models/engine.py set_segments/capture) and the
round is laid out over two streams:

    compute stream : [graph 0: prologue (scatter the fetched fp32 remainder, unpack the bf16
                     operands from the weight wire), forward, loss, backward of bucket 0]
                     [graph 1: backward of bucket 1] ... [graph K-1] -> (next step) wait comm
    comm stream    :   after graph k: RCCL reduce(grad bucket k -> rank 0)
                       -> [rank 0] fused SGD apply of bucket k, writing the bf16 image straight
                          into the weight wire (csrc/kernels/optim.hip)
                       -> RCCL broadcast(image slice k)
                     tail: [rank 0] gather the fp32 remainder -> broadcast it

Buckets follow backward order (parallel/overlap.py plan_buckets: fc+layer4 first), so the big
layer-4 reduce/apply/broadcast runs while layers 3..1 still compute; only the small stem bucket
and the 60K-element remainder are exposed. The compute stream never waits on communication
inside a step (the earlier overlap channel, parallel/overlap.py, applied on the compute stream
behind each reduce). The collectives are psx's own RCCL communicator (parallel/rccl.py), issued
on the communication stream — torch.distributed's internal stream is not involved. A single
graph with the collectives as fork/join branches was measured slower (+0.24 ms/step at N=1: the
runtime dispatches branched graphs in pieces), and in-graph wait points need external event
nodes, which ROCm's stream capture refuses.

The next step's fetch is already done when the round ends: every rank's weight wire holds the
new version (rank 0's co-located worker reads the server's wire in place), so ``fetch`` is
bookkeeping except for the very first one, which broadcasts the initial state.

Opt-in (PSX_GRAPH_ROUND=1, see graph_round_enabled for the N=1 measurement). Applies when the
fast-path conditions hold (codec.weight_image_enabled), every rank trains
(colocated topology), the server optimizer has no state whose first step differs
(momentum 0) and --bn-sync is off; everything else uses the serial or the bucketed channel.
With --no-graph the same hooks run eagerly between the backward segments.
"""
from __future__ import annotations

import torch

from .worker import SyncCollectiveChannel


def graph_round_enabled(cfg, transport) -> bool:
    import os

    # opt-in (PSX_GRAPH_ROUND=1): at N=1 (RCCL forced, nothing to hide) it measured 2.20-2.24 vs
    # 2.03 ms/step for the serial round — ~15 us idle at every graph boundary, a cross-stream
    # join at the end and the apply running beside the backward kernels; it pays only when the
    # exposed xGMI time of the serial round (reduce 22.4 MB + broadcast 22.5 MB) exceeds that
    return (os.environ.get("PSX_GRAPH_ROUND", "0") == "1" and getattr(transport, "native", False)
            and cfg.topology == "colocated" and not cfg.momentum and not cfg.bn_sync)


class GraphRoundChannel(SyncCollectiveChannel):
    """Sync channel whose reduce/apply/broadcast run on a communication stream between the
    worker's per-bucket step graphs."""

    in_graph = True

    def __init__(self, transport, server, members, codec, wire, buckets, device):
        super().__init__(transport, server, members, codec, wire=wire)
        assert wire is not None, "every rank of the graph round trains (colocated topology)"
        self.buckets = buckets
        self.device = torch.device(device)
        self.cstream = torch.cuda.Stream(device=self.device)
        self.weight = 1.0 / max(1, len(self.members))
        self._primed = False
        self._grads = None

    # ---------------------------------------------------------------- captured hooks
    def bind(self, grads: torch.Tensor):
        self._grads = grads

    def after_segment(self, k: int):
        """Bucket k's reduce -> [rank 0] apply (+ bf16 image into the wire) -> broadcast, on the
        communication stream, ordered after what the compute stream has enqueued so far (the
        backward segment that finalises bucket k)."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.cstream.wait_event(ev)
        b = self.buckets[k]
        g = self._grads[b.lo:b.hi]
        with torch.cuda.stream(self.cstream):
            self.t.reduce_sum_to_server(g)
            if self.server is not None:
                self.server.apply_range(g, self.weight, b.lo, b.hi)
            self.t.broadcast_from_server(self.image_wire.buf[2 * b.lo:2 * b.hi])

    def finish(self):
        """Round tail: the fp32 remainder (BN affine, FC, BN buffers) after every bucket's apply;
        the compute stream then waits for the whole round (the next step needs the new state)."""
        w = self.image_wire
        with torch.cuda.stream(self.cstream):
            if self.server is not None:
                w.publish_small(self.server.arena)
            self.t.broadcast_from_server(w.buf[w.img_bytes:])
        torch.cuda.current_stream().wait_stream(self.cstream)

    # ---------------------------------------------------------------- protocol
    def _fetch(self, worker_id, local_arena):
        if self.server is not None:
            for w in self.members:
                self.server.core.on_fetch(w)
        if not self._primed:  # initial state; afterwards every round ends with the new version
            if self.server is not None:
                self.server.wire_for_fetch()
            self.t.broadcast_from_server(self.image_wire.buf)
            self._primed = True
        if self.server is not None:
            self.server.bytes_fetched += self.image_wire.nbytes * max(0, len(self.members) - 1)
            return self.server.core.global_step
        return self._gs_after_fetch()

    def _push(self, worker_id, grads, local_step, buffers=None):
        """The round's device work ran inside the step graph; record it in the server core."""
        if self.server is not None:
            res = None
            for w in self.members:
                res = self.server.core.on_push(w, local_step)
            assert res is not None and res.apply, "sync round did not complete on the server core"
            self.server.bytes_pushed += len(self.members) * self.server.n * grads.element_size()
            self.server.finish_round_apply()
            self.server.maybe_checkpoint()
        else:
            self._gs = getattr(self, "_gs", 0) + 1
        return True
