"""Sharded parameter server (``--topology sharded``): every rank is a worker AND owns 1/world of
the server state.

The reference has one server process holding the whole model (reference:
src/parameter_server/server.py:95-96, SURVEY.md §2.4 "Sharded PS ... no"); SURVEY.md §2.4 lists a
sharded-server variant as the xGMI-friendly stretch next to the rank-0 PS the north star fixes.
Here the sync round is

    push : all-to-all of the fp16 gradient wire chunks — rank r receives every rank's chunk r
           (the bytes of a reduce-scatter, without its fp16 running sum)
    apply: rank r runs the fused SGD (csrc/kernels/optim.hip sgd_apply_multi: the W chunks
           decoded and summed in fp32 in rank order) on params[lo_r:hi_r] only, writing the
           parameter image of that range (bf16 for the bf16 compute path, fp32 for fp32) and
           gathers the fp32 entries of its range that a worker needs (BN affine, FC; rank 0 also
           the BN running buffers)
    fetch: all-gather of the image chunks + all-gather of the fp32 chunks

so every link carries (world-1)/world of the payload in each direction and no rank serialises
the whole update (ring reduce + broadcast through rank 0 in the default topology). Rank 0 keeps
the bookkeeping role (registration, round barrier, global step, metrics) through its
ParameterServer's native core; every rank's ParameterServer holds a full fp32 replica of which it
only updates its own range (the momentum buffer likewise). ``gather_master`` all-gathers the fp32
ranges into rank 0's arena at the end of the run (final checksum / metrics).

Scope: sync mode, one push per batch, dense fp16/fp32 gradients (no top-k), no --bn-sync, no
checkpoints (utils/config.py validates this). Opt-in; the default stays the rank-0 PS.
"""
from __future__ import annotations

import torch

from .codec import small_index_of
from .liveness import WatchedRounds


class ShardPlan:
    """Equal per-rank chunks of the parameter prefix (8-element aligned) and each rank's share
    of the fp32 remainder."""

    def __init__(self, layout, world: int):
        n = layout.param_numel
        self.n, self.world = n, world
        self.chunk = -(-n // (world * 8)) * 8
        self.padded = self.chunk * world
        self.lo = [min(n, r * self.chunk) for r in range(world)]
        self.hi = [min(n, (r + 1) * self.chunk) for r in range(world)]
        small = small_index_of(layout)
        params = small[small < n]
        buffers = small[small >= n]
        self.idx = []
        for r in range(world):
            sel = params[(params >= self.lo[r]) & (params < self.hi[r])]
            if r == 0:
                sel = torch.cat([sel, buffers])  # static server buffers: published by rank 0
            self.idx.append(sel)
        self.S = max(1, max(int(t.numel()) for t in self.idx))
        # worker-side scatter: position r*S + j of the gathered remainder -> arena index idx[r][j]
        self.dst = torch.cat(self.idx)
        self.src = torch.cat([torch.arange(t.numel(), dtype=torch.int64) + r * self.S for r, t in enumerate(self.idx)])


class ShardedWire:
    """The fetch payload of the sharded round: ``img`` = image of all params (padded to world
    equal chunks, arena offsets; bf16 for the bf16 compute path, fp32 for fp32), ``small`` =
    [world][S] fp32 remainder blocks."""

    def __init__(self, plan: ShardPlan, device, img_dtype=torch.bfloat16):
        self.plan = plan
        self.device = torch.device(device)
        self.img = torch.zeros(plan.padded, dtype=img_dtype, device=self.device)
        self.small = torch.zeros(plan.world * plan.S, dtype=torch.float32, device=self.device)
        self.small_index = plan.dst.to(self.device)
        self.small_src = plan.src.to(self.device)

    @property
    def nbytes(self) -> int:
        return self.img.numel() * self.img.element_size() + self.small.numel() * 4

    def publish_full(self, arena: torch.Tensor, rank: int | None = None):
        self.img[: self.plan.n].copy_(arena[: self.plan.n])
        for r in range(self.plan.world) if rank is None else [rank]:
            self.publish_small(arena, r)

    def publish_small(self, arena: torch.Tensor, rank: int):
        idx = self.plan.idx[rank]
        if idx.numel():
            blk = self.small[rank * self.plan.S: rank * self.plan.S + idx.numel()]
            torch.index_select(arena, 0, idx.to(arena.device), out=blk)

    def scatter_spec(self, local_arena: torch.Tensor, small_from=None):
        return (self.small, self.small_index, local_arena, False, self.small_src)

    def to_arena(self, local_arena: torch.Tensor):
        local_arena[: self.plan.n].copy_(self.img[: self.plan.n])
        local_arena[self.small_index.to(local_arena.device)] = self.small[self.small_src.to(self.small.device)].to(
            local_arena.device)
        return local_arena


class ShardedSyncChannel(WatchedRounds):
    """Sync rounds against the sharded server (see the module docstring). ``server`` is this
    rank's ParameterServer (its range only is updated); rank 0's also does the bookkeeping."""

    def __init__(self, cfg, transport, server, members: list[int], layout, device, in_place: bool):
        self.cfg, self.t, self.server = cfg, transport, server
        self.rank, self.world = transport.rank, transport.world_size
        self.members = members
        self.plan = ShardPlan(layout, self.world)
        f32 = getattr(cfg, "dtype", "bf16") == "fp32"
        self.wire = ShardedWire(self.plan, device, torch.float32 if f32 else torch.bfloat16)
        self.wire.publish_full(server.arena)  # every rank starts from the same replica
        # the bf16 HIP engine reads the wire's image itself (use_wire); the fp32 engine unpacks
        # from its fp32 local arena, which the fetch fills from the fp32 image
        self.in_place = in_place and not f32
        r = self.rank
        self.lo, self.hi = self.plan.lo[r], self.plan.hi[r]
        dt = torch.float16 if cfg.codec == "fp16" else torch.float32
        # chunk r of every other rank's wire (all-to-all); this rank's own chunk stays in place
        self.recv = {p: torch.zeros(self.plan.chunk, dtype=dt, device=device) for p in range(self.world) if p != r}
        server.wire = None  # this rank's image range is written by apply_shard, not server.apply
        self._gs = 0

    # ---- worker-facing channel API
    def register(self, name, requested_id=-1):
        return requested_id, len(self.members)

    def weight_wire(self):
        return self.wire if self.in_place else None

    def bind_compute(self, compute):
        compute.pad_grads(self.plan.padded)

    def _fetch(self, worker_id, local_arena):
        if self.rank == 0:
            for w in self.members:
                self.server.core.on_fetch(w)
            self.server.bytes_fetched += self.wire.nbytes * max(0, len(self.members) - 1)
        self.t.all_gather_into(self.wire.img, self.plan.chunk)
        self.t.all_gather_into(self.wire.small, self.plan.S)
        if not self.in_place:
            self.wire.to_arena(local_arena)
        return self.server.core.global_step if self.rank == 0 else self._gs

    def _push(self, worker_id, grads, local_step, buffers=None):
        if grads.dtype == torch.int32 or buffers is not None:
            raise RuntimeError("the sharded server takes dense gradients without --bn-sync")
        if grads.numel() < self.plan.padded:
            raise RuntimeError("gradient buffer not padded to the shard plan (bind_compute)")
        c, r = self.plan.chunk, self.rank
        self.t.exchange_chunks(grads[: self.plan.padded], c, self.recv)
        srcs = [grads[r * c:(r + 1) * c] if p == r else self.recv[p] for p in range(self.world)]
        W = len(self.members)
        weight = 1.0 / W
        if self.rank == 0:
            res = None
            for wid in self.members:
                res = self.server.core.on_push(wid, local_step)
            self.server.bytes_pushed += W * self.plan.n * grads.element_size()
            if res is None or not res.apply:
                raise RuntimeError("sharded sync round did not complete at the barrier")
            weight = res.weight
        self.apply_shard(weight, srcs)
        self._gs += 1
        return True

    def finished(self, worker_id):
        pass

    # ---- server side of this rank
    def apply_shard(self, weight: float, srcs: list):
        """params[lo:hi] -= lr * weight * sum_r srcs[r] (fp32 sum in rank order), image range."""
        s = self.server
        n = self.hi - self.lo
        t0 = s._time_begin()
        if n > 0:
            bf16_img = self.wire.img.dtype == torch.bfloat16
            if s.device.type == "cuda":
                from ..ops import kernels as K

                buf = s.momentum_buf[self.lo:self.hi] if s.momentum_buf is not None else None
                K.sgd_apply_multi(s.params[self.lo:self.hi], [x[:n] for x in srcs], s.lr, gscale=weight,
                                  momentum=s.cfg.momentum, wd=s.cfg.weight_decay, buf=buf, first=s._mom_first, n=n,
                                  img=self.wire.img[self.lo:self.hi] if bf16_img else None)
                if not bf16_img:
                    self.wire.img[self.lo:self.hi].copy_(s.params[self.lo:self.hi])
            else:
                agg = torch.zeros(n, dtype=torch.float32, device=s.device)
                for x in srcs:  # fixed order, fp32 accumulation
                    agg.add_(x[:n].to(torch.float32))
                s.apply_range(agg, weight, self.lo, self.hi)
                self.wire.img[self.lo:self.hi].copy_(s.params[self.lo:self.hi])
        self.wire.publish_small(s.arena, self.rank)
        s.finish_round_apply(s._time_end(t0))

    def gather_master(self):
        """fp32 parameter ranges of every rank -> every rank's arena (rank 0's feeds the final
        metrics / checksum)."""
        tmp = torch.zeros(self.plan.padded, dtype=torch.float32, device=self.server.arena.device)
        tmp[self.rank * self.plan.chunk: self.rank * self.plan.chunk + (self.hi - self.lo)].copy_(
            self.server.params[self.lo:self.hi])
        self.t.all_gather_into(tmp, self.plan.chunk)
        self.server.params.copy_(tmp[: self.plan.n])
