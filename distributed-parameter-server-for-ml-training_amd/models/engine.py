"""HIP training engine: ResNet forward/backward on hand-written CDNA4 kernels.

This is the MI355X replacement for the worker's ``train_local_batch`` (reference:
src/workers/worker.py:333-348 — zero_grad, forward, CrossEntropyLoss, backward) and for
``evaluate_model`` (worker.py:313-331). Instead of autograd over ``nn.Module``s it runs an
explicit, statically-scheduled forward + backward over pre-allocated HBM buffers:

* activations NHWC in the compute dtype — bf16 (fast path) or fp32 (``dtype=torch.float32``,
  the reference's training precision, worker.py:333-348: conv operands and activations fp32,
  every product on the exact-f32 MFMA ``v_mfma_f32_16x16x4_f32``); conv = MFMA implicit GEMM
  (fwd / dgrad / split-K wgrad), BN batch statistics produced by the conv epilogue,
  BN+ReLU(+residual) fused elementwise passes, fused pool+FC+softmax-xent head;
* gradients are written straight into one flat wire buffer (fp16 codec by default) laid out
  like the trainable-parameter prefix of the parameter arena (models/layout.py), so a push is
  a single RCCL reduce/send of one buffer and the server update one fused kernel;
* parameters are read from a worker-local fp32 arena (the fetched server state) and unpacked
  to implicit-GEMM operands of the compute dtype by one table-driven kernel per fetch;
* no allocation, host sync or data-dependent host control flow inside a step, so the whole
  step (unpack + augment + fwd + bwd) is captured once into a HIP graph and replayed.

The network is described by a generic block list so ResNet-18 (CIFAR stem) and ResNet-50
(ImageNet stem with max-pool) share one engine.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from ..ops import kernels as K
from ..utils.tune import tune, tune_flag
from .layout import ParamLayout
from .resnet import Bottleneck, BasicBlock

CIFAR_MEAN = (0.5071, 0.4867, 0.4408)  # reference worker.py:149-150
CIFAR_STD = (0.2675, 0.2565, 0.2761)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _pow2_ceil(v: int, lo: int = 8) -> int:
    p = lo
    while p < v:
        p *= 2
    return p


@dataclass
class ConvSpec:
    name: str
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    h: int = 0  # input spatial
    w: int = 0
    need_dgrad: bool = True
    cp: int = 0
    kg: int = 0
    kgd: int = 0
    wf_off: int = 0
    wd_off: int = -1

    def finalize(self, chunk: int = 8):
        # input channels padded to a power of two >= one 16-byte chunk (8 bf16 / 4 fp32)
        self.cp = _pow2_ceil(self.cin, chunk)
        self.kg = -(-(self.k * self.k * self.cp) // 64) * 64
        self.kgd = self.k * self.k * self.cout  # cout % 64 == 0 for every ResNet conv
        assert self.kgd % 64 == 0 and self.cout % 64 == 0, self.name

    @property
    def out_hw(self):
        return K.conv_out_hw(self.h, self.w, self.k, self.stride, self.pad)


@dataclass
class BNSpec:
    name: str
    c: int


@dataclass
class BlockSpec:
    convs: list
    bns: list
    down: tuple | None = None  # (ConvSpec, BNSpec)


@dataclass
class NetSpec:
    stem_conv: ConvSpec
    stem_bn: BNSpec
    maxpool: bool
    blocks: list = field(default_factory=list)
    fc: str = "fc"
    fc_in: int = 512
    classes: int = 100
    in_hw: tuple = (32, 32)


def netspec_from_module(model: torch.nn.Module, in_hw) -> NetSpec:
    def conv_of(m, name, h, w):
        return ConvSpec(name, m.in_channels, m.out_channels, m.kernel_size[0], m.stride[0], m.padding[0], h, w)

    h, w = in_hw
    stem = conv_of(model.conv1, "conv1", h, w)
    stem.need_dgrad = False
    h, w = stem.out_hw
    maxpool = hasattr(model, "maxpool")
    if maxpool:
        h, w = (h + 2 - 3) // 2 + 1, (w + 2 - 3) // 2 + 1
    spec = NetSpec(stem, BNSpec("bn1", model.bn1.num_features), maxpool)
    for li in range(1, 5):
        layer = getattr(model, f"layer{li}")
        for bi, blk in enumerate(layer):
            pre = f"layer{li}.{bi}"
            if isinstance(blk, BasicBlock):
                names = ["conv1", "conv2"]
                down_mod = blk.shortcut if len(blk.shortcut) else None
                down_names = (f"{pre}.shortcut.0", f"{pre}.shortcut.1")
            elif isinstance(blk, Bottleneck):
                names = ["conv1", "conv2", "conv3"]
                down_mod = blk.downsample
                down_names = (f"{pre}.downsample.0", f"{pre}.downsample.1")
            else:
                raise TypeError(type(blk))
            convs, bns = [], []
            ch, cw = h, w
            for i, n in enumerate(names):
                m = getattr(blk, n)
                cs = conv_of(m, f"{pre}.{n}", ch, cw)
                convs.append(cs)
                bns.append(BNSpec(f"{pre}.bn{i + 1}", getattr(blk, f"bn{i + 1}").num_features))
                ch, cw = cs.out_hw
            down = None
            if down_mod is not None:
                ds = conv_of(down_mod[0], down_names[0], h, w)
                down = (ds, BNSpec(down_names[1], down_mod[1].num_features))
            spec.blocks.append(BlockSpec(convs, bns, down))
            h, w = ch, cw
    spec.fc_in = model.fc.in_features
    spec.classes = model.fc.out_features
    spec.in_hw = tuple(in_hw)
    return spec


def all_convs(spec: NetSpec):
    yield spec.stem_conv
    for b in spec.blocks:
        yield from b.convs
        if b.down:
            yield b.down[0]


class HipResNetEngine:
    """Pre-allocated, graph-capturable ResNet training step on psx HIP kernels."""

    def __init__(self, model: torch.nn.Module, layout: ParamLayout, batch: int, device="cuda",
                 grad_dtype=torch.float16, in_hw=(32, 32), mean=CIFAR_MEAN, std=CIFAR_STD, bn_eps=1e-5,
                 bn_momentum=0.1, seed=1234, dtype=torch.bfloat16, deterministic=None):
        if not torch.cuda.is_available():
            raise RuntimeError("HipResNetEngine needs an MI355X (torch.cuda / HIP device)")
        K.unpack_desc_size()  # fail loudly right here if the native library is missing
        self.dev = torch.device(device)
        self.layout = layout
        self.B = batch
        self.spec = netspec_from_module(model, in_hw)
        self.grad_dtype = grad_dtype
        self.grad_fp16 = grad_dtype == torch.float16
        # compute dtype of activations and conv operands (fp32 = the reference's precision)
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError(f"engine dtype {dtype}: bfloat16 or float32")
        self.dtype = dtype
        self.f32 = dtype == torch.float32
        # deterministic mode (the default; PSX_DETERMINISTIC=0 or deterministic=False: off): every
        # BN statistic accumulates as exact fixed-point integers (csrc/kernels/bnfin.hpp DetRed),
        # so two runs of a step give bit-identical gradients, for +0-2 % step time
        if deterministic is None:
            deterministic = os.environ.get("PSX_DETERMINISTIC", "1") == "1"
        self.deterministic = bool(deterministic)
        self.mean, self.std = mean, std
        self.eps, self.mom = bn_eps, bn_momentum
        self.seed = seed
        self.graph = None
        self.graphs = None
        self.segments = None  # backward split points (set_segments), None = one segment
        # BN finalize inside the producing launch (csrc/kernels/bnfin.hpp): off (tests switch the
        # attribute: tests/test_engine_gpu.py)
        self.fuse_fin = False
        # BN-backward sums from the dgrad epilogue (skips the separate bn_bwd_reduce pass where a
        # dgrad produces the BN's input gradient): neutral with 32 stat slots + separate finalize
        # (2.215 vs 2.217 ms/step), a small win with 8 slots + folded finalize (1.996/2.000 vs
        # 2.010/2.006 ms/step, two same-box A/B pairs), so on (the attribute is a test switch)
        # BN finalize folded into the consuming apply launches (bnfin.hpp bn_fin_lds): every apply
        # workgroup re-derives the affine/coefficients from the stat slots, removing 40 finalize
        # launches per step. With 32 slot rows it measured slower (2.18 vs 2.10 ms/step); with 8
        # rows (csrc/kernels/common.hpp) it wins: 1.999 vs 2.019 ms/step.
        self.fin_apply = not self.fuse_fin
        self.fuse_bnbwd = True
        self._prereduced = set()
        # with the fused sums the dgrad epilogue already reads the ReLU mask operand o: it stores
        # dz = g*[o > 0] instead of g (bwd_stats_desc mask_store), the BN-backward apply then runs
        # without o (one activation read less per BN layer) and dz doubles as the identity
        # shortcut's gradient (no dzout copy)
        self.mask_store = self.fuse_bnbwd
        # BN-backward applies folded into the fused Winograd data gradient + dy transform (_bn_bwd_to)
        self.bwd_fold = self.mask_store and tune_flag("wino_bwdfold", True)
        self._bwd_fold = {}
        self._premasked = set()
        # weight gradients (+ their batched reductions) on a side stream, a parallel branch of the
        # captured step graph next to the dgrad -> BN-backward chain. PSX_TUNE wgrad_stream=1 / 0
        # forces it; the default keeps it except for the fp32 engine on CIFAR-size images, whose
        # fused Winograd weight gradients (1 workgroup per CU, like the data gradients beside them)
        # only time-share the chip with the dgrad chain and add cross-queue waits: same box
        # 3.35-3.38 -> 3.28-3.29 ms/step without it (r4_call20/21); bf16 ResNet-18 (1.85 -> 1.89)
        # and fp32 ResNet-50 (40.4 -> 41.5) keep it.
        ws = tune("wgrad_stream", "auto")
        if ws == "auto":
            ws = "0" if (self.f32 and max(self.spec.in_hw) <= 64) else "1"
        self.wg_stream = torch.cuda.Stream(device=self.dev) if ws == "1" else None
        # the stride-2 block's 1x1 shortcut data gradient folded into the 3x3 one's launch
        self.fold_sc = True
        # the CIFAR stem on the direct vector-ALU kernel (csrc/kernels/stem.hip): fp32 27.4 -> 19.5 us
        # in isolation (bench/stem_probe.py); step A/B within noise, bf16 unmeasured in isolation.
        # The direct stems: fp32 (CIFAR 3x3 and ImageNet 7x7) and the bf16 ImageNet 7x7 (stem.hip)
        self.stem_direct = self.f32 or self.spec.stem_conv.k == 7
        # the later stages' Winograd weight transforms overlap the first stage's forward on the
        # side stream; without one they stay on the compute stream (a stream of their own measured
        # 3.36 vs 3.28 ms/step — a forked branch at the step start costs more than the overlap
        # returns, r4_numbers.jsonl r4_call23 — and was removed)
        self.wt_stream = self.wg_stream
        self._wg_batch = None
        self._fins = {}
        self.wsrc = None        # bf16 weight image to unpack from (set_weight_source), None = arena
        self.pre_unpack = None
        self._build()

    def _set_unpack_descs(self, convs):
        """The param_unpack_tiles table: one descriptor per conv whose implicit-GEMM operands
        (forward rows at wf_off, data-gradient rows at wd_off of wbuf) are unpacked each step."""
        descs = []
        tile0 = 0  # flat grid of param_unpack_tiles: (64x64 (oc, c) tile, chunk of <= 3 taps) units
        for cs in convs:
            descs.append((self.layout.offset(f"{cs.name}.weight"), cs.wf_off, cs.wd_off, cs.cout, cs.cin, cs.k, cs.k,
                          cs.cp, cs.kg, cs.kgd, tile0))
            tile0 += -(-cs.cout // 64) * -(-cs.cp // 64) * -(-(cs.k * cs.k) // 3)
        self.ntiles = tile0
        dsz = K.unpack_desc_size()
        assert dsz == 3 * 8 + 8 * 4, dsz
        raw = np.zeros(len(descs), dtype=np.dtype([("o", "<i8", 3), ("i", "<i4", 8)]))
        for j, d in enumerate(descs):
            raw[j]["o"] = d[:3]
            raw[j]["i"] = d[3:]
        self.descs = torch.from_numpy(raw.view(np.uint8).copy()).to(self.dev)
        self.ndesc = len(descs)

    # ------------------------------------------------------------------ allocation
    def _bf(self, *shape):
        """An activation buffer of the compute dtype."""
        return torch.empty(*shape, dtype=self.dtype, device=self.dev)

    def _f32(self, *shape):
        return torch.zeros(*shape, dtype=torch.float32, device=self.dev)

    def _build(self):
        sp, B = self.spec, self.B
        # weights: one bf16 buffer holding every conv's fwd (and dgrad) operand
        off = 0
        for cs in all_convs(sp):
            cs.finalize(4 if self.f32 else 8)
            cs.wf_off = off
            off += cs.cout * cs.kg
            if cs.need_dgrad:
                cs.wd_off = off
                off += cs.cp * cs.kgd
            else:
                cs.wd_off = -1
        self.wbuf = torch.zeros(off, dtype=self.dtype, device=self.dev)
        self._set_unpack_descs(list(all_convs(sp)))

        H, W = sp.in_hw
        self.x0 = self._bf(B, H, W, sp.stem_conv.cp)
        self.labels = torch.zeros(B, dtype=torch.int32, device=self.dev)
        # [sample indices of the batch | step counter]: one host->device copy per step
        self.batch_meta = torch.zeros(B + 1, dtype=torch.int32, device=self.dev)
        self.index = self.batch_meta[:B]
        self.step_dev = self.batch_meta[B:]

        # per-BN persistent state: affine [2,C] (scale, shift), saved [2,C] (mean, invstd), coef [3,C]
        self.bn = {}

        # Cross-workgroup reductions (BN fwd statistics from the conv epilogue, BN bwd sums) use
        # fp32 atomics into PSX_STAT_SLOTS slot rows per BN layer; all slot rows live in one
        # buffer that is zeroed once at the start of every step (one memset node in the graph).
        self.nslots = K.bn_bwd_reduce_T(1, 64)
        # BN statistic shifts (csrc/kernels/bnfin.hpp BnFin::sshift): the forward statistics are
        # sums of (y - k) and (y - k)^2 with k = the layer's previous batch mean, so the variance
        # never cancels two large numbers when |mean| >> std. Row 0 = this step's k (read-only
        # during the step), row 1 = the batch means the finalizes write; the next training step's
        # augment launch copies row 1 -> row 0. Zero at the first step (plain sums).
        nshift = sp.stem_bn.c + sum(bs.c for b in sp.blocks for bs in b.bns) + \
            sum(b.down[1].c for b in sp.blocks if b.down)
        self.bn_shift = torch.zeros(2, nshift, dtype=torch.float32, device=self.dev)
        shift_off = [0]
        # the first CTR words of the slot buffer are the in-launch finalize counters (two per BN
        # layer: forward, backward; csrc/kernels/bnfin.hpp) — zeroed with the slots every step
        nbn = 1 + sum(len(b.bns) + (1 if b.down else 0) for b in sp.blocks)
        self.ctr_words = -(-2 * nbn // 64) * 64
        red_off = [self.ctr_words]
        nctr = [0]

        # deterministic mode: every slot entry is a 16-byte fixed-point pair (bnfin.hpp DetRed)
        sw = K.det_slot_scale() if self.deterministic else 1

        def bn_state(bs: BNSpec):
            fwd = red_off[0]
            bwd = fwd + sw * self.nslots * 2 * bs.c
            red_off[0] = bwd + sw * self.nslots * 3 * bs.c
            nctr[0] += 2
            so = shift_off[0]
            shift_off[0] += bs.c
            self.bn[bs.name] = dict(affine=self._f32(2, bs.c), saved=self._f32(2, bs.c), coef=self._f32(3, bs.c),
                                    c=bs.c, fwd=(fwd, sw * self.nslots * 2 * bs.c), bwd=(bwd, sw * self.nslots * 3 * bs.c),
                                    ctr=nctr[0] - 2, sshift=self.bn_shift[0, so:so + bs.c],
                                    sshift_next=self.bn_shift[1, so:so + bs.c])

        # activation / gradient buffers
        st = sp.stem_conv
        p, q = st.out_hw
        self.y0 = self._bf(B, p, q, st.cout)
        self.a0 = self._bf(B, p, q, st.cout)
        self.g0 = self._bf(B, p, q, st.cout)   # grad wrt a0 (or wrt maxpool input)
        self.dy0 = self._bf(B, p, q, st.cout)
        bn_state(sp.stem_bn)
        max_wg = 0
        max_wp = 0

        def track(cs: ConvSpec):
            # fp32 scratch: wgrad split-K partials (own buffer: wgrad may run on a side stream)
            # and conv split-K slabs (stream-ordered on the main stream)
            nonlocal max_wg, max_wp
            s = K.conv_wgrad2_splits(B, cs.h, cs.w, cs.cp, cs.cout, cs.k, cs.stride, cs.pad, cs.kg, self.f32)
            cs.splits = s
            oh, ow = cs.out_hw
            cs.wp = s * cs.cout * cs.kg  # fp32 partials of this layer (offset wp_off: _plan_wpart)
            cs.wp_off = 0
            max_wp = max(max_wp, cs.wp)
            max_wg = max(max_wg, K.conv2_workspace_bytes(B, oh, ow, cs.cout, cs.kg, self.f32) // 4,
                         K.conv2_workspace_bytes(B, cs.h, cs.w, cs.cp, cs.kgd, self.f32) // 4 if cs.need_dgrad else 0)

        track(st)
        h_in = self.a0
        if sp.maxpool:  # ImageNet stem: 3x3/s2 max-pool after bn1+relu (csrc/kernels/pool.hip)
            mh, mw = (p + 2 - 3) // 2 + 1, (q + 2 - 3) // 2 + 1
            self.p0 = self._bf(B, mh, mw, st.cout)
            self.pidx = torch.empty(B, mh, mw, st.cout, dtype=torch.uint8, device=self.dev)
            h_in = self.p0
        self.blk = []
        for b in sp.blocks:
            d = dict(inp=h_in)
            d["y"] = [self._bf(B, *cs.out_hw, cs.cout) for cs in b.convs]
            d["a"] = [self._bf(B, *cs.out_hw, cs.cout) for cs in b.convs[:-1]]
            d["dy"] = [self._bf(B, *cs.out_hw, cs.cout) for cs in b.convs]
            d["da"] = [self._bf(B, *cs.out_hw, cs.cout) for cs in b.convs[:-1]]
            last = b.convs[-1]
            d["out"] = self._bf(B, *last.out_hw, last.cout)
            d["gin"] = torch.empty_like(h_in)  # grad wrt block input
            for cs in b.convs:
                track(cs)
            for bs in b.bns:
                bn_state(bs)
            if b.down:
                ds, dbn = b.down
                track(ds)
                bn_state(dbn)
                d["ys"] = self._bf(B, *ds.out_hw, ds.cout)
                d["dys"] = self._bf(B, *ds.out_hw, ds.cout)
                d["dxs"] = torch.empty_like(h_in)
            else:
                d["dz"] = self._bf(B, *last.out_hw, last.cout)
            self.blk.append(d)
            h_in = d["out"]
        self.final = h_in
        self.red = self._f32(red_off[0])
        self.wpart = self._f32(max(1, max_wg))
        self.wpart_w = self._f32(max(1, self._plan_wpart(max_wp)))
        self._plan_wino()
        if self.wino_layers:
            # Winograd layers read their own transformed weights (unpack -> _wino_unpack): drop
            # them from the implicit-GEMM operand unpack (13 of ResNet-18's 20 convs, most bytes)
            self._set_unpack_descs([cs for cs in all_convs(sp) if cs.name not in self.wino_layers])
        # head
        fh, fw = self.final.shape[1], self.final.shape[2]
        self.head_hw = fh * fw
        self.pooled = self._f32(B, sp.fc_in)
        self.dlogits = self._f32(B, sp.classes)
        self.loss = self._f32(B)
        self.correct = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.dfinal = torch.empty_like(self.final)
        # gradient wire buffer (trainable-parameter prefix of the arena)
        self.grads = torch.zeros(self.layout.param_numel, dtype=self.grad_dtype, device=self.dev)

    def _plan_wino(self):
        """fp32 Winograd F(4x4,3x3) (csrc/kernels/wino.hip) for the 3x3 / stride-1 layers: forward
        and data gradient on images up to 64x64 (every 3x3 stride-1 layer of
        ResNet-18 CIFAR and ResNet-50's 56x56 / 28x28 ones; R50 fp32 top-k 3,060 -> 3,188 img/s),
        weight gradient up to 64x64
        (default 16: on 32x32 the direct tap-reuse kernel is faster, 101 vs 129 us). Same-box
        per-layer A/B in profiles/r2s4_wino_*.jsonl. Per layer: the transformed forward weights
        U [cout][36][cin] and data-gradient weights U' [cin][36][cout] (rebuilt by unpack() every
        step) and, where the weight gradient is Winograd, the transformed input V [36][T][cin] the
        forward leaves for it. In deterministic mode its BN sums take the fixed-order reduction
        like every other producer (wino_out_kernel + bnfin.hpp DetRed). Not for bf16. PSX_TUNE wino=0:
        direct kernels everywhere. Layers with 64 / 128 input channels (ResNet-18's 32x32 and 16x16
        stages) run forward and data gradient as ONE fused launch each (wino_fused.hip: the
        transforms inside the GEMM, V / P never in HBM; the other layers take the three-launch path;
        bench/wino_fused_ab.py: 32x32x64 fwd / dgrad 80 / 95 -> 58 / 63 us, 16x16x128 59 / 62 -> 50 / 51).
        The fused forward still writes V where the Winograd weight gradient reads it."""
        self.wino_layers = {}
        self.wino_wgrad = set()
        self.wino_wgf = set()   # weight gradient by the fused kernel (wino_wgrad.hip): reads x, not V
        self.wino_bnfold = {}
        self.wino_fused = {}
        self._xfold = {}        # conv -> (pre-BN y, BN affine): its input is relu(BN(y)), never written
        if not self.f32 or not tune_flag("wino", True):
            return
        fuse = True  # the fused single-launch kernel (wino_fused.hip) wherever it applies
        # fused weight gradient (wino_wgrad.hip) on images of at least 16x16: same box,
        # B = 128, us incl. output transform, fused vs three-launch (bench/wino_wgrad_ab.py,
        # profiles/r4_wino_wgrad_ab.jsonl): 32x32x64 58.4 vs 71.2, 16x16x128 55.3 vs 46.9 (+ the
        # forward's V store the three-launch path needs, ~7), 8x8x256 53.7 vs 43.2, 4x4x512 61.7 vs
        # 44.1. In the step (side stream; the forward's V store is on the critical path) same box:
        # off 3.568, >= 32 3.412, >= 16 3.363-3.372 ms/step (profiles/r4_numbers.jsonl)
        wgf, wgf_minhw = True, 16
        maxhw = 64
        wg = True
        # Winograd weight gradient up to 64x64 images: ResNet-50's 56x56 3x3 layers take the fused
        # one (their direct alternative is wgrad2f: the tap-reuse kernel needs power-of-two rows):
        # same box 36.8 -> 36.4 ms/step (profiles/r5_numbers.jsonl r5_call6)
        wg_maxhw = 64
        B = self.B
        s_main = s_d = s_part = 0
        for cs in all_convs(self.spec):
            if (cs.k != 3 or cs.stride != 1 or cs.pad != 1 or cs.cp != cs.cin or cs.h > maxhw or cs.w > maxhw
                    or not K.wino_ok(cs.h, cs.w, cs.cp, cs.cout)):
                continue
            vk, vc = K.wino_v_floats(B, cs.h, cs.w, cs.cout), K.wino_v_floats(B, cs.h, cs.w, cs.cp)
            s_main = max(s_main, vk, vc, K.wino_p_floats(B, cs.h, cs.w, cs.cp, cs.cout),
                         K.wino_p_floats(B, cs.h, cs.w, cs.cout, cs.cp))
            q = K.wino_wgrad_q(B, cs.h, cs.w, cs.cp, cs.cout) if wg and max(cs.h, cs.w) <= wg_maxhw else 0
            # fused single-launch kernel (wino_fused.hip) where it applies, per direction
            ff = fuse and K.wino_fused_ok(B, cs.h, cs.w, cs.cp, cs.cout)
            fd = fuse and cs.need_dgrad and K.wino_fused_ok(B, cs.h, cs.w, cs.cout, cs.cp)
            self.wino_fused[cs.name] = (ff, fd)
            uf = self._f32((40 if ff else 36) * cs.cout * cs.cp)
            ud = self._f32((40 if fd else 36) * cs.cout * cs.cp) if cs.need_dgrad else None
            # fused weight gradient (wino_wgrad.hip): transforms x and dy itself, so
            # the forward keeps no V and no D is formed
            qf = (K.wino_wgrad_fused_q(B, cs.h, cs.w, cs.cp, cs.cout)
                  if q > 0 and wgf and min(cs.h, cs.w) >= wgf_minhw else 0)
            v = self._f32(vc) if q > 0 and not qf else None  # None: the forward's V goes to scratch
            self.wino_layers[cs.name] = (uf, ud, v)
            if q > 0:
                self.wino_wgrad.add(cs.name)
                if qf:
                    self.wino_wgf.add(cs.name)
                    s_part = max(s_part, 36 * qf * cs.cout * cs.cp)
                else:
                    s_d = max(s_d, vk)
                    s_part = max(s_part, 36 * q * cs.cout * cs.cp)
        # BN folded into the next conv's input transform (PSX_TUNE wino_bnfold=1, default): a block's inner
        # BN (+ ReLU) whose only consumer is a Winograd conv with a Winograd weight gradient (that
        # reads V, not the activation) is finalized and applied inside wino_in_kernel, so its
        # activation is never written; the data gradient's ReLU mask comes from the BN affine
        # (needs the masked dz store, so the BN-backward apply never reads the activation either)
        self.wino_bnfold = {}
        if self._fold and self.mask_store and tune_flag("wino_bnfold", True):
            for b in self.spec.blocks:
                for i in range(len(b.convs) - 1):
                    nxt = b.convs[i + 1]
                    if nxt.name in self.wino_wgrad and nxt.cin == b.bns[i].c:
                        self.wino_bnfold[b.bns[i].name] = nxt.name
        # main-stream scratch (forward V of layers without a Winograd weight gradient / GEMM output;
        # data-gradient input tiles + GEMM output) and the weight-gradient side stream's own (dy
        # tiles, GEMM partials)
        self.wino_s1 = self._f32(max(1, s_main))
        self.wino_s2 = self._f32(max(1, s_main))
        self.wino_wd = self._f32(max(1, s_d))
        self.wino_wpart = self._f32(max(1, s_part))
        # the first block's first conv's weight gradient runs on the compute stream, concurrently
        # with the side stream's (_bwd_stem): its own scratch
        self.tail_split = (self.wg_stream is not None
                           and bool(self.spec.blocks) and self.spec.blocks[0].convs[0].name in self.wino_wgrad)
        self.wino_wd2 = self._f32(max(1, s_d)) if self.tail_split else None
        self.wino_wpart2 = self._f32(max(1, s_part)) if self.tail_split else None

    def _wino_unpack(self, arena):
        """Every Winograd layer's forward and data-gradient weight transforms: the first stage's
        layers in one launch on the compute stream, the rest (ResNet-18: 9.3 M of the 9.4 M
        Winograd weights, ~280 MB of transformed operands, ~80 us) in one launch on the side
        stream, overlapped with the forward of the first stage; the compute stream waits for it
        before the first conv that reads one of them (``_wino_late_wait``)."""
        key = arena.data_ptr()
        if getattr(self, "_wino_wb_key", None) != key:
            convs = [cs for cs in all_convs(self.spec) if cs.name in self.wino_layers]
            hw0 = max((cs.h for cs in convs), default=0)
            split = self.wt_stream is not None
            early, late = [], []
            self._wino_late = set()
            for cs in convs:
                u = self.wino_layers[cs.name]
                w = self._aview(arena, f"{cs.name}.weight")
                ff, fd = self.wino_fused[cs.name]
                dst = early if (not split or cs.h == hw0) else late
                if dst is late:
                    self._wino_late.add(cs.name)
                dst.append((w, u[0], cs.cout, cs.cp, False, int(ff)))
                if u[1] is not None:
                    dst.append((w, u[1], cs.cout, cs.cp, True, int(fd)))
            self._wino_wb = K.WinoWeightBatch(early) if early else None
            self._wino_wb_late = K.WinoWeightBatch(late) if late else None
            self._wino_wb_key = key
        if self._wino_wb is not None:
            self._wino_wb()
        self._late_ev = None
        if self._wino_wb_late is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self.wt_stream.wait_event(ev)
            with torch.cuda.stream(self.wt_stream):
                self._wino_wb_late()
                self._late_ev = torch.cuda.Event()
                self._late_ev.record(self.wt_stream)

    _late_ev = None
    _wino_late = frozenset()

    def _wino_late_wait(self, name):
        """The compute stream waits (once per step) for the side-stream weight transforms before
        the first conv that reads one of them."""
        if self._late_ev is not None and name in self._wino_late:
            torch.cuda.current_stream(self.dev).wait_event(self._late_ev)
            self._late_ev = None

    # ------------------------------------------------------------------ helpers
    def _gptr(self, name: str) -> int:
        return self.grads.data_ptr() + self.grads.element_size() * self.layout.offset(name)

    def _aview(self, arena, name):
        return self.layout.view(arena, name)

    def _red(self, bs: BNSpec, which: str):
        off, n = self.bn[bs.name][which]
        return self.red[off:off + n]

    def _ctr(self, bs: BNSpec, which: int) -> int:
        return self.red.data_ptr() + 4 * (self.bn[bs.name]["ctr"] + which)

    def _fin_fwd(self, bs: BNSpec, arena, count):
        key = ("f", bs.name, arena.data_ptr(), count)
        f = self._fins.get(key)
        if f is None:
            st = self.bn[bs.name]
            f = K.bn_fin(self._aview(arena, f"{bs.name}.weight"), self._aview(arena, f"{bs.name}.bias"),
                         self._aview(arena, f"{bs.name}.running_mean"), self._aview(arena, f"{bs.name}.running_var"),
                         st["affine"], st["saved"], self._ctr(bs, 0), count, self.eps, self.mom, bs.c,
                         sshift=st["sshift"], sshift_next=st["sshift_next"])
            self._fins[key] = f
        return f

    def _fin_bwd(self, bs: BNSpec, arena, count):
        key = ("b", bs.name, arena.data_ptr(), count)
        f = self._fins.get(key)
        if f is None:
            st = self.bn[bs.name]
            f = K.bn_bwd_fin(self._aview(arena, f"{bs.name}.weight"), st["saved"], st["coef"],
                             self._gptr(f"{bs.name}.weight"), self._gptr(f"{bs.name}.bias"), self._ctr(bs, 1), count,
                             1.0, bs.c, self.grad_fp16)
            self._fins[key] = f
        return f

    def _conv_bn_fwd(self, cs: ConvSpec, x, y, bs: BNSpec, arena, train: bool, bn_in=None):
        """conv -> (train) batch statistics + BN finalize | (eval) running-statistics affine.
        With conv v2 the finalize runs inside the conv launch (last workgroup, bnfin.hpp)."""
        oh, ow = cs.out_hw
        npix = self.B * oh * ow
        wf = self.wbuf[cs.wf_off:cs.wf_off + cs.cout * cs.kg]
        stats = self._red(bs, "fwd") if train else None
        fin = self._fin_fwd(bs, arena, npix) if (train and self.fuse_fin) else None
        wl = self.wino_layers.get(cs.name)
        assert bn_in is None or wl is not None, cs.name
        sshift = self.bn[bs.name]["sshift"] if train else None
        if wl is not None:
            self._wino_late_wait(cs.name)
            if self.wino_fused[cs.name][0]:
                K.wino_fused(x, wl[0], y, None, stats, wl[2], self.B, cs.h, cs.w, cs.cp, cs.cout, bn_in=bn_in,
                             sshift=sshift)
            else:
                v = wl[2] if wl[2] is not None else self.wino_s2
                K.wino_conv(x, wl[0], y, None, stats, v, self.wino_s1, self.B, cs.h, cs.w, cs.cp, cs.cout,
                            bn_in=bn_in, sshift=sshift)
            if not train:
                self._bn_eval(bs, arena)
            elif not self._fold:  # no in-launch finalize on this path
                self._bn_train(bs, arena, self.nslots, npix)
            return
        if not (self.stem_direct and fin is None and cs.cin == 3 and (cs.k, cs.stride, cs.pad) in ((3, 1, 1), (7, 2, 3))
                and K.stem_conv(x, wf, y, stats, self.B, cs.h, cs.w, cs.cin, cs.cp, cs.cout, cs.kg, sshift=sshift,
                                k=cs.k)):
            K.conv_fwd2(x, wf, y, stats, self.wpart, self.B, cs.h, cs.w, cs.cp, cs.cout, cs.k, cs.stride, cs.pad,
                        cs.kg, fin=fin, sshift=sshift)
        if not train:
            self._bn_eval(bs, arena)
        elif fin is None and not self._fold:
            self._bn_train(bs, arena, self.nslots, npix)

    @property
    def _fold(self) -> bool:
        return self.fin_apply and not self.fuse_fin

    def _apply(self, bs: BNSpec, y, out, arena, train: bool, res=None, bs2: BNSpec | None = None):
        """BN (+ residual, + shortcut BN bs2 on res) + ReLU; with fin_apply the training-mode
        finalize of bs (and bs2) runs inside this launch."""
        c = bs.c
        if train and self._fold:
            npix = y.numel() // c
            if bs2 is not None:
                K.bn_apply_fin(y, self._red(bs, "fwd"), self._fin_fwd(bs, arena, npix), out, c, relu=True, res=res,
                               part2=self._red(bs2, "fwd"), fin2=self._fin_fwd(bs2, arena, npix))
            else:
                K.bn_apply_fin(y, self._red(bs, "fwd"), self._fin_fwd(bs, arena, npix), out, c, relu=True, res=res)
            return
        K.bn_apply(y, self.bn[bs.name]["affine"], out, c, relu=True, res=res,
                   affine2=self.bn[bs2.name]["affine"] if bs2 is not None else None)

    def _bn_train(self, bs: BNSpec, arena, T, count):
        st = self.bn[bs.name]
        K.bn_finalize(self._red(bs, "fwd"), T, bs.c, count, self._aview(arena, f"{bs.name}.weight"),
                      self._aview(arena, f"{bs.name}.bias"), self.eps, self.mom,
                      self._aview(arena, f"{bs.name}.running_mean"), self._aview(arena, f"{bs.name}.running_var"),
                      st["affine"], st["saved"], sshift=st["sshift"], sshift_next=st["sshift_next"])

    def _bn_eval(self, bs: BNSpec, arena):
        st = self.bn[bs.name]
        K.bn_eval_affine(bs.c, self._aview(arena, f"{bs.name}.weight"), self._aview(arena, f"{bs.name}.bias"),
                         self._aview(arena, f"{bs.name}.running_mean"), self._aview(arena, f"{bs.name}.running_var"),
                         self.eps, st["affine"])

    def _side(self):
        """Weight gradients only feed the push, so they run on a side stream concurrently with
        the dgrad -> BN-backward critical path (ordered after their dy by an event; joined at
        the end of every backward segment)."""
        if self.wg_stream is None:
            return contextlib.nullcontext()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        self.wg_stream.wait_event(ev)
        return torch.cuda.stream(self.wg_stream)

    def join_side(self):
        if self.wg_stream is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self.wg_stream)

    def _plan_wpart(self, max_wp: int) -> int:
        """Batched weight-gradient reduction (PSX_TUNE wgrad_rbatch, default on): the layers of one
        residual block keep their split-K partials in disjoint slices of wpart_w until ONE
        wgrad_reduce_batch launch at the end of the block's backward reduces them all (8 launches
        instead of 19 for ResNet-18). Returns the fp32 size wpart_w needs."""
        self.rbatch = tune_flag("wgrad_rbatch", True)
        if not self.rbatch:
            return max_wp
        need = max_wp
        for b in self.spec.blocks:
            convs = list(b.convs) + ([b.down[0]] if b.down else [])
            if len(convs) > K.WRBATCH_MAX:
                continue
            off = 0
            for cs in convs:
                cs.wp_off = off
                off += cs.wp
            need = max(need, off)
        return need

    def _wgrad(self, cs: ConvSpec, x, dy):
        fold = self._bwd_fold.get(cs.name)
        if self._wg_batch is not None:  # deferred: issued together at the end of the unit
            self._wg_batch.append((cs, x, dy, fold))
            return
        with self._side():
            self._wgrad_now(cs, x, dy, fold)

    def _flush_wgrads(self):
        batch, self._wg_batch = self._wg_batch, None
        if batch:
            with self._side():
                for cs, x, dy, fold in batch:
                    self._wgrad_now(cs, x, dy, fold)

    def _wgrad_now(self, cs: ConvSpec, x, dy, fold=None, scratch=None):
        if cs.name in self.wino_wgf:  # fused Winograd weight gradient straight into the wire
            wpart = scratch[1] if scratch is not None else self.wino_wpart
            xf = self._xfold.get(cs.name)  # its input was never written: y + the BN affine instead
            K.wino_wgrad_fused(xf[0] if xf else x, dy, wpart, self.layout.grad_view(self.grads, f"{cs.name}.weight"),
                               self.B, cs.h, cs.w, cs.cp, cs.cout, xaff=xf[1] if xf else None, bwd_in=fold)
            return
        if cs.name in self.wino_wgrad:  # straight into the wire: no split partials to reduce
            wd, wpart = scratch if scratch is not None else (self.wino_wd, self.wino_wpart)
            K.wino_wgrad(self.wino_layers[cs.name][2], dy, wd, wpart,
                         self.layout.grad_view(self.grads, f"{cs.name}.weight"), self.B, cs.h, cs.w, cs.cp, cs.cout,
                         bwd_in=fold)
            return
        assert fold is None, cs.name
        part = self.wpart_w[cs.wp_off:cs.wp_off + cs.wp]
        K.conv_wgrad2(x, dy, part, self.B, cs.h, cs.w, cs.cp, cs.cout, cs.k, cs.stride, cs.pad, cs.kg)
        item = (part, cs.splits, cs.cout, cs.kg, cs.cin, cs.cp, cs.k, self._gptr(f"{cs.name}.weight"))
        if self._wr_batch is not None and K.wgrad_reduce_batchable(cs.cp, cs.k):
            self._wr_batch.append(item)  # reduced with the block's other layers (_flush_reduces)
            return
        K.wgrad_reduce(*item[:7], 1.0, item[7], self.grad_fp16)

    _wr_batch = None

    def _flush_reduces(self):
        batch, self._wr_batch = self._wr_batch, None
        if batch:
            with self._side():
                K.wgrad_reduce_batch(batch, 1.0, self.grad_fp16)

    def _dgrad(self, cs: ConvSpec, dy, dx, res=None, bn_next=None, sc=None):
        """bn_next = (BNSpec, o, y, two|None): the BN whose backward consumes dx; with conv v2 its
        reduction (sum dz, sum dz*xhat) is produced by the dgrad epilogue (fuse_bnbwd).
        sc = (shortcut ConvSpec, its output gradient): fold the block's 1x1 / stride-2 shortcut
        data gradient into this 3x3 / stride-2 launch; returns False (nothing launched) when the
        layer cannot fold."""
        wl = self.wino_layers.get(cs.name)
        if sc is not None:
            ds, dys_sc = sc
            if wl is not None or cs.k != 3 or cs.stride != 2 or cs.pad != 1 or ds.k != 1 or ds.stride != 2 \
                    or ds.pad != 0 or ds.cp != cs.cp or ds.cout != cs.cout or ds.kgd != cs.cout:
                return False
        bst = None
        if bn_next is not None and self.fuse_bnbwd:
            bs, o, y, two = bn_next
            st = self.bn[bs.name]
            ms = self.mask_store
            if bs.name in self.wino_bnfold:  # o was never written: the mask comes from the affine
                bst = K.bwd_stats_desc(self._red(bs, "bwd"), None, y, st["saved"], mask_store=ms,
                                       mask_aff=st["affine"])
            elif two is None:
                bst = K.bwd_stats_desc(self._red(bs, "bwd"), o, y, st["saved"], mask_store=ms)
            else:
                bs2, y2 = two
                bst = K.bwd_stats_desc(self._red(bs, "bwd"), o, y, st["saved"], y2, self.bn[bs2.name]["saved"],
                                       mask_store=ms)
            self._prereduced.add(bs.name)
            if ms:
                self._premasked.add(bs.name)
        if wl is not None:  # Winograd: the output transform produces the same fused sums
            if self.wino_fused[cs.name][1]:
                K.wino_fused(dy, wl[1], dx, res, None, None, self.B, cs.h, cs.w, cs.cout, cs.cp, bst=bst,
                             bwd_in=self._bwd_fold.get(cs.name))
            else:
                K.wino_conv(dy, wl[1], dx, res, None, self.wino_s1, self.wino_s2, self.B, cs.h, cs.w, cs.cout,
                            cs.cp, bst=bst)
            return
        wd = self.wbuf[cs.wd_off:cs.wd_off + cs.cp * cs.kgd]
        if sc is not None:
            wds = self.wbuf[ds.wd_off:ds.wd_off + ds.cp * ds.kgd]
            if not K.conv_dgrad2_sc(dy, wd, dx, self.wpart, self.B, cs.h, cs.w, cs.cp, cs.cout, cs.kgd, dys_sc, wds,
                                    ds.kgd, bst=bst):
                if bn_next is not None and self.fuse_bnbwd:  # nothing ran: the sums are not produced
                    self._prereduced.discard(bn_next[0].name)
                    self._premasked.discard(bn_next[0].name)
                return False
            return True
        K.conv_dgrad2(dy, wd, dx, res, self.wpart, self.B, cs.h, cs.w, cs.cp, cs.cout, cs.k, cs.stride, cs.pad,
                      cs.kgd, bst=bst)

    def _bn_bwd_to(self, cs: ConvSpec, bs: BNSpec, arena, g, o, y, dx, npix, dzout=None):
        """The backward of BN bs whose output gradient feeds only conv cs's data and weight
        gradients. Returns (dz, dy): dz as _bn_bwd returns it, dy the buffer cs's gradients read.
        Folded (PSX_TUNE wino_bwdfold=1, default: cs has the fused Winograd data gradient and a Winograd
        weight gradient, g is already the masked dz and its sums came from the producing dgrad's
        epilogue): no apply pass — dy = k1 dz + k2 y + k3 is formed inside both consumers'
        operand loads (wino_fused.hip, wino.hip dy transform), and the fused data gradient
        publishes the coefficients and dgamma / dbeta."""
        ok = (self.bwd_fold and self._fold and bs.name in self._premasked and bs.name in self._prereduced
              and cs.name in self.wino_wgrad and self.wino_fused.get(cs.name, (False, False))[1])
        if not ok:
            dz = self._bn_bwd(bs, arena, g, o, y, dx, npix, dzout=dzout)
            return dz, dx
        self._premasked.discard(bs.name)
        self._prereduced.discard(bs.name)
        self._bwd_fold[cs.name] = (y, self._red(bs, "bwd"), self._fin_bwd(bs, arena, npix))
        return g, g

    def _bn_bwd(self, bs: BNSpec, arena, g, o, y, dx, npix, two=None, dzout=None):
        """BN (+ReLU mask from o) backward; two = (bs2, y2, dx2) for a shared-dz second BN.
        Returns the buffer that holds dz = g*[o > 0]: ``g`` itself when the producing dgrad stored
        it masked (mask_store), else ``dzout`` (written here when given)."""
        if bs.name in self._premasked:
            self._premasked.discard(bs.name)
            self._bn_bwd_body(bs, arena, g, None, y, dx, npix, two, None)
            return g
        self._bn_bwd_body(bs, arena, g, o, y, dx, npix, two, dzout)
        return dzout

    def _bn_bwd_body(self, bs: BNSpec, arena, g, o, y, dx, npix, two, dzout):
        st = self.bn[bs.name]
        part = self._red(bs, "bwd")
        fuse = self.fuse_fin
        pre = bs.name in self._prereduced  # sums already produced by the dgrad epilogue
        self._prereduced.discard(bs.name)
        if pre:
            fuse = False
        if self._fold and not fuse:  # finalize inside the apply launch
            if two is None:
                if not pre:
                    K.bn_bwd_reduce(g, o, y, st["saved"], part, npix, bs.c)
                K.bn_bwd_apply_fin(g, o, y, part, self._fin_bwd(bs, arena, npix), dx, bs.c, dzout=dzout)
            else:
                bs2, y2, dx2 = two
                if not pre:
                    K.bn_bwd_reduce(g, o, y, st["saved"], part, npix, bs.c, y2=y2, saved2=self.bn[bs2.name]["saved"])
                K.bn_bwd_apply_fin(g, o, y, part, self._fin_bwd(bs, arena, npix), dx, bs.c, y2=y2,
                                   fin2=self._fin_bwd(bs2, arena, npix), dx2=dx2, dzout=dzout)
            return
        if two is None:
            T = self.nslots if pre else K.bn_bwd_reduce(g, o, y, st["saved"], part, npix, bs.c,
                                                        fin1=self._fin_bwd(bs, arena, npix) if fuse else None)
            if not fuse:
                K.bn_bwd_finalize(part, T, 2, 1, bs.c, npix, self._aview(arena, f"{bs.name}.weight"),
                                  st["saved"], st["coef"], self._gptr(f"{bs.name}.weight"),
                                  self._gptr(f"{bs.name}.bias"), 1.0, self.grad_fp16)
            K.bn_bwd_apply(g, o, y, st["coef"], dx, bs.c, dzout=dzout)
        else:
            bs2, y2, dx2 = two
            st2 = self.bn[bs2.name]
            T = self.nslots if pre else K.bn_bwd_reduce(g, o, y, st["saved"], part, npix, bs.c, y2=y2,
                                                        saved2=st2["saved"],
                                                        fin1=self._fin_bwd(bs, arena, npix) if fuse else None,
                                                        fin2=self._fin_bwd(bs2, arena, npix) if fuse else None)
            if not fuse:
                K.bn_bwd_finalize(part, T, 3, 1, bs.c, npix, self._aview(arena, f"{bs.name}.weight"),
                                  st["saved"], st["coef"], self._gptr(f"{bs.name}.weight"),
                                  self._gptr(f"{bs.name}.bias"), 1.0, self.grad_fp16)
                K.bn_bwd_finalize(part, T, 3, 2, bs2.c, npix, self._aview(arena, f"{bs2.name}.weight"),
                                  st2["saved"], st2["coef"], self._gptr(f"{bs2.name}.weight"),
                                  self._gptr(f"{bs2.name}.bias"), 1.0, self.grad_fp16)
            K.bn_bwd_apply(g, o, y, st["coef"], dx, bs.c, y2=y2, coef2=st2["coef"], dx2=dx2, dzout=dzout)

    # ------------------------------------------------------------------ public API
    def unpack(self, arena: torch.Tensor):
        """OIHW master weights -> bf16 implicit-GEMM operands. The source is the fp32 arena, or
        the bf16 weight image ``self.wsrc`` when the fetch delivers one (parallel/codec.py
        WeightWire: the server's apply wrote those bits; identical operands either way)."""
        src = self.wsrc if self.wsrc is not None else arena
        K.param_unpack_tiles(src, self.descs, self.ndesc, self.ntiles, self.wbuf, scatter=self.small_scatter)
        if self.wino_layers:
            self._wino_unpack(arena)

    small_scatter = None
    _zeroed = False       # red zeroed by this step's augment launch (consumed by forward)
    _zeroed_head = False  # correct zeroed by it (consumed by head)

    def set_weight_source(self, img: torch.Tensor | None, pre_unpack=None, scatter=None):
        """Read conv weights from a bf16 image (same offsets as the arena's parameter prefix)
        instead of the fp32 arena. The fp32 remainder reaches the local arena either through
        ``scatter`` = (src, idx, dst, gather), done by extra workgroups of the unpack launch
        (kernels.param_unpack_tiles), or through ``pre_unpack``, run first inside every captured
        step. Invalidates graphs."""
        if img is not None:
            assert not self.f32, "the fp32 engine unpacks its operands from the fp32 arena (fetch codec fp32)"
            assert img.dtype == torch.bfloat16 and img.numel() >= self.layout.param_numel
        assert scatter is None or (img is not None and pre_unpack is None)
        self.wsrc = img
        self.pre_unpack = pre_unpack
        self.small_scatter = scatter
        self.graph = None
        self.graphs = None

    def load_batch(self, images_u8, labels_all, train=True):
        """Gather self.index rows of the HBM-resident dataset + fused crop/flip/normalize."""
        H, W = self.spec.in_hw
        # a training step's per-step zeroing (BN statistic slots, accuracy counter) rides on the
        # augment launch (forward/head then skip their own zero_ launches)
        zero = (self.red, self.correct) if train else None
        self._zeroed_head = train
        K.augment(images_u8, labels_all, self.index, self.x0, self.labels, self.B, H, W, 4, self.seed, self.step_dev,
                  train, self.mean, self.std, zero=zero,
                  copy=(self.bn_shift[1], self.bn_shift[0]) if train else None)
        self._zeroed = train

    def forward(self, arena: torch.Tensor, train: bool = True):
        # the kernel library's deterministic-reduction state is process-wide host state: every
        # step (and every captured graph) takes this engine's setting
        K.set_deterministic(self.deterministic)
        sp, B = self.spec, self.B
        st = sp.stem_conv
        zeroed, self._zeroed = self._zeroed, False
        if train and not zeroed:
            self.red.zero_()
            self.bn_shift[0].copy_(self.bn_shift[1])  # this step's statistic shifts (see _build)
        self._conv_bn_fwd(st, self.x0, self.y0, sp.stem_bn, arena, train)
        self._apply(sp.stem_bn, self.y0, self.a0, arena, train)
        if sp.maxpool:
            K.maxpool3s2_fwd(self.a0, self.p0, self.pidx)
        for b, d in zip(sp.blocks, self.blk):
            src = d["inp"]
            L = len(b.convs)
            bn_in = None
            for i, cs in enumerate(b.convs):
                self._conv_bn_fwd(cs, src, d["y"][i], b.bns[i], arena, train, bn_in=bn_in)
                bn_in = None
                if i < L - 1:
                    bs = b.bns[i]
                    if train and bs.name in self.wino_bnfold:  # applied by the next conv's input transform
                        bn_in = (self._red(bs, "fwd"), self._fin_fwd(bs, arena, d["y"][i].numel() // bs.c))
                        src = d["y"][i]
                        self._xfold[b.convs[i + 1].name] = (d["y"][i], self.bn[bs.name]["affine"])
                        continue
                    self._apply(bs, d["y"][i], d["a"][i], arena, train)
                    src = d["a"][i]
            if b.down:
                ds, dbn = b.down
                self._conv_bn_fwd(ds, d["inp"], d["ys"], dbn, arena, train)
                self._apply(b.bns[-1], d["y"][-1], d["out"], arena, train, res=d["ys"], bs2=dbn)
            else:
                self._apply(b.bns[-1], d["y"][-1], d["out"], arena, train, res=d["inp"])
        return self.final

    def head(self, arena: torch.Tensor, backward: bool = True):
        sp = self.spec
        zeroed, self._zeroed_head = self._zeroed_head, False
        if not zeroed:
            self.correct.zero_()
        # the last block's output BN: its backward sums come out of the head launch (one
        # bn_bwd_reduce pass fewer) when the fused per-sample head runs and that BN has no
        # shortcut BN sharing its gradient
        bst, last = None, None
        if backward and self.fuse_bnbwd and sp.blocks and not sp.blocks[-1].down:
            last = sp.blocks[-1].bns[-1]
            bst = K.bwd_stats_desc(self._red(last, "bwd"), self.final, self.blk[-1]["y"][-1],
                                   self.bn[last.name]["saved"])
        fused = K.head_fwd_bwd(self.final, self.B, self.head_hw, sp.fc_in, self._aview(arena, f"{sp.fc}.weight"),
                               self._aview(arena, f"{sp.fc}.bias"), sp.classes, self.labels, self.pooled,
                               self.dlogits, self.dfinal if backward else None, self.loss, self.correct, bst=bst)
        if fused and last is not None:
            self._prereduced.add(last.name)

    def _bwd_fc(self, arena):
        self._bwd_fold = {}  # the first backward unit: this step's folds are recorded afresh
        sp = self.spec
        with self._side():
            K.head_wgrad(self.dlogits, self.pooled, self.B, sp.classes, sp.fc_in, self._gptr(f"{sp.fc}.weight"),
                         self._gptr(f"{sp.fc}.bias"), 1.0, self.grad_fp16)

    def _bwd_block(self, arena, j: int):
        """Backward of residual block j; its incoming gradient is the next block's input grad.
        With the side stream its weight gradients are issued as one batch after the block."""
        self._wg_batch = [] if self.wg_stream is not None else None
        b = self.spec.blocks[j]
        nconv = len(b.convs) + (1 if b.down else 0)
        self._wr_batch = [] if self.rbatch and nconv <= K.WRBATCH_MAX else None
        try:
            self._bwd_block_body(arena, j)
        finally:
            if j == 0 and self._split_tail() and self._wg_batch:
                # the step's tail: this weight gradient runs on the compute stream after the stem's
                # BN backward (_bwd_stem), concurrently with the side stream's, instead of after it
                first = self.spec.blocks[0].convs[0].name
                keep = [it for it in self._wg_batch if it[0].name != first]
                self._tail_wgrad = [it for it in self._wg_batch if it[0].name == first] or None
                self._wg_batch = keep
            self._flush_wgrads()
            self._flush_reduces()

    _tail_wgrad = None
    tail_split = False
    wino_wd2 = wino_wpart2 = None

    def _split_tail(self) -> bool:
        """Only when block 0 and the stem end in the same backward segment (a gradient bucket is
        pushed when its segment ends)."""
        if not self.tail_split:
            return False
        if self.segments is None:
            return True
        key = ".".join(self.spec.blocks[0].convs[0].name.split(".")[:2])
        return any(key in g and "stem" in g for g in self.segments)

    def _bwd_block_body(self, arena, j: int):
        sp, B = self.spec, self.B
        b, d = sp.blocks[j], self.blk[j]
        g = self.blk[j + 1]["gin"] if j + 1 < len(self.blk) else self.dfinal
        L = len(b.convs)
        last = b.convs[-1]
        oh, ow = last.out_hw
        npix = B * oh * ow
        dys = list(d["dy"])  # the buffers each conv's gradients read (dz where a BN apply is folded)
        if b.down:
            ds, dbn = b.down
            self._bn_bwd(b.bns[-1], arena, g, d["out"], d["y"][-1], d["dy"][-1], npix, two=(dbn, d["ys"], d["dys"]))
        else:
            dz, dys[-1] = self._bn_bwd_to(b.convs[-1], b.bns[-1], arena, g, d["out"], d["y"][-1], d["dy"][-1], npix,
                                          dzout=d["dz"])
        for i in range(L - 1, -1, -1):
            cs = b.convs[i]
            x_in = d["inp"] if i == 0 else d["a"][i - 1]
            self._wgrad(cs, x_in, dys[i])
            if i > 0:
                self._dgrad(cs, dys[i], d["da"][i - 1], bn_next=(b.bns[i - 1], d["a"][i - 1], d["y"][i - 1], None))
                _, dys[i - 1] = self._bn_bwd_to(b.convs[i - 1], b.bns[i - 1], arena, d["da"][i - 1], d["a"][i - 1],
                                                d["y"][i - 1], d["dy"][i - 1], B * cs.h * cs.w)
            elif b.down:
                ds, dbn = b.down
                self._wgrad(ds, d["inp"], d["dys"])
                # the 1x1 / stride-2 shortcut's data gradient folded into the 3x3 / stride-2 one
                # (PSX_TUNE dgrad_fold_sc=0: two launches + a residual pass)
                if not (self.fold_sc and self._dgrad(cs, dys[0], d["gin"], bn_next=self._bn_into(j),
                                                     sc=(ds, d["dys"]))):
                    self._dgrad(ds, d["dys"], d["dxs"])
                    self._dgrad(cs, dys[0], d["gin"], res=d["dxs"], bn_next=self._bn_into(j))
            else:
                self._dgrad(cs, dys[0], d["gin"], res=dz, bn_next=self._bn_into(j))

    def _bn_into(self, j: int):
        """The BN whose backward consumes block j's input gradient: the previous block's output
        BN (+ its shortcut BN), or the stem BN (not across the ResNet-50 max-pool)."""
        if j > 0:
            pb, pd = self.spec.blocks[j - 1], self.blk[j - 1]
            two = (pb.down[1], pd["ys"]) if pb.down else None
            return (pb.bns[-1], pd["out"], pd["y"][-1], two)
        if self.spec.maxpool:
            return None
        return (self.spec.stem_bn, self.a0, self.y0, None)

    def _bwd_stem(self, arena):
        sp, B = self.spec, self.B
        st = sp.stem_conv
        p, q = st.out_hw
        g = self.blk[0]["gin"] if self.blk else self.dfinal
        if sp.maxpool:
            K.maxpool3s2_bwd(g, self.pidx, self.g0)
            g = self.g0
        self._bn_bwd(sp.stem_bn, arena, g, self.a0, self.y0, self.dy0, B * p * q)
        self._wgrad(st, self.x0, self.dy0)
        tail, self._tail_wgrad = self._tail_wgrad, None
        for cs, x, dy, fold in tail or ():
            self._wgrad_now(cs, x, dy, fold, scratch=(self.wino_wd2, self.wino_wpart2))

    def backward_units(self, arena):
        """The backward pass as (unit key, thunk) in execution order. Unit keys name the
        gradient-arena region each unit finalizes: "fc", "layer<i>.<j>" (one residual block),
        "stem" (conv1 + bn1) — the same keys as parallel/overlap.py:unit_key, so a gradient
        bucket can be pushed as soon as the units that write it have run."""
        units = [("fc", lambda: self._bwd_fc(arena))]
        for j in range(len(self.spec.blocks) - 1, -1, -1):
            key = ".".join(self.spec.blocks[j].convs[0].name.split(".")[:2])
            units.append((key, lambda j=j: self._bwd_block(arena, j)))
        units.append(("stem", lambda: self._bwd_stem(arena)))
        return units

    def backward(self, arena: torch.Tensor):
        for _, fn in self.backward_units(arena):
            fn()
        self.join_side()

    def set_segments(self, groups):
        """Split the backward into segments (lists of unit keys, in backward order) so that a
        callback can run — and a bucket's collective be issued — between them."""
        keys = [k for k, _ in self.backward_units(None)]
        flat = [k for grp in groups for k in grp]
        if flat != keys:
            raise ValueError(f"segments {groups} do not cover the backward units {keys}")
        self.segments = [list(g) for g in groups]
        self.graph = None
        self.graphs = None

    def _segment_fns(self, arena, images_u8, labels_all, unpack):
        units = dict(self.backward_units(arena))
        groups = self.segments or [[k for k, _ in self.backward_units(arena)]]

        def prologue():
            if unpack:
                if self.pre_unpack is not None:
                    self.pre_unpack()
                self.unpack(arena)
            if images_u8 is not None:
                self.load_batch(images_u8, labels_all, train=True)
            self.forward(arena, train=True)
            self.head(arena, backward=True)

        fns = []
        for si, grp in enumerate(groups):
            def seg(grp=grp, first=(si == 0)):
                if first:
                    prologue()
                for k in grp:
                    units[k]()
                self.join_side()  # a segment's gradients are complete when it ends
            fns.append(seg)
        return fns

    def train_step(self, arena: torch.Tensor, images_u8=None, labels_all=None, unpack=True, on_segment=None):
        """unpack (optional) + batch load + forward + loss + backward -> self.grads.
        ``on_segment(i)`` runs after backward segment i has been issued (see set_segments)."""
        for si, fn in enumerate(self._segment_fns(arena, images_u8, labels_all, unpack)):
            fn()
            if on_segment is not None:
                on_segment(si)

    def reset_stat_shift(self):
        """Forget the BN statistic shifts (the previous batch means, see _build): the next step
        sums plainly, as the first step of a fresh engine does."""
        self.bn_shift.zero_()

    # ------------------------------------------------------------------ graphs
    def capture(self, arena, images_u8, labels_all, unpack=True, warmup=2):
        """Capture the step into HIP graphs (one per backward segment, all sharing one memory
        pool); replay with ``step_graph()``."""
        shift = self.bn_shift.clone()  # the warm-up steps' batch means must not become the first replay's shifts
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.train_step(arena, images_u8, labels_all, unpack)
        torch.cuda.current_stream().wait_stream(s)
        self.bn_shift.copy_(shift)
        graphs = []
        for fn in self._segment_fns(arena, images_u8, labels_all, unpack):
            g = torch.cuda.CUDAGraph()
            # thread-local capture: in torch's default (global) mode any other thread's stream
            # synchronize, allocation or copy invalidates the capture (hipErrorStreamCaptureInvalidated,
            # profiles/r6_capture_probe.jsonl) — the co-located async server's comm thread does all
            # three while this worker thread captures its first step (docs/ARCHITECTURE.md)
            with torch.cuda.graph(g, pool=graphs[0].pool() if graphs else None, capture_error_mode="thread_local"):
                fn()
            graphs.append(g)
        self.graphs = graphs
        self.graph = graphs[0]
        return graphs[0]

    def step_graph(self, on_segment=None):
        for si, g in enumerate(self.graphs):
            g.replay()
            if on_segment is not None:
                on_segment(si)

    def evaluate_batch(self, arena, images_u8, labels_all):
        self.load_batch(images_u8, labels_all, train=False)
        self.forward(arena, train=False)
        self.head(arena, backward=False)
