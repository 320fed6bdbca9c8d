"""Thin, allocation-free Python wrappers over the HIP kernel library.

Every function takes pre-allocated torch tensors (device memory), launches on the current
torch stream (so it composes with torch ops and is captured by ``torch.cuda.CUDAGraph``) and
raises on a launch error. Layout conventions: NHWC activations with channels padded to a
16-byte chunk (8 bf16 / 4 fp32 channels); conv weights as ``[OC][Kg]`` implicit-GEMM rows of the
activation dtype (see models/engine.py); fp32 parameter arenas; fp16 (wire codec) or fp32
gradient sinks. The activation dtype (bf16 or fp32, the reference's precision) is taken from
the tensors: every activation kernel is instantiated for both (csrc/kernels/common.hpp).
"""
from __future__ import annotations

import ctypes as C

import torch

from ..utils.tune import tune
from ._lib import check, kernels, ptr, stream_ptr

def conv_out_hw(h: int, w: int, k: int, stride: int, pad: int):
    return (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1


STAT_SLOTS = 8  # PSX_STAT_SLOTS in csrc/kernels/common.hpp


_ZERO_PAGES = {}


_DET_ON = False


def det_slot_scale() -> int:
    """Size factor of every BN slot buffer in deterministic mode: entry i of the float layout
    [STAT_SLOTS][NS][C] becomes a 16-byte fixed-point pair (csrc/kernels/bnfin.hpp DetRed)."""
    return int(kernels().psx_det_slot_scale())


def set_deterministic(on) -> None:
    """Deterministic BN reductions (csrc/kernels/bnfin.hpp DetRed: exact fixed-point pairs in the
    slot buffers, order-independent) on or off. Every slot buffer handed to a kernel while it is
    on must be det_slot_scale() times the float layout and zeroed like the float one. Host state
    of the kernel library: set it before capturing a HIP graph."""
    global _DET_ON
    _DET_ON = bool(on)
    check(kernels().psx_set_deterministic(int(_DET_ON)), "set_deterministic")


def deterministic() -> bool:
    return _DET_ON


def det_slot_values(buf, shape):
    """Decode a deterministic-mode slot buffer: float64 values of its fixed-point pairs in the
    float layout ``shape`` (e.g. (STAT_SLOTS, 2, C)); NaN where a partial was not finite."""
    n = 1
    for d in shape:
        n *= int(d)
    qi = buf.reshape(-1).view(torch.int64)[:2 * n].view(n, 2)
    poison = qi[:, 1] < 0  # bit 63 of the low word (bnfin.hpp kFixPoison): a non-finite partial
    q = qi.double()
    lo = q[:, 1]  # legitimate low words stay below 2^56 (positive as int64)
    v = q[:, 0] * 2.0 ** -24 + lo * 2.0 ** -64
    return torch.where(poison, torch.full_like(v, float("nan")), v).view(*shape)


def is_f32(t) -> int:
    """1 when an activation / operand tensor is fp32 (the fp32 compute path), 0 for bf16."""
    if t.dtype == torch.float32:
        return 1
    if t.dtype == torch.bfloat16:
        return 0
    raise TypeError(f"activation dtype {t.dtype} (expected bfloat16 or float32)")


def zero_page(device=None):
    """16-byte-aligned zero block used as the DMA source for conv padding (conv v2)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    z = _ZERO_PAGES.get(dev)
    if z is None:
        z = torch.zeros(64, dtype=torch.uint8, device=dev)
        _ZERO_PAGES[dev] = z
    return z


def conv2_workspace_bytes(nb, oh, ow, oc, kg, f32=False) -> int:
    return int(kernels().psx_conv2_workspace(nb, oh, ow, oc, kg, int(bool(f32))))


class BnFin(C.Structure):
    """csrc/kernels/bnfin.hpp BnFin: in-launch forward BN finalize descriptor."""
    _fields_ = [("gamma", C.c_void_p), ("beta", C.c_void_p), ("run_mean", C.c_void_p), ("run_var", C.c_void_p),
                ("scale", C.c_void_p), ("shift", C.c_void_p), ("save_mean", C.c_void_p),
                ("save_invstd", C.c_void_p), ("counter", C.c_void_p), ("count", C.c_float), ("eps", C.c_float),
                ("momentum", C.c_float), ("C", C.c_int), ("sshift", C.c_void_p), ("sshift_next", C.c_void_p),
                ("det", C.c_int)]  # det: set by the launcher (deterministic mode)


class BnBwdFin(C.Structure):
    """csrc/kernels/bnfin.hpp BnBwdFin: in-launch backward BN finalize descriptor."""
    _fields_ = [("gamma", C.c_void_p), ("mean", C.c_void_p), ("invstd", C.c_void_p), ("coef", C.c_void_p),
                ("dgamma", C.c_void_p), ("dbeta", C.c_void_p), ("counter", C.c_void_p), ("count", C.c_float),
                ("gscale", C.c_float), ("C", C.c_int), ("grad_fp16", C.c_int), ("det", C.c_int)]


def bn_fin(gamma, beta, run_mean, run_var, affine, saved, counter_ptr, count, eps, momentum, c, sshift=None,
           sshift_next=None) -> BnFin:
    """affine: [2, C] (scale, shift); saved: [2, C] (mean, invstd). sshift / sshift_next [C]
    (optional): the statistics are shifted sums around sshift (what the producers were given);
    the finalize writes the batch mean to sshift_next (csrc/kernels/bnfin.hpp BnFin)."""
    a, sv = ptr(affine), ptr(saved)
    return BnFin(ptr(gamma), ptr(beta), ptr(run_mean), ptr(run_var), a, a + 4 * c, sv, sv + 4 * c, counter_ptr,
                 float(count), float(eps), float(momentum), int(c), ptr(sshift), ptr(sshift_next))


def bn_bwd_fin(gamma, saved, coef, dgamma_ptr, dbeta_ptr, counter_ptr, count, gscale, c, grad_fp16) -> BnBwdFin:
    sv = ptr(saved)
    return BnBwdFin(ptr(gamma), sv, sv + 4 * c, ptr(coef), dgamma_ptr, dbeta_ptr, counter_ptr, float(count),
                    float(gscale), int(c), int(grad_fp16))


def conv_fwd2(x, wf, y, stats, ws, nb, h, w, ic, oc, k, stride, pad, kg, fin: BnFin | None = None, sshift=None):
    """LDS-DMA pipelined implicit-GEMM conv (csrc/kernels/conv_v2.hip); ws: fp32 split-K
    workspace of >= conv2_workspace_bytes(...) bytes (or None when that is 0). With ``fin`` the
    kernel's last workgroup also finalizes the BN layer its statistics feed (bnfin.hpp).
    sshift [oc] (optional): the BN statistics are sums of (y - sshift) and (y - sshift)^2."""
    check(kernels().psx_conv_fwd2(ptr(x), ptr(wf), ptr(y), ptr(stats), ptr(zero_page(x.device)), ptr(ws), nb, h, w,
                                  ic, oc, k, k, stride, pad, kg, C.byref(fin) if fin is not None else None,
                                  is_f32(x), ptr(sshift), stream_ptr()), "conv_fwd2")


def stem_conv(x, wf, y, stats, nb, h, w, cin, cp, oc, kg, sshift=None, k=3) -> bool:
    """A 3-channel stem conv with its BN statistics (csrc/kernels/stem.hip), same operands as
    conv_fwd2: k = 3 the CIFAR stem (3 -> 64, 3x3 / stride 1 / pad 1, direct vector-ALU conv;
    not in deterministic mode), k = 7 the ImageNet stem (3 -> 64, 7x7 / stride 2 / pad 3,
    224 -> 112, on the MFMA with the input patch in LDS; fp32 or bf16). False: not this shape (run
    conv_fwd2 instead)."""
    if k == 7:
        rc = kernels().psx_stem7_conv(ptr(x), ptr(wf), ptr(y), ptr(stats), ptr(sshift), nb, h, w, cin, cp, oc, kg,
                                      is_f32(x), stream_ptr())
    else:
        rc = kernels().psx_stem_conv(ptr(x), ptr(wf), ptr(y), ptr(stats), ptr(sshift), nb, h, w, cin, cp, oc, kg,
                                     is_f32(x), stream_ptr())
    if rc == -11:
        return False
    check(rc, "stem_conv")
    return True


class BwdStatsDesc(C.Structure):
    """csrc/kernels/conv_v2.hip BwdStatsDesc: fused BN-backward reduction over a dgrad output."""
    _fields_ = [("part", C.c_void_p), ("o", C.c_void_p), ("y1", C.c_void_p), ("y2", C.c_void_p),
                ("saved1", C.c_void_p), ("saved2", C.c_void_p), ("mask_store", C.c_int),
                ("mask_aff", C.c_void_p)]


def bwd_stats_desc(part, o, y1, saved1, y2=None, saved2=None, mask_store=False, mask_aff=None) -> BwdStatsDesc:
    """``mask_store`` (dgrad only): the epilogue stores dz = g * [o > 0] instead of g, so the BN
    backward apply reading it runs without the mask operand o. ``mask_aff`` (Winograd data
    gradient only; o = None): the ReLU mask is [y1 * scale + shift > 0] with the BN affine
    [2][C] — the layer whose post-ReLU activation was never written (wino_conv ``bn_in``)."""
    assert o is not None or mask_aff is not None
    return BwdStatsDesc(ptr(part), ptr(o), ptr(y1), ptr(y2), ptr(saved1), ptr(saved2), int(bool(mask_store)),
                        ptr(mask_aff))


def conv_dgrad2(dy, wd, dx, res, ws, nb, h, w, ic_fwd, oc_fwd, k, stride, pad, kgd, bst: BwdStatsDesc | None = None):
    """With ``bst`` the epilogue also produces the BN-backward slot sums of dx (what
    bn_bwd_reduce would compute), so that pass can be skipped."""
    check(kernels().psx_conv_dgrad2(ptr(dy), ptr(wd), ptr(dx), ptr(res), ptr(zero_page(dy.device)), ptr(ws), nb, h,
                                    w, ic_fwd, oc_fwd, k, k, stride, pad, kgd,
                                    C.byref(bst) if bst is not None else None, is_f32(dy), stream_ptr()), "conv_dgrad2")


def conv_dgrad2_sc(dy, wd, dx, ws, nb, h, w, ic_fwd, oc_fwd, kgd, dy_sc, wd_sc, kgd_sc,
                   bst: BwdStatsDesc | None = None) -> bool:
    """The 3x3 / stride-2 / pad-1 data gradient with the block's 1x1 / stride-2 shortcut folded
    in: dx = dgrad(dy, wd) + dgrad_sc(dy_sc, wd_sc) in one launch (csrc/kernels/conv_v2.hip
    psx_conv_dgrad2_sc). False: this layer cannot fold (run the two launches instead)."""
    rc = kernels().psx_conv_dgrad2_sc(ptr(dy), ptr(wd), ptr(dx), None, ptr(zero_page(dy.device)), ptr(ws), nb, h, w,
                                      ic_fwd, oc_fwd, 3, 3, 2, 1, kgd, C.byref(bst) if bst is not None else None,
                                      is_f32(dy), ptr(dy_sc), ptr(wd_sc), kgd_sc, stream_ptr())
    if rc == -11:
        return False
    check(rc, "conv_dgrad2_sc")
    return True


def bgemm_f32(a, b, p, m, n, kd, nb, cfg=0):
    """nb batched fp32 GEMMs p[i] = a[i] @ b[:, i, :].T (a [nb][m][kd], b [n][nb][kd], p [nb][m][n];
    kd a power of two >= 32) on the conv_v2 mainloop (csrc/kernels/conv_v2.hip psx_bgemm_f32)."""
    assert a.dtype == b.dtype == p.dtype == torch.float32
    assert a.numel() >= m * nb * kd and b.numel() >= n * nb * kd and p.numel() >= nb * m * n
    check(kernels().psx_bgemm_f32(ptr(a), ptr(b), ptr(p), ptr(zero_page(a.device)), m, n, kd, nb, cfg, stream_ptr()),
          "bgemm_f32")


def bgemm_tn_f32(x, d, part, t, c, k, nb, q=1, br=64, bc=64):
    """Batched TN GEMMs part[i * q + j] = d[i, range j].T @ x[i, range j] (x [nb][t][c],
    d [nb][t][k], part [nb*q][k][c]) on the fp32 weight-gradient mainloop (wgrad_v2.hip)."""
    assert x.dtype == d.dtype == part.dtype == torch.float32
    assert x.numel() >= nb * t * c and d.numel() >= nb * t * k and part.numel() >= nb * q * k * c
    check(kernels().psx_bgemm_tn_f32(ptr(x), ptr(d), ptr(part), ptr(zero_page(x.device)), t, c, k, nb, q, br, bc,
                                     stream_ptr()), "bgemm_tn_f32")


def wino_ok(h, w, c, k) -> bool:
    return bool(kernels().psx_wino_ok(h, w, c, k))


def wino_v_floats(nb, h, w, c) -> int:
    """Floats of a layer's transformed operand [36][T][c] (T = nb * h/4 * w/4 tiles)."""
    return int(kernels().psx_wino_v_floats(nb, h, w, c))


def wino_p_floats(nb, h, w, c, k) -> int:
    """Floats of wino_conv's GEMM output P (36 x T x k x its reduction split; c = input channels)."""
    return int(kernels().psx_wino_p_floats(nb, h, w, c, k))


def wino_workspace_floats(nb, h, w, c, k) -> int:
    return int(kernels().psx_wino_workspace(nb, h, w, c, k))


def wino_wgrad_q(nb, h, w, c, k) -> int:
    """Tile-range splits of the Winograd weight-gradient GEMM (0: not applicable)."""
    return int(kernels().psx_wino_wgrad_q(nb, h, w, c, k))


def wino_weights(w_oihw, u, k, c, flip=False):
    """Winograd F(4x4,3x3) weight transform (csrc/kernels/wino.hip): forward U[k][36][c] from the
    fp32 OIHW weights, or (flip) the data-gradient operand U[c][36][k] of rot180(w)^T."""
    assert w_oihw.dtype == torch.float32 and w_oihw.numel() == k * c * 9 and u.numel() >= 36 * k * c
    check(kernels().psx_wino_weights(ptr(w_oihw), ptr(u), k, c, int(bool(flip)), stream_ptr()), "wino_weights")


class WinoWeightBatch:
    """Every Winograd weight transform of a step as ONE launch (wino.hip psx_wino_weights_multi):
    items = [(w_oihw, u, k, c, flip[, layout])], pointers fixed at construction (<= 40 items).
    layout 1: the fused kernel's operand order (wino_fused; 40 * k * c floats)."""

    def __init__(self, items):
        n = len(items)
        assert 1 <= n <= 40
        for w, u, k, c, *rest in items:
            lay = rest[1] if len(rest) > 1 else 0
            assert w.dtype == torch.float32 and w.numel() == k * c * 9 and u.numel() >= (40 if lay else 36) * k * c
        self.n = n
        self.keep = [(it[0], it[1]) for it in items]
        self.w = (C.c_void_p * n)(*[ptr(it[0]) for it in items])
        self.u = (C.c_void_p * n)(*[ptr(it[1]) for it in items])
        self.k = (C.c_int * n)(*[int(it[2]) for it in items])
        self.c = (C.c_int * n)(*[int(it[3]) for it in items])
        self.flip = (C.c_int * n)(*[int(bool(it[4])) for it in items])
        self.layout = (C.c_int * n)(*[int(it[5]) if len(it) > 5 else 0 for it in items])

    def __call__(self):
        check(kernels().psx_wino_weights_multi(self.w, self.u, self.k, self.c, self.flip, self.n, self.layout,
                                               stream_ptr()), "wino_weights_multi")


def wino_fused_ok(nb, h, w, c, k) -> bool:
    """psx_wino_fused handles this layer (csrc/kernels/wino_fused.hip: 64 or 128 input channels,
    output channels a multiple of 64, whole 16-tile blocks)."""
    return bool(kernels().psx_wino_fused_ok(nb, h, w, c, k))


def wino_fused(x, uf, y, res, stats, v, nb, h, w, c, k, bst: "BwdStatsDesc | None" = None, bn_in=None, sshift=None,
               bwd_in=None):
    """wino_conv in ONE launch (csrc/kernels/wino_fused.hip: input transform, 36 GEMMs and output
    transform fused; V / P never reach HBM). uf: the transformed weights in layout 1
    (WinoWeightBatch item layout=1, 40 * k * c floats); v (nullable): receives the transformed input [36][T][c] for
    wino_wgrad. The other arguments as wino_conv. bwd_in = (y, part, BnBwdFin) (data gradient):
    x is dz of a BN whose backward apply is folded into the operand loads, dy = k1 dz + k2 y + k3
    from the slot sums ``part`` [STAT_SLOTS][2][c]; the launch writes the BnBwdFin's coefficients
    and dgamma / dbeta."""
    assert x.dtype == torch.float32 and y.dtype == torch.float32
    assert x.numel() == nb * h * w * c and y.numel() == nb * h * w * k and uf.numel() >= 40 * k * c
    assert v is None or v.numel() >= wino_v_floats(nb, h, w, c)
    assert res is None or res.numel() == y.numel()
    check(kernels().psx_wino_fused(ptr(x), ptr(uf), ptr(y), ptr(res), ptr(stats), ptr(v), nb, h, w, c, k,
                                   C.byref(bst) if bst is not None else None,
                                   ptr(bn_in[0]) if bn_in is not None else None,
                                   C.byref(bn_in[1]) if bn_in is not None else None, ptr(sshift),
                                   ptr(bwd_in[0]) if bwd_in is not None else None,
                                   ptr(bwd_in[1]) if bwd_in is not None else None,
                                   C.byref(bwd_in[2]) if bwd_in is not None else None, stream_ptr()),
          "wino_fused")


def wino_conv(x, u, y, res, stats, v, p, nb, h, w, c, k, cfg=None, bst: "BwdStatsDesc | None" = None, bn_in=None,
              sshift=None):
    """fp32 3x3/s1/p1 conv y = conv(x) (+ res) via Winograd F(4x4,3x3) with pre-transformed
    weights u (wino_weights); stats: BN slot sums of y (pre-zeroed) or None; bst (data gradient,
    bwd_stats_desc): the consumer BN's backward sums (and the masked store) instead. v (>=
    wino_v_floats of c) receives the transformed input (kept for wino_wgrad), p (>= wino_v_floats
    of k) is scratch. bn_in = (slot rows [STAT_SLOTS][2][c], BnFin): x is the previous layer's
    pre-BN output; its training-mode BN finalize + BN + ReLU are folded into the input transform
    (the BnFin's affine / saved / running statistics are written by the launch)."""
    assert x.dtype == torch.float32 and y.dtype == torch.float32
    assert x.numel() == nb * h * w * c and y.numel() == nb * h * w * k and u.numel() >= 36 * k * c
    assert v.numel() >= wino_v_floats(nb, h, w, c) and p.numel() >= wino_p_floats(nb, h, w, c, k)
    assert res is None or res.numel() == y.numel()
    check(kernels().psx_wino_conv(ptr(x), ptr(u), ptr(y), ptr(res), ptr(stats), ptr(v), ptr(p), ptr(zero_page(x.device)),
                                  nb, h, w, c, k, 0 if cfg is None else cfg,
                                  C.byref(bst) if bst is not None else None,
                                  ptr(bn_in[0]) if bn_in is not None else None,
                                  C.byref(bn_in[1]) if bn_in is not None else None, ptr(sshift), stream_ptr()),
          "wino_conv")


def wino_wgrad(v, dy, d, part, out, nb, h, w, c, k, scale=1.0, bwd_in=None):
    """Weight gradient of a wino_conv layer from its transformed input v and dy [nb][h][w][k]:
    out (OIHW, fp16 wire or fp32) = scale * dW. d: >= wino_v_floats(k) scratch, part:
    36 * q * k * c floats (q = wino_wgrad_q). bwd_in = (y, part, BnBwdFin): dy is dz of a BN whose
    backward apply is folded into the dy transform (as wino_fused's bwd_in; this launch writes
    nothing of the BnBwdFin)."""
    q = wino_wgrad_q(nb, h, w, c, k)
    assert q > 0 and dy.dtype == torch.float32 and dy.numel() == nb * h * w * k
    assert d.numel() >= wino_v_floats(nb, h, w, k) and part.numel() >= 36 * q * k * c
    assert out.dtype in (torch.float16, torch.float32) and out.numel() >= k * c * 9
    check(kernels().psx_wino_wgrad(ptr(v), ptr(dy), ptr(d), ptr(part), ptr(out), int(out.dtype == torch.float16),
                                   float(scale), ptr(zero_page(dy.device)), nb, h, w, c, k,
                                   ptr(bwd_in[0]) if bwd_in is not None else None,
                                   ptr(bwd_in[1]) if bwd_in is not None else None,
                                   C.byref(bwd_in[2]) if bwd_in is not None else None, stream_ptr()), "wino_wgrad")


def wino_wgrad_fused_q(nb, h, w, c, k) -> int:
    """Tile ranges of the fused Winograd weight gradient (csrc/kernels/wino_wgrad.hip; 0: not
    applicable): its partial slabs take 36 * q * k * c floats."""
    return int(kernels().psx_wino_wgrad_fused_q(nb, h, w, c, k))


def wino_wgrad_fused(x, dy, part, out, nb, h, w, c, k, scale=1.0, xaff=None, bwd_in=None):
    """Weight gradient of a 3x3 / stride-1 / pad-1 fp32 conv in one fused Winograd launch
    (csrc/kernels/wino_wgrad.hip: x and dy transformed in registers, 36 tile-reduction GEMMs on
    the f32 MFMA; neither V nor D in HBM) + the output transform. x [nb][h][w][c] is the conv
    input, or with xaff ([2][c] scale, shift) the pre-BN y whose BN + ReLU the forward folded
    into its input transform (x = relu(scale y + shift)). dy [nb][h][w][k]; bwd_in = (y, part,
    BnBwdFin) as wino_wgrad. part: >= 36 * q * k * c floats (q = wino_wgrad_fused_q). out: OIHW
    gradient (fp16 wire or fp32) = scale * dW."""
    q = wino_wgrad_fused_q(nb, h, w, c, k)
    assert q > 0 and x.dtype == torch.float32 and dy.dtype == torch.float32
    assert x.numel() == nb * h * w * c and dy.numel() == nb * h * w * k
    assert part.numel() >= 36 * q * k * c and out.dtype in (torch.float16, torch.float32) and out.numel() >= k * c * 9
    assert xaff is None or (xaff.dtype == torch.float32 and xaff.numel() >= 2 * c)
    check(kernels().psx_wino_wgrad_fused(ptr(x), ptr(xaff), ptr(dy),
                                         ptr(bwd_in[0]) if bwd_in is not None else None,
                                         ptr(bwd_in[1]) if bwd_in is not None else None,
                                         C.byref(bwd_in[2]) if bwd_in is not None else None, ptr(part), ptr(out),
                                         int(out.dtype == torch.float16), float(scale), nb, h, w, c, k, stream_ptr()),
          "wino_wgrad_fused")


def conv_wgrad2_splits(nb, h, w, ic, oc, k, stride, pad, kg, f32=False) -> int:
    n = kernels().psx_conv_wgrad2(None, None, None, None, nb, h, w, ic, oc, k, k, stride, pad, kg, int(bool(f32)), None)
    if n <= 0:
        raise RuntimeError(f"conv_wgrad2 split query failed ({n})")
    return n


def conv_wgrad2(x, dy, part, nb, h, w, ic, oc, k, stride, pad, kg) -> int:
    """LDS-DMA pipelined weight gradient (csrc/kernels/wgrad_v2.hip) -> fp32 split slabs in part."""
    n = kernels().psx_conv_wgrad2(ptr(x), ptr(dy), ptr(part), ptr(zero_page(x.device)), nb, h, w, ic, oc, k, k,
                                  stride, pad, kg, is_f32(x), stream_ptr())
    if n <= 0:
        raise RuntimeError(f"conv_wgrad2 failed ({n})")
    return n


def wgrad_reduce(part, splits, oc, kg, cin, ic, k, scale, out_ptr: int, out_fp16: bool):
    """Reduce the split slabs into the OIHW gradient. CONSUMES ``part``: a layer with few
    columns and many splits (the stem) is pre-summed in place (csrc/kernels/wgrad_reduce.hip
    wgrad_presum_kernel), so reduce a given set of partials once."""
    check(kernels().psx_wgrad_reduce(ptr(part), splits, oc, kg, cin, ic, k, k, float(scale), out_ptr, int(out_fp16),
                                     stream_ptr()), "wgrad_reduce")


WRBATCH_MAX = 4


def wgrad_reduce_batchable(ic, k) -> bool:
    """The v2 reduce handles the layer (what wgrad_reduce_batch requires)."""
    return k * k <= 49 and ic % 16 == 0


def wgrad_reduce_batch(items, scale, out_fp16: bool):
    """One launch reducing up to WRBATCH_MAX layers' split-K partials; items = [(part, splits,
    oc, kg, cin, ic, k, out_ptr)] (see wgrad_reduce), each wgrad_reduce_batchable."""
    n = len(items)
    assert 1 <= n <= WRBATCH_MAX
    P = (C.c_void_p * n)(*[ptr(it[0]) for it in items])
    O = (C.c_void_p * n)(*[it[7] for it in items])

    def ints(j, f=lambda v: v):
        return (C.c_int * n)(*[int(f(it[j])) for it in items])

    check(kernels().psx_wgrad_reduce_batch(n, P, O, ints(1), ints(2), ints(3), ints(4), ints(5),
                                           ints(6, lambda k: k * k), float(scale), int(out_fp16), stream_ptr()),
          "wgrad_reduce_batch")


def bn_finalize(part, T, c, count, gamma, beta, eps, momentum, run_mean, run_var, affine, saved, sshift=None,
                sshift_next=None):
    """affine: [2, C] (scale, shift); saved: [2, C] (mean, invstd); sshift / sshift_next: as bn_fin."""
    check(kernels().psx_bn_finalize(ptr(part), T, c, float(count), ptr(gamma), ptr(beta), float(eps),
                                    float(momentum), ptr(run_mean), ptr(run_var), ptr(affine), ptr(affine) + 4 * c,
                                    ptr(saved), ptr(saved) + 4 * c, ptr(sshift), ptr(sshift_next), stream_ptr()),
          "bn_finalize")


def bn_eval_affine(c, gamma, beta, rm, rv, eps, affine):
    check(kernels().psx_bn_eval_affine(c, ptr(gamma), ptr(beta), ptr(rm), ptr(rv), float(eps), ptr(affine),
                                       ptr(affine) + 4 * c, stream_ptr()), "bn_eval_affine")


def bn_apply(y, affine, out, c, relu=True, res=None, affine2=None):
    mode = 0 if res is None else (1 if affine2 is None else 2)
    a2 = ptr(affine2)
    check(kernels().psx_bn_apply(ptr(y), ptr(affine), ptr(affine) + 4 * c, ptr(res), a2,
                                 (a2 + 4 * c) if a2 else None, ptr(out), y.numel(), c, mode, int(relu),
                                 is_f32(y), stream_ptr()), "bn_apply")


def bn_apply_fin(y, part1, fin1: BnFin, out, c, relu=True, res=None, part2=None, fin2: BnFin | None = None):
    """Training-mode bn_apply with the finalize folded in: every workgroup computes the affine
    from the [STAT_SLOTS][2][C] slot sums (part1; part2/fin2 = the shortcut BN, mode 2) and
    workgroup 0 writes fin1/fin2's side outputs (csrc/kernels/bnfin.hpp bn_fin_lds)."""
    mode = 0 if res is None else (1 if part2 is None else 2)
    check(kernels().psx_bn_apply_fin(ptr(y), ptr(part1), C.byref(fin1), ptr(res), ptr(part2),
                                     C.byref(fin2) if fin2 is not None else None, ptr(out), y.numel(), c, mode,
                                     int(relu), is_f32(y), stream_ptr()), "bn_apply_fin")


def bn_bwd_reduce_T(npix: int, c: int) -> int:
    return kernels().psx_bn_bwd_reduce(None, None, None, None, None, None, None, None, None, npix, c, None, None,
                                       0, None)


def bn_bwd_reduce(g, o, y1, saved1, part, npix, c, y2=None, saved2=None, fin1: BnBwdFin | None = None,
                  fin2: BnBwdFin | None = None) -> int:
    """With fin1 (and fin2 for the shared-dz pair) the last block also runs the backward
    finalize (coefficients + dgamma/dbeta), see csrc/kernels/bnfin.hpp."""
    s2 = ptr(saved2)
    T = kernels().psx_bn_bwd_reduce(ptr(g), ptr(o), ptr(y1), ptr(saved1), ptr(saved1) + 4 * c, ptr(y2), s2,
                                    (s2 + 4 * c) if s2 else None, ptr(part), npix, c,
                                    C.byref(fin1) if fin1 is not None else None,
                                    C.byref(fin2) if fin2 is not None else None, is_f32(g), stream_ptr())
    if T <= 0:
        raise RuntimeError(f"bn_bwd_reduce failed ({T})")
    return T


def bn_bwd_finalize(part, T, ns, which, c, count, gamma, saved, coef, dgamma_ptr, dbeta_ptr, gscale, grad_fp16):
    check(kernels().psx_bn_bwd_finalize(ptr(part), T, ns, which, c, float(count), ptr(gamma), ptr(saved),
                                        ptr(saved) + 4 * c, ptr(coef), dgamma_ptr, dbeta_ptr, float(gscale),
                                        int(grad_fp16), stream_ptr()), "bn_bwd_finalize")


def bn_bwd_apply(g, o, y1, coef1, dx1, c, y2=None, coef2=None, dx2=None, dzout=None):
    check(kernels().psx_bn_bwd_apply(ptr(g), ptr(o), ptr(y1), ptr(coef1), ptr(dx1), ptr(y2), ptr(coef2), ptr(dx2),
                                     ptr(dzout), g.numel(), c, is_f32(g), stream_ptr()), "bn_bwd_apply")


def bn_bwd_apply_fin(g, o, y1, part, fin1: BnBwdFin, dx1, c, y2=None, fin2: BnBwdFin | None = None, dx2=None,
                     dzout=None):
    """bn_bwd_apply with the backward finalize folded in (coefficients from the
    [STAT_SLOTS][NS][C] slot sums per workgroup; workgroup 0 writes coef and dgamma/dbeta)."""
    check(kernels().psx_bn_bwd_apply_fin(ptr(g), ptr(o), ptr(y1), ptr(part), C.byref(fin1), ptr(dx1), ptr(y2),
                                         C.byref(fin2) if fin2 is not None else None, ptr(dx2), ptr(dzout),
                                         g.numel(), c, is_f32(g), stream_ptr()), "bn_bwd_apply_fin")


def head_fwd_bwd(act, b, hw, c, fcw, fcb, k, labels, pooled, dlogits, dact, loss, correct,
                 bst: BwdStatsDesc | None = None) -> bool:
    """``bst``: also produce the BN-backward sums of the layer whose output ``act`` is (fused
    per-sample head only). Returns whether they were produced."""
    r = kernels().psx_head_fwd_bwd(ptr(act), b, hw, c, ptr(fcw), ptr(fcb), k, ptr(labels), ptr(pooled),
                                   ptr(dlogits), ptr(dact), ptr(loss), ptr(correct),
                                   C.byref(bst) if bst is not None else None, is_f32(act), stream_ptr())
    check(min(r, 0), "head_fwd_bwd")
    return r == 1


def head_wgrad(dlogits, pooled, b, k, c, dw_ptr, db_ptr, gscale, grad_fp16):
    check(kernels().psx_head_wgrad(ptr(dlogits), ptr(pooled), b, k, c, dw_ptr, db_ptr, float(gscale),
                                   int(grad_fp16), stream_ptr()), "head_wgrad")


def sgd_apply(p, g, lr, gscale=1.0, momentum=0.0, wd=0.0, buf=None, first=False, n=None, img=None):
    """p -= lr*(gscale*g + wd*p) [momentum]; ``img`` (bf16, >= n elements) also receives the
    bf16 bits of the updated parameters in the same pass (fetch wire / weight image)."""
    n = p.numel() if n is None else n
    fp16 = g.dtype == torch.float16
    if img is not None:
        assert img.dtype == torch.bfloat16 and img.numel() >= n and img.device == p.device, "sgd_apply img"
    check(kernels().psx_sgd_apply(ptr(p), ptr(g), ptr(buf), n, float(lr), float(gscale), float(momentum), float(wd),
                                  int(first), int(fp16), ptr(img), stream_ptr()), "sgd_apply")


def sgd_apply_multi(p, srcs, lr, gscale=1.0, momentum=0.0, wd=0.0, buf=None, first=False, n=None, img=None):
    """p -= lr*(gscale * sum_k srcs[k] + wd*p) [momentum]: the sync round's update from the W
    gathered wires, decoded and summed in fp32 in list order (reference decompress + aggregate +
    apply, server.py:126-169,232-237). All sources fp16 or all fp32; at most 32."""
    n = p.numel() if n is None else n
    assert 1 <= len(srcs) <= 32
    fp16 = srcs[0].dtype == torch.float16
    assert all(s.dtype == srcs[0].dtype and s.numel() >= n and s.device == p.device for s in srcs), "sgd_apply_multi"
    if img is not None:
        assert img.dtype == torch.bfloat16 and img.numel() >= n and img.device == p.device, "sgd_apply_multi img"
    arr = (C.c_void_p * len(srcs))(*[s.data_ptr() for s in srcs])
    check(kernels().psx_sgd_apply_multi(ptr(p), arr, len(srcs), ptr(buf), n, float(lr), float(gscale), float(momentum),
                                        float(wd), int(first), int(fp16), ptr(img), stream_ptr()), "sgd_apply_multi")


def maxpool3s2_fwd(x, y, arg):
    """3x3/s2/p1 max-pool, NHWC bf16 or fp32; arg (uint8, y's shape) keeps the window argmax."""
    B, H, W, C = x.shape
    check(kernels().psx_maxpool3s2_fwd(ptr(x), ptr(y), ptr(arg), B, H, W, C, is_f32(x), stream_ptr()),
          "maxpool3s2_fwd")


def maxpool3s2_bwd(dy, arg, dx):
    B, H, W, C = dx.shape
    check(kernels().psx_maxpool3s2_bwd(ptr(dy), ptr(arg), ptr(dx), B, H, W, C, is_f32(dy), stream_ptr()),
          "maxpool3s2_bwd")


def topk_workspace_words(n: int) -> int:
    return kernels().psx_topk_workspace_words(int(n))


def topk_payload_words(kcap: int) -> int:
    return kernels().psx_topk_payload_words(int(kcap))


def topk_encode(g, resid, k, kcap, payload, ws):
    """Error-feedback top-k of (resid + g) into payload (csrc/kernels/topk.hip); g may be None."""
    fp16 = g is not None and g.dtype == torch.float16
    check(kernels().psx_topk_encode(ptr(g), int(fp16), ptr(resid), resid.numel(), int(k), int(kcap), ptr(payload),
                                    ptr(ws), stream_ptr()), "topk_encode")


def topk_decode_add(payload, dst, scale, kcap):
    """dst[idx] += scale * val for every (idx, val) of a top-k payload."""
    check(kernels().psx_topk_decode_add(ptr(payload), ptr(dst), float(scale), int(kcap), stream_ptr()),
          "topk_decode_add")


def grad_aggregate(srcs_dev_ptrs, nsrc, src_fp16, dst, n, scale=1.0, accumulate=False):
    """srcs_dev_ptrs: int64 device tensor holding nsrc device pointers."""
    check(kernels().psx_grad_aggregate(ptr(srcs_dev_ptrs), nsrc, int(src_fp16), ptr(dst),
                                       int(dst.dtype == torch.float16), n, float(scale), int(accumulate),
                                       stream_ptr()), "grad_aggregate")


def fp16_pack(src, dst, scale=1.0):
    check(kernels().psx_fp16_pack(ptr(src), ptr(dst), src.numel(), float(scale), stream_ptr()), "fp16_pack")


def fp16_unpack(src, dst, scale=1.0):
    check(kernels().psx_fp16_unpack(ptr(src), ptr(dst), src.numel(), float(scale), stream_ptr()), "fp16_unpack")


def param_unpack(arena, descs_dev, ndesc, wbuf):
    check(kernels().psx_param_unpack(ptr(arena), ptr(descs_dev), ndesc, ptr(wbuf), stream_ptr()), "param_unpack")


def param_unpack_tiles(src, descs_dev, ndesc, ntiles, wbuf, scatter=None):
    """Flat-grid unpack (one workgroup per 64x64 tile x 3-tap chunk of every conv). ``src`` is
    the fp32 arena or a bf16 weight image with the same element offsets; descs carry each conv's
    first tile. ``wbuf``'s dtype picks the operand type (bf16, or fp32 from an fp32 source). ``scatter = (src_f32, idx_i64, dst_f32, gather[, sidx_i64])``: extra workgroups
    of the same launch write dst[idx[j]] = src[j] (gather False), src[idx[j]] (gather True) or
    src[sidx[j]] (sidx given: the sharded wire's padded per-rank blocks)."""
    assert src.dtype in (torch.float32, torch.bfloat16), src.dtype
    sc = (None, None, 0, None, 0, None)
    if scatter is not None:
        s_src, s_idx, s_dst, gather = scatter[:4]
        sidx = scatter[4] if len(scatter) > 4 else None
        assert s_src.dtype == torch.float32 and s_dst.dtype == torch.float32 and s_idx.dtype == torch.int64
        assert s_src.device == s_dst.device == s_idx.device == src.device
        n = s_idx.numel()
        if sidx is not None:
            assert sidx.dtype == torch.int64 and sidx.numel() == n and sidx.device == src.device
        else:
            assert gather or s_src.numel() >= n
        sc = (ptr(s_src), ptr(s_idx), n, ptr(s_dst), int(bool(gather)), ptr(sidx) if sidx is not None else None)
    check(kernels().psx_param_unpack_tiles(ptr(src), int(src.dtype == torch.bfloat16), ptr(descs_dev), ndesc,
                                           int(ntiles), ptr(wbuf), *sc, is_f32(wbuf), stream_ptr()),
          "param_unpack_tiles")


def unpack_desc_size() -> int:
    return kernels().psx_unpack_desc_size()


def synth_gen(img, labels, n, h, w, classes, seed, offset=0):
    check(kernels().psx_synth_gen(ptr(img), ptr(labels), n, h, w, classes, seed & 0xFFFFFFFF, offset & 0xFFFFFFFF,
                                  stream_ptr()), "synth_gen")


_F3 = C.c_float * 3


def augment(img, labels, index, out, out_labels, b, h, w, pad, seed, step_dev, train, mean, std, zero=None,
            copy=None):
    """zero: up to two contiguous tensors of 32-bit elements zeroed by the same launch; copy:
    (src, dst) 32-bit tensors of equal size copied by it (the BN statistic shifts)."""
    zs = []
    for t in zero or ():
        assert t.is_contiguous() and t.element_size() == 4 and t.device == out.device
        zs += [ptr(t), t.numel()]
    zs += [None, 0] * (2 - len(zs) // 2)
    cp = [None, None, 0]
    if copy is not None:
        src, dst = copy
        assert src.numel() == dst.numel() and src.element_size() == dst.element_size() == 4
        assert src.is_contiguous() and dst.is_contiguous()
        cp = [ptr(src), ptr(dst), src.numel()]
    check(kernels().psx_augment(ptr(img), ptr(labels), ptr(index), ptr(out), ptr(out_labels), b, h, w, pad,
                                seed & 0xFFFFFFFF, ptr(step_dev), int(train), _F3(*mean), _F3(*std), *zs, *cp,
                                is_f32(out), stream_ptr()), "augment")


def nchw_to_nhwc(x, y, n, c, h, w, cp):
    check(kernels().psx_nchw_to_nhwc(ptr(x), ptr(y), n, c, h, w, cp, is_f32(y), stream_ptr()), "nchw_to_nhwc")
