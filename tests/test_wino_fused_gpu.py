"""Fused fp32 Winograd conv (csrc/kernels/wino_fused.hip: input transform + 36 GEMMs + output
transform in one launch) against torch float64 and against the three-launch path (wino.hip) it
replaces: forward (+ residual, BN slot sums, the transformed-input side output V), data gradient
with the consumer BN's backward sums (mask from o / from the affine, one or two BNs, masked store),
the folded input BN + ReLU (finalize outputs included) and deterministic mode."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"
TOL = 1e-4


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _uf(w, k, c, flip=False):
    """(layout-1 fused operand, layout-0 batched-GEMM operand) of w [k][c][3][3]."""
    uf = torch.full((40 * k * c,), float("nan"), device=DEV)
    u0 = torch.full((36 * k * c,), float("nan"), device=DEV)
    K.WinoWeightBatch([(w, uf, k, c, flip, 1), (w, u0, k, c, flip, 0)])()
    return uf, u0


def test_fused_layout_is_a_permutation():
    """Layout 1 holds the layout-0 values at [row/16][col/4][slot][(col%4)*16 + row%16][4], slot
    5h + i = points 18h + 4i.. (i < 4), slot 5h + 4 = points 18h + 16, 18h + 17 and two zeros."""
    torch.manual_seed(0)
    k, c = 64, 128
    w = torch.randn(k, c, 3, 3, device=DEV)
    uf, u0 = _uf(w, k, c)
    torch.cuda.synchronize()
    u = u0.view(k, 36, c)  # [row][b][col]
    idx = torch.arange(40 * k * c, device=DEV)
    j, lane, slot = idx % 4, (idx // 4) % 64, (idx // 256) % 10
    cs, rg = (idx // 2560) % (c // 4), idx // (2560 * (c // 4))
    row, col = rg * 16 + lane % 16, cs * 4 + lane // 16
    hh, i = slot // 5, slot % 5
    b = 18 * hh + 4 * i + j
    pad = (i == 4) & (j >= 2)
    assert torch.equal(uf[pad], torch.zeros_like(uf[pad]))
    assert torch.equal(uf[~pad], u[row[~pad], b[~pad], col[~pad]])


@pytest.mark.parametrize("nb,h,c,k,res,vout", [(16, 32, 64, 64, False, True), (4, 16, 128, 128, True, False),
                                               (4, 8, 64, 128, False, False), (8, 16, 64, 128, True, True),
                                               (2, 16, 128, 64, False, True)])
def test_wino_fused_fwd(nb, h, c, k, res, vout):
    torch.manual_seed(nb * h + c + k)
    x = torch.relu(torch.randn(nb, c, h, h, device=DEV, dtype=torch.float64))
    w = torch.randn(k, c, 3, 3, device=DEV, dtype=torch.float64) * (2.0 / (9 * c)) ** 0.5
    r = torch.randn(nb, k, h, h, device=DEV, dtype=torch.float64) if res else None
    ref = _nhwc(F.conv2d(x, w, padding=1) + (r if res else 0))
    assert K.wino_fused_ok(nb, h, h, c, k)
    uf, u0 = _uf(w.float().contiguous(), k, c)
    y = torch.full((nb, h, h, k), float("nan"), device=DEV)
    stats = torch.zeros(K.STAT_SLOTS, 2, k, device=DEV)
    v = torch.full((K.wino_v_floats(nb, h, h, c),), float("nan"), device=DEV) if vout else None
    xs, rs = _nhwc(x.float()), _nhwc(r.float()) if res else None
    K.wino_fused(xs, uf, y, rs, stats, v, nb, h, h, c, k)
    torch.cuda.synchronize()
    assert _rel(y, ref) < TOL
    s = stats.double().sum(0)
    assert torch.allclose(s[0], ref.sum((0, 1, 2)), rtol=1e-4, atol=1e-3 * ref.abs().max().item())
    assert torch.allclose(s[1], (ref ** 2).sum((0, 1, 2)), rtol=1e-4)
    if vout:  # the same B^T d B as the separate input transform (wino_conv's V)
        v0 = torch.empty_like(v)
        p0 = torch.empty(K.wino_p_floats(nb, h, h, c, k), device=DEV)
        y0 = torch.empty_like(y)
        K.wino_conv(xs, u0, y0, rs, None, v0, p0, nb, h, h, c, k)
        torch.cuda.synchronize()
        assert _rel(v, v0) < 1e-6


@pytest.mark.parametrize("nb,h,c,k", [(8, 16, 64, 128), (16, 32, 64, 64)])
@pytest.mark.parametrize("two,mask_store,res,maff", [(False, False, False, False), (True, True, True, False),
                                                     (False, True, False, True), (True, False, False, True)])
def test_wino_fused_dgrad_bn_bwd_sums(nb, h, c, k, two, mask_store, res, maff):
    """Data gradient (forward conv of dy with the flipped transform, output channels = the forward's
    input channels c) with the consumer BN's backward sums: the same contract as wino_conv's bst."""
    torch.manual_seed(c + k + 3 * two + mask_store)
    w = torch.randn(k, c, 3, 3, device=DEV) * (2.0 / (9 * c)) ** 0.5
    dy = torch.randn(nb, h, h, k, device=DEV)
    r = torch.randn(nb, h, h, c, device=DEV) if res else None
    o = torch.randn(nb, h, h, c, device=DEV)
    y1, y2 = torch.randn(nb, h, h, c, device=DEV), torch.randn(nb, h, h, c, device=DEV)
    saved1 = torch.stack([torch.randn(c, device=DEV), torch.rand(c, device=DEV) + 0.5])
    saved2 = torch.stack([torch.randn(c, device=DEV), torch.rand(c, device=DEV) + 0.5])
    aff = torch.stack([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)]).contiguous()
    part = torch.zeros(K.STAT_SLOTS, 3 if two else 2, c, device=DEV)
    bst = K.bwd_stats_desc(part, None if maff else o, y1, saved1, y2 if two else None, saved2 if two else None,
                           mask_store=mask_store, mask_aff=aff if maff else None)
    assert K.wino_fused_ok(nb, h, h, k, c)
    uf, _ = _uf(w, k, c, flip=True)
    dx = torch.full((nb, h, h, c), float("nan"), device=DEV)
    K.wino_fused(dy, uf, dx, r, None, None, nb, h, h, k, c, bst=bst)
    torch.cuda.synchronize()
    g = torch.nn.grad.conv2d_input((nb, c, h, h), w.double(), dy.double().permute(0, 3, 1, 2), padding=1)
    g = g.permute(0, 2, 3, 1) + (r.double() if res else 0)
    pos = (y1.double() * aff[0].double() + aff[1].double() > 0) if maff else (o.double() > 0)
    dz = torch.where(pos, g, torch.zeros_like(g))
    assert _rel(dx, dz if mask_store else g) < TOL
    s = part.double().sum(0)
    sums = [dz.sum((0, 1, 2)), (dz * (y1.double() - saved1[0].double()) * saved1[1].double()).sum((0, 1, 2))]
    if two:
        sums.append((dz * (y2.double() - saved2[0].double()) * saved2[1].double()).sum((0, 1, 2)))
    for i, ref in enumerate(sums):
        assert _rel(s[i], ref) < 1e-4, i


def _bn_in(c, part_scale=1.0, seed=0):
    """Slot rows of a previous layer's BN statistics and its BnFin (+ the tensors it writes)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    t = {n: torch.empty(c, device=DEV) for n in ("gamma", "beta", "rm", "rv", "ssh", "ssh_next")}
    t["gamma"].uniform_(0.5, 1.5, generator=g)
    t["beta"].normal_(0, 0.5, generator=g)
    t["rm"].normal_(0, 1, generator=g)
    t["rv"].uniform_(0.5, 2, generator=g)
    t["ssh"].normal_(0, 1, generator=g)
    t["affine"] = torch.zeros(2, c, device=DEV)
    t["saved"] = torch.zeros(2, c, device=DEV)
    t["ctr"] = torch.zeros(4, dtype=torch.int32, device=DEV)
    return t


@pytest.mark.parametrize("nb,h,c,k", [(8, 16, 128, 128)])
def test_wino_fused_bn_in_fold(nb, h, c, k):
    """The previous layer's training BN finalize + BN + ReLU folded into the input transform: the
    fused launch == the three-launch path with the same fold (output, statistics, the published
    affine / saved / running / shift statistics)."""
    torch.manual_seed(3)
    z = torch.randn(nb, h, h, c, device=DEV) * 2 + 0.5  # pre-BN output of the previous conv
    cnt = nb * h * h
    sl = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
    out = {}
    w = torch.randn(k, c, 3, 3, device=DEV) * (2.0 / (9 * c)) ** 0.5
    uf, u0 = _uf(w, k, c)
    for path in ("fused", "split"):
        t = _bn_in(c, seed=1)
        zs = z - t["ssh"]
        sl.zero_()
        sl[0, 0] = zs.sum((0, 1, 2))  # shifted sums around ssh, spread over two slots
        sl[1, 1] = (zs * zs).sum((0, 1, 2)) / 2
        sl[2, 1] = (zs * zs).sum((0, 1, 2)) / 2
        fin = K.bn_fin(t["gamma"], t["beta"], t["rm"], t["rv"], t["affine"], t["saved"], t["ctr"].data_ptr(), cnt,
                       1e-5, 0.1, c, sshift=t["ssh"], sshift_next=t["ssh_next"])
        y = torch.full((nb, h, h, k), float("nan"), device=DEV)
        stats = torch.zeros(K.STAT_SLOTS, 2, k, device=DEV)
        if path == "fused":
            K.wino_fused(z, uf, y, None, stats, None, nb, h, h, c, k, bn_in=(sl, fin))
        else:
            v = torch.empty(K.wino_v_floats(nb, h, h, c), device=DEV)
            p = torch.empty(K.wino_p_floats(nb, h, h, c, k), device=DEV)
            K.wino_conv(z, u0, y, None, stats, v, p, nb, h, h, c, k, bn_in=(sl, fin))
        torch.cuda.synchronize()
        out[path] = (y.clone(), stats.sum(0), {n: t[n].clone() for n in ("affine", "saved", "rm", "rv", "ssh_next")})
    (yf, sf, tf), (ys, ss, ts) = out["fused"], out["split"]
    assert _rel(yf, ys) < 1e-5
    assert _rel(sf, ss) < 1e-4
    for n in tf:
        assert torch.allclose(tf[n], ts[n], rtol=1e-6, atol=1e-6), n
    # and against fp64: relu(BN(z)) convolved
    mean = z.double().mean((0, 1, 2))
    var = z.double().var((0, 1, 2), unbiased=False)
    t = _bn_in(c, seed=1)
    a = torch.relu((z.double() - mean) / torch.sqrt(var + 1e-5) * t["gamma"].double() + t["beta"].double())
    ref = _nhwc(F.conv2d(a.permute(0, 3, 1, 2), w.double(), padding=1))
    assert _rel(yf, ref) < TOL


def test_wino_fused_deterministic():
    """Deterministic mode: exact fixed-point pairs in the slot buffer (bnfin.hpp DetRed) — two runs
    bit-identical, and equal to the atomic slots' sums to fp32 rounding."""
    torch.manual_seed(9)
    nb, h, c, k = 16, 32, 64, 64
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    w = torch.randn(k, c, 3, 3, device=DEV) * (2.0 / (9 * c)) ** 0.5
    uf, _ = _uf(w, k, c)
    res = []
    try:
        for det in (True, True, False):
            K.set_deterministic(det)
            y = torch.empty(nb, h, h, k, device=DEV)
            stats = torch.zeros(K.STAT_SLOTS * (K.det_slot_scale() if det else 1), 2, k, device=DEV)
            K.wino_fused(x, uf, y, None, stats, None, nb, h, h, c, k)
            torch.cuda.synchronize()
            res.append((y.clone(), stats.clone()))
    finally:
        K.set_deterministic(None)
    # the pairs' bits (as floats some are NaN patterns)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1].view(torch.int32), res[1][1].view(torch.int32))
    fixed = K.det_slot_values(res[0][1], (K.STAT_SLOTS, 2, k)).sum(0)
    assert _rel(fixed, res[2][1].sum(0).double()) < 1e-5


def _bwd_case(nb, h, c, seed):
    """dz, y, the BN's saved statistics / gamma and its backward slot sums (two slots)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    dz = torch.randn(nb, h, h, c, device=DEV, generator=g)
    y = torch.randn(nb, h, h, c, device=DEV, generator=g) * 1.5 + 0.3
    mean = torch.randn(c, device=DEV, generator=g) * 0.2 + 0.3
    invstd = torch.rand(c, device=DEV, generator=g) * 0.5 + 0.5
    gamma = torch.rand(c, device=DEV, generator=g) + 0.5
    xhat = (y - mean) * invstd
    part = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
    part[0, 0] = dz.sum((0, 1, 2)) * 0.5
    part[3, 0] = dz.sum((0, 1, 2)) * 0.5
    part[1, 1] = (dz * xhat).sum((0, 1, 2))
    saved = torch.stack([mean, invstd]).contiguous()
    return dz, y, saved, gamma, part


def _bwd_ref(dz, y, saved, gamma, part, cnt):
    """dx = gamma invstd (dz - mean(dz) - xhat mean(dz xhat)) in float64, and dgamma / dbeta."""
    mean, invstd = saved[0].double(), saved[1].double()
    sdz, sxh = part[:, 0].double().sum(0), part[:, 1].double().sum(0)
    xhat = (y.double() - mean) * invstd
    dx = gamma.double() * invstd * (dz.double() - sdz / cnt - xhat * sxh / cnt)
    return dx, sxh, sdz


@pytest.mark.parametrize("nb,h,c,k", [(8, 16, 64, 128), (16, 32, 64, 64), (4, 16, 128, 128)])
def test_wino_fused_bwd_fold(nb, h, c, k):
    """The BN-backward apply folded into the fused data gradient's operand loads: dgrad(dy) with
    dy = BNbwd(dz, y) never written == dgrad of the float64 BN backward, and the launch publishes
    the coefficients and dgamma / dbeta; the Winograd weight gradient's dy transform folds the
    same apply (== the weight gradient of the explicit dy)."""
    torch.manual_seed(k + c)
    cnt = nb * h * h
    dz, yb, saved, gamma, part = _bwd_case(nb, h, k, seed=nb + h)
    coef = torch.full((3, k), float("nan"), device=DEV)
    dgb = torch.full((2, k), float("nan"), device=DEV)
    ctr = torch.zeros(4, dtype=torch.int32, device=DEV)
    fin = K.bn_bwd_fin(gamma, saved, coef, dgb[0].data_ptr(), dgb[1].data_ptr(), ctr.data_ptr(), cnt, 1.0, k, False)
    w = torch.randn(k, c, 3, 3, device=DEV) * (2.0 / (9 * c)) ** 0.5
    uf, u0 = _uf(w, k, c, flip=True)
    dx = torch.full((nb, h, h, c), float("nan"), device=DEV)
    K.wino_fused(dz, uf, dx, None, None, None, nb, h, h, k, c, bwd_in=(yb, part, fin))
    torch.cuda.synchronize()
    dy_ref, sxh, sdz = _bwd_ref(dz, yb, saved, gamma, part, cnt)
    ref = torch.nn.grad.conv2d_input((nb, c, h, h), w.double(), dy_ref.permute(0, 3, 1, 2), padding=1)
    assert _rel(dx, ref.permute(0, 2, 3, 1)) < TOL
    assert torch.allclose(dgb[0].double(), sxh, rtol=1e-5, atol=1e-5)
    assert torch.allclose(dgb[1].double(), sdz, rtol=1e-5, atol=1e-5)
    dyc = coef[0] * dz + coef[1] * yb + coef[2]  # the published coefficients reproduce dy
    assert _rel(dyc, dy_ref) < 1e-5
    # weight gradient: folded dy transform vs the explicit dy (same coefficients, same rounding)
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    uff, _ = _uf(w, k, c)
    v = torch.empty(K.wino_v_floats(nb, h, h, c), device=DEV)
    K.wino_fused(x, uff, torch.empty(nb, h, h, k, device=DEV), None, None, v, nb, h, h, c, k)
    q = K.wino_wgrad_q(nb, h, h, c, k)
    d = torch.empty(K.wino_v_floats(nb, h, h, k), device=DEV)
    wp = torch.empty(36 * q * k * c, device=DEV)
    g1, g0 = torch.empty(k * c * 9, device=DEV), torch.empty(k * c * 9, device=DEV)
    K.wino_wgrad(v, dz, d, wp, g1, nb, h, h, c, k, bwd_in=(yb, part, fin))
    dy_x = torch.addcmul(coef[2].expand_as(dz), coef[0].expand_as(dz), dz)
    dy_x = torch.addcmul(dy_x, coef[1].expand_as(yb), yb)
    K.wino_wgrad(v, dy_x.contiguous(), d, wp, g0, nb, h, h, c, k)
    torch.cuda.synchronize()
    wref = torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (k, c, 3, 3), dy_ref.permute(0, 3, 1, 2),
                                       padding=1)
    assert _rel(g1, wref.reshape(-1)) < 1e-4
    assert _rel(g1, g0) < 1e-5


def test_engine_bwd_fold_matches_unfolded(monkeypatch):
    """Whole fp32 step, deterministic, BN-backward applies folded (PSX_TUNE wino_bwdfold=1, default)
    vs the separate apply passes: loss bit-equal, gradients equal to the rounding of the folded
    apply (a different FMA order and slot-sum order), amplified by the BN backward of a random
    init network."""
    from psx.models.engine import HipResNetEngine
    from psx.models.layout import ParamLayout
    from psx.models.resnet import ResNet18

    torch.manual_seed(2)
    model = ResNet18(100)
    layout = ParamLayout.from_module(model)
    arena0, _ = layout.pack(model)
    arena0 = arena0.to(DEV)
    B = 32
    imgs = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (64,), dtype=torch.int32, device=DEV)
    out = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("PSX_TUNE", f"wino_bwdfold={fold}")
        eng = HipResNetEngine(model, layout, B, dtype=torch.float32, deterministic=True)
        eng.index.copy_(torch.arange(B, dtype=torch.int32, device=DEV))
        a = arena0.clone()
        eng.train_step(a, imgs, labs)
        torch.cuda.synchronize()
        assert bool(eng._bwd_fold) == (fold == "1"), eng._bwd_fold.keys()
        out[fold] = (eng.loss.double().mean().item(), eng.grads.double().clone())
    (l1, g1), (l0, g0) = out["1"], out["0"]
    assert l1 == l0  # the forward is untouched
    errs = []
    for name, e in layout.entries.items():
        if e.region != "param":
            continue
        a, b = g1[e.offset:e.offset + e.numel], g0[e.offset:e.offset + e.numel]
        errs.append((((a - b).norm() / b.norm().clamp_min(1e-30)).item(), name))
    errs.sort()
    print("bwd fold vs apply: median %.2e, worst %s" % (errs[len(errs) // 2][0], errs[-3:]))
    assert errs[-1][0] < 1e-2, errs[-3:]
    assert errs[len(errs) // 2][0] < 1e-3, errs


@pytest.mark.parametrize("bad", [float("inf"), float("nan"), 1e30])
def test_deterministic_poison(bad):
    """Deterministic mode: a non-finite or out-of-range partial (|v| >= 2^38, past the fixed-point
    pairs' exact range) poisons its slot entry (bnfin.hpp kFixPoison) instead of adding an undefined
    integer: the decoded sums and the finalized mean / variance read NaN, as the float-atomic mode
    lets an Inf / NaN through; finite inputs leave every entry clean."""
    torch.manual_seed(4)
    nb, h, c, k = 16, 16, 64, 64
    w = torch.randn(k, c, 3, 3, device=DEV) * (2.0 / (9 * c)) ** 0.5
    uf, _ = _uf(w, k, c)
    try:
        K.set_deterministic(True)
        for poisoned in (False, True):
            x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
            if poisoned:
                x[3, 5, 7, :] = bad  # every output channel sees it
            y = torch.empty(nb, h, h, k, device=DEV)
            stats = torch.zeros(K.STAT_SLOTS * K.det_slot_scale(), 2, k, device=DEV)
            K.wino_fused(x, uf, y, None, stats, None, nb, h, h, c, k)
            t = _bn_in(k, seed=2)
            K.bn_finalize(stats, K.STAT_SLOTS, k, nb * h * h, t["gamma"], t["beta"], 1e-5, 0.1, t["rm"], t["rv"],
                          t["affine"], t["saved"])
            torch.cuda.synchronize()
            vals = K.det_slot_values(stats, (K.STAT_SLOTS, 2, k)).sum(0)
            if poisoned:
                assert torch.isnan(vals).all()
                assert torch.isnan(t["saved"][0]).all() and torch.isnan(t["affine"]).all()
            else:
                assert torch.isfinite(vals).all() and torch.isfinite(t["saved"]).all()
    finally:
        K.set_deterministic(None)
