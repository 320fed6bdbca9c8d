"""fp32 compute path — the reference's training precision (reference src/workers/worker.py:333-348
and baseline/baseline_training.py:149-179 run torch fp32): every activation kernel instantiated
for fp32 (conv fwd / dgrad / wgrad on the exact-f32 MFMA, BN, head, augment, max-pool) against a
torch float64 reference at fp32-level tolerance (max-abs error <= 1e-4 of the reference's
max-abs), and one whole ResNet-18 step of the fp32 engine against torch fp64 autograd."""
import copy

import numpy as np
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


def _pow2(v, lo=4):
    p = lo
    while p < v:
        p *= 2
    return p


def operands_f32(w):
    """OIHW fp32 weight -> fp32 (wf [OC][Kg], wd [Cp][Kgd]) through the table-driven unpack."""
    oc, cin, k, _ = w.shape
    cp = _pow2(cin)
    kg = -(-(k * k * cp) // 64) * 64
    kgd = k * k * oc
    wbuf = torch.zeros(oc * kg + cp * kgd, dtype=torch.float32, device=DEV)
    raw = np.zeros(1, dtype=np.dtype([("o", "<i8", 3), ("i", "<i4", 8)]))
    raw[0]["o"] = (0, 0, oc * kg)
    raw[0]["i"] = (oc, cin, k, k, cp, kg, kgd, 0)
    desc = torch.from_numpy(raw.view(np.uint8).copy()).to(DEV)
    ntiles = -(-oc // 64) * -(-cp // 64) * -(-(k * k) // 3)
    K.param_unpack_tiles(w.contiguous().reshape(-1), desc, 1, ntiles, wbuf)
    return wbuf[:oc * kg], wbuf[oc * kg:], cp, kg, kgd


def nhwc(x, cp):
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, cp, dtype=torch.float32, device=DEV)
    out[..., :c] = x.permute(0, 2, 3, 1)
    return out


def _ws(nb, oh, ow, oc, kg):
    n = K.conv2_workspace_bytes(nb, oh, ow, oc, kg, True)
    return torch.empty(max(1, n // 4), dtype=torch.float32, device=DEV) if n else None


# (batch, cin, cout, hw, k, stride, pad): every distinct ResNet-18 conv (batch 16, and the
# split-K / tap-reuse planner cases at the benchmark batch 128) + ResNet-50 shapes at batch 2
R18 = [(3, 64, 32, 3, 1, 1), (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (64, 128, 32, 1, 2, 0),
       (128, 128, 16, 3, 1, 1), (128, 256, 16, 3, 2, 1), (128, 256, 16, 1, 2, 0), (256, 256, 8, 3, 1, 1),
       (256, 512, 8, 3, 2, 1), (256, 512, 8, 1, 2, 0), (512, 512, 4, 3, 1, 1)]
SHAPES = [(16,) + s for s in R18] + [(128,) + s for s in R18 if s[0] >= 256 or s == (64, 64, 32, 3, 1, 1)]
SHAPES += [(2, 3, 64, 224, 7, 2, 3), (2, 64, 64, 56, 3, 1, 1), (2, 256, 128, 56, 1, 1, 0),
           (2, 128, 128, 56, 3, 2, 1), (2, 512, 512, 7, 3, 1, 1), (2, 1024, 2048, 14, 1, 2, 0)]


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_f32(shape):
    torch.manual_seed(0)
    n, cin, cout, hw, k, s, p = shape
    x = torch.randn(n, cin, hw, hw, device=DEV)
    w = torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5
    wf, wd, cp, kg, kgd = operands_f32(w)
    oh = (hw + 2 * p - k) // s + 1
    y = torch.empty(n, oh, oh, cout, dtype=torch.float32, device=DEV)
    stats = torch.zeros(K.STAT_SLOTS, 2, cout, device=DEV)
    K.conv_fwd2(nhwc(x, cp), wf, y, stats, _ws(n, oh, oh, cout, kg), n, hw, hw, cp, cout, k, s, p, kg)
    ref = F.conv2d(x.double(), w.double(), stride=s, padding=p).permute(0, 2, 3, 1)
    assert _rel(y, ref) < TOL, shape
    yd = y.double().reshape(-1, cout)
    assert torch.allclose(stats[:, 0].double().sum(0), yd.sum(0), rtol=1e-4, atol=1e-3), shape
    assert torch.allclose(stats[:, 1].double().sum(0), (yd * yd).sum(0), rtol=1e-4, atol=1e-3), shape


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] != 3])
def test_conv_dgrad_f32(shape):
    torch.manual_seed(1)
    n, cin, cout, hw, k, s, p = shape
    w = torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5
    wf, wd, cp, kg, kgd = operands_f32(w)
    oh = (hw + 2 * p - k) // s + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV)
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.double(), dy.double(), stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.float32, device=DEV)
    res = torch.randn(n, hw, hw, cp, device=DEV)
    ws = _ws(n, hw, hw, cp, kgd)
    K.conv_dgrad2(nhwc(dy, cout), wd, dx, None, ws, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], ref) < TOL, shape
    K.conv_dgrad2(nhwc(dy, cout), wd, dx, res, ws, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], ref + res[..., :cin].double()) < TOL, shape


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_wgrad_f32(shape):
    torch.manual_seed(2)
    n, cin, cout, hw, k, s, p = shape
    x = torch.randn(n, cin, hw, hw, device=DEV)
    oh = (hw + 2 * p - k) // s + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV)
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, k, k), dy.double(), stride=s, padding=p)
    cp = _pow2(cin)
    kg = -(-(k * k * cp) // 64) * 64
    splits = K.conv_wgrad2_splits(n, hw, hw, cp, cout, k, s, p, kg, True)
    part = torch.full((splits * cout * kg,), float("nan"), device=DEV)  # every slab element must be written
    assert K.conv_wgrad2(nhwc(x, cp), nhwc(dy, cout), part, n, hw, hw, cp, cout, k, s, p, kg) == splits
    out = torch.zeros(cout * cin * k * k, device=DEV)
    K.wgrad_reduce(part, splits, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False)
    assert _rel(out.view_as(ref), ref) < TOL, shape


@pytest.mark.parametrize("tile", [(64, 128, 2), (64, 64, 2), (64, 256, 1), (64, 128, 1)])
@pytest.mark.parametrize("shape", [(16, 64, 64, 32, 3, 1, 1), (16, 128, 128, 16, 3, 1, 1), (16, 64, 128, 32, 3, 2, 1)])
def test_conv_f32_every_tile(shape, tile, monkeypatch):
    bm, bn, wgm = tile
    n, cin, cout, hw, k, s, p = shape
    monkeypatch.setenv("PSX_TUNE", f"cv_bm={bm},cv_bn={bn},cv_wgm={wgm},cv_splits=1,cv_tapr=0")
    torch.manual_seed(3)
    x = torch.randn(n, cin, hw, hw, device=DEV)
    w = torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5
    wf, wd, cp, kg, kgd = operands_f32(w)
    oh = (hw + 2 * p - k) // s + 1
    y = torch.empty(n, oh, oh, cout, dtype=torch.float32, device=DEV)
    K.conv_fwd2(nhwc(x, cp), wf, y, None, None, n, hw, hw, cp, cout, k, s, p, kg)
    assert _rel(y, F.conv2d(x.double(), w.double(), stride=s, padding=p).permute(0, 2, 3, 1)) < TOL, (shape, tile)
    dy = torch.randn(n, cout, oh, oh, device=DEV)
    dref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.double(), dy.double(), stride=s, padding=p)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.float32, device=DEV)
    K.conv_dgrad2(nhwc(dy, cout), wd, dx, None, None, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], dref.permute(0, 2, 3, 1)) < TOL, (shape, tile)


@pytest.mark.parametrize("bn", [64, 128, "halo"])
def test_conv_f32_tap_reuse_bn_bwd_sums(bn, monkeypatch):
    """Tap-reuse mainloop in fp32 + the dgrad epilogue's fused BN-backward sums."""
    if bn == "halo":
        monkeypatch.setenv("PSX_TUNE", "cv_tapr_halo=1")
    else:
        monkeypatch.setenv("PSX_TUNE", f"cv_tapr_bn={bn}")
    n, c, hw = 8, 64, 32
    torch.manual_seed(4)
    w = torch.randn(c, c, 3, 3, device=DEV) / (c * 9) ** 0.5
    wf, wd, cp, kg, kgd = operands_f32(w)
    dy = torch.randn(n, c, hw, hw, device=DEV)
    dref = torch.nn.grad.conv2d_input((n, c, hw, hw), w.double(), dy.double(), padding=1).permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, c, dtype=torch.float32, device=DEV)
    o = torch.randn(n, hw, hw, c, device=DEV)
    y1 = torch.randn(n, hw, hw, c, device=DEV)
    saved = torch.stack([0.1 * torch.randn(c, device=DEV), 1.0 + torch.rand(c, device=DEV)])
    part = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
    K.conv_dgrad2(nhwc(dy, c), wd, dx, None, None, n, hw, hw, c, c, 3, 1, 1, kgd, bst=K.bwd_stats_desc(part, o, y1, saved))
    assert _rel(dx, dref) < TOL
    dz = (dx.double() * (o > 0)).reshape(-1, c)
    xhat = (y1.double().reshape(-1, c) - saved[0].double()) * saved[1].double()
    assert torch.allclose(part[:, 0].double().sum(0), dz.sum(0), rtol=1e-4, atol=1e-3)
    assert torch.allclose(part[:, 1].double().sum(0), (dz * xhat).sum(0), rtol=1e-4, atol=1e-3)


def test_bn_kernels_f32():
    torch.manual_seed(5)
    npix, c = 4096, 128
    y = torch.randn(npix, c, device=DEV)
    res = torch.randn(npix, c, device=DEV)
    aff = torch.stack([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)])
    out = torch.empty_like(y)
    K.bn_apply(y, aff, out, c, relu=True, res=res)
    ref = torch.relu(y.double() * aff[0].double() + aff[1].double() + res.double())
    assert _rel(out, ref) < 1e-6
    g, o = torch.randn(npix, c, device=DEV), torch.randn(npix, c, device=DEV)
    saved = torch.stack([0.1 * torch.randn(c, device=DEV), 1.0 + torch.rand(c, device=DEV)])
    part = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
    K.bn_bwd_reduce(g, o, y, saved, part, npix, c)
    dz = g.double() * (o > 0)
    xh = (y.double() - saved[0].double()) * saved[1].double()
    assert torch.allclose(part[:, 0].double().sum(0), dz.sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(part[:, 1].double().sum(0), (dz * xh).sum(0), rtol=1e-5, atol=1e-4)
    coef = torch.randn(3, c, device=DEV)
    dx = torch.empty_like(y)
    dzo = torch.empty_like(y)
    K.bn_bwd_apply(g, o, y, coef, dx, c, dzout=dzo)
    cd = coef.double()
    assert _rel(dx, cd[0] * dz + cd[1] * y.double() + cd[2]) < 1e-6
    assert torch.equal(dzo, (g * (o > 0)).float())


def test_head_f32():
    torch.manual_seed(6)
    B, hw, c, k = 32, 16, 512, 100
    act = torch.relu(torch.randn(B, hw, c, device=DEV))
    fcw = torch.randn(k, c, device=DEV) * 0.05
    fcb = torch.randn(k, device=DEV) * 0.1
    labels = torch.randint(0, k, (B,), dtype=torch.int32, device=DEV)
    pooled = torch.empty(B, c, device=DEV)
    dl = torch.empty(B, k, device=DEV)
    dact = torch.empty_like(act)
    loss = torch.empty(B, device=DEV)
    correct = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.head_fwd_bwd(act, B, hw, c, fcw, fcb, k, labels, pooled, dl, dact, loss, correct)
    a = act.double().requires_grad_(True)
    logits = a.mean(1) @ fcw.double().t() + fcb.double()
    lref = F.cross_entropy(logits, labels.long(), reduction="none")
    lref.mean().backward()
    assert _rel(loss, lref.detach()) < 1e-5
    assert _rel(dact, a.grad) < 1e-5
    assert correct.item() == (logits.argmax(1) == labels.long()).sum().item()


def test_augment_and_maxpool_f32():
    torch.manual_seed(7)
    B, H, W = 8, 32, 32
    imgs = torch.randint(0, 256, (16, H, W, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (16,), dtype=torch.int32, device=DEV)
    index = torch.arange(B, dtype=torch.int32, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    out32 = torch.empty(B, H, W, 4, dtype=torch.float32, device=DEV)
    out16 = torch.empty(B, H, W, 8, dtype=torch.bfloat16, device=DEV)
    ol = torch.empty(B, dtype=torch.int32, device=DEV)
    mean, std = (0.5071, 0.4867, 0.4408), (0.2675, 0.2565, 0.2761)
    K.augment(imgs, labs, index, out32, ol, B, H, W, 4, 1, step, False, mean, std)
    K.augment(imgs, labs, index, out16, ol, B, H, W, 4, 1, step, False, mean, std)
    ref = (imgs[:B].float() / 255 - torch.tensor(mean, device=DEV)) / torch.tensor(std, device=DEV)
    assert torch.allclose(out32[..., :3], ref, atol=1e-5)
    assert (out32[..., 3] == 0).all()
    assert torch.allclose(out16[..., :3].float(), out32[..., :3], atol=2e-2)
    x = torch.randn(2, 16, 16, 64, device=DEV)
    y = torch.empty(2, 8, 8, 64, device=DEV)
    arg = torch.empty(2, 8, 8, 64, dtype=torch.uint8, device=DEV)
    K.maxpool3s2_fwd(x, y, arg)
    assert torch.equal(y, F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1))
    # backward (2x2-block gather) against torch's max-pool autograd, odd sizes included
    for (b, h, w, c) in ((2, 16, 16, 64), (3, 7, 9, 16), (2, 112, 112, 64)):
        x = torch.randn(b, h, w, c, device=DEV)
        oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty(b, oh, ow, c, device=DEV)
        arg = torch.empty(b, oh, ow, c, dtype=torch.uint8, device=DEV)
        K.maxpool3s2_fwd(x, y, arg)
        xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
        dy = torch.randn(b, oh, ow, c, device=DEV)
        F.max_pool2d(xr, 3, 2, 1).backward(dy.permute(0, 3, 1, 2))
        dx = torch.full_like(x, float("nan"))
        K.maxpool3s2_bwd(dy, arg, dx)
        assert torch.allclose(dx, xr.grad.permute(0, 2, 3, 1), atol=1e-5, rtol=1e-6), (b, h, w, c)


# Bars of the whole-step test RELATIVE to torch's own fp32 autograd error against the same fp64
# reference: the worst tensor's error <= max(STEP_K * torch's worst,
# STEP_FLOOR) and the median over tensors <= max(STEP_MED_K * torch's median, STEP_MED_FLOOR).
# The amplification is chaotic (which forward values cross a ReLU), so it is compared per job, not
# per tensor: torch's error concentrates in the layers its own flips feed (one run: 3e-3 on
# stem..layer2.0, 7e-4 below) and the engine's where its flips are (the same run: 2-3e-3 from
# layer4.0 up, 5-6e-3 on stem..layer2). Measured (round 4): Winograd path worst 6.6e-3 / median
# 3.4e-3 against torch worst 3.4e-3 / median 7.5e-4 (an earlier build 2.6e-3 / 1.5e-3); direct
# path worst 5.0e-3 / median 3.4e-3 (round 3: 6.6e-3 / 3.9e-3). Round 5 (deterministic mode's
# exact fixed-point BN sums: a third reduction order) Winograd path: median 7.0e-3, worst 1.1e-2
# against torch's 8.2e-4 / 3.4e-3 — the same spread as round 3's second reduction tree (7e-3 /
# 1.1e-2). The floors cover that chaos; the per-tensor bars are test_engine_step_f32_per_tensor_damped.
STEP_K, STEP_FLOOR = 3.0, 1.5e-2
STEP_MED_K, STEP_MED_FLOOR = 3.0, 1e-2


@pytest.mark.parametrize("wino", ["1", "0"])
def test_engine_step_f32_matches_torch_fp64(wino, monkeypatch):
    """One fp32 ResNet-18 training step on the HIP engine vs torch float64 autograd of the
    reference model: loss, every parameter gradient and the running statistics. Both conv paths:
    Winograd F(4x4,3x3) on the 3x3 stride-1 layers (the default) and the direct kernels."""
    monkeypatch.setenv("PSX_TUNE", f"wino={wino}")
    from psx.models.engine import HipResNetEngine
    from psx.models.layout import ParamLayout
    from psx.models.resnet import ResNet18

    torch.manual_seed(0)
    B = 32
    model = ResNet18(100)
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    arena = arena.to(DEV)
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, dtype=torch.float32, deterministic=True)
    x = torch.randn(B, 3, 32, 32, device=DEV)
    y = torch.randint(0, 100, (B,), device=DEV)
    eng.unpack(arena)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 32, 32, eng.x0.shape[-1])
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(arena, train=True)
    eng.head(arena, backward=True)
    eng.backward(arena)
    torch.cuda.synchronize()

    # torch's own fp32 autograd (MIOpen) sets the bar next to the fp64 reference: BN-normalised
    # early layers of a random-init ResNet amplify fp32 rounding differences
    ref = copy.deepcopy(model).to(DEV).double()
    m32 = model.to(DEV)
    m32.train()
    F.cross_entropy(m32(x), y).backward()
    g32 = {n: p.grad.double().clone() for n, p in m32.named_parameters()}
    ref.train()
    loss = F.cross_entropy(ref(x.double()), y)
    loss.backward()
    assert abs(eng.loss.double().mean().item() - loss.item()) < 1e-5 * max(1.0, loss.item())
    rows = []
    for name, p in ref.named_parameters():
        g = layout.grad_view(eng.grads, name).double()
        nrm = p.grad.norm().clamp_min(1e-30)
        err, err32 = ((g - p.grad).norm() / nrm).item(), ((g32[name] - p.grad).norm() / nrm).item()
        rows.append((name, err, err32))
    for name, err, err32 in rows:
        print(f"{name:32s} engine {err:.2e}  torch-fp32 {err32:.2e}")
    # At random init BN-normalised backward passes amplify fp32 rounding: a forward value that
    # lands on the other side of a ReLU flips its mask, and a BN bias gradient (a sum of dz with
    # heavy cancellation) moves by far more than the rounding. torch's own fp32 autograd sits at
    # 0.7-3.6e-3 from fp64 per tensor, and moves from run to run (MIOpen's algorithm choice:
    # conv1.weight 3.1e-3 in one run, 8.4e-4 in the next). The engine runs deterministic, but the
    # amplified value still depends on the association of its reductions: with Winograd (~3e-6
    # forward rounding per layer, 15x direct fp32's) two reduction trees measured median 3.9e-3 /
    # 7e-3, worst 6.6e-3 / 1.1e-2 (round 3; the fused Winograd weight gradient of round 4 measures
    # median 1.5e-3, worst 2.6e-3 in one build, 3.4e-3 / 6.6e-3 in the next). Bars: relative to
    # torch-fp32's own error (STEP_K, STEP_MED_K above), the head (no BN amplification) tight.
    errs, errs32 = sorted(r[1] for r in rows), sorted(r[2] for r in rows)
    assert errs[-1] <= max(STEP_K * errs32[-1], STEP_FLOOR), max(rows, key=lambda r: r[1])
    med, med32 = errs[len(errs) // 2], errs32[len(errs32) // 2]
    assert med <= max(STEP_MED_K * med32, STEP_MED_FLOOR), (med, med32)
    assert dict((r[0], r[1]) for r in rows)["fc.weight"] < 1e-5
    sd = ref.state_dict()
    for name in ("bn1.running_mean", "layer2.0.bn1.running_var", "layer4.1.bn2.running_mean"):
        assert torch.allclose(layout.view(arena, name).double(), sd[name], rtol=1e-5, atol=1e-6), name
    print(f"fp32 engine vs fp64 autograd: worst per-tensor relative gradient error {max(r[1] for r in rows):.2e}")


# Per-tensor bars: every tensor's error <= max(PT_K * torch-fp32's error on
# that tensor, floor), residual branches damped as torchvision's zero_init_residual does (each
# block's last BN gamma 0.2). Measured (profiles/r5_numerics_wino_variants.jsonl, deterministic):
# the direct kernels (wino=0) median 2.4e-6, worst 5.3e-4 — far below torch's own fp32 (MIOpen:
# 3-4e-3 on the early layers); with Winograd F(4x4,3x3) (the default) every tensor sits near
# 5e-3: the transform's conditioning (points 0, +-1, +-2: ~10x direct fp32's rounding per layer)
# amplified by the BN backward's cancellation; restricting Winograd to the 8x8 / 4x4 layers puts
# layer4 back at 7e-6, so the error enters through the 32x32 / 16x16 layers' forward. The
# Winograd path's floor is therefore 1e-2 (convergence parity with torch fp32 over 500 steps:
# docs/artifacts/README.md), the direct path's 2e-3.
PT_K = 3.0
PT_FLOOR = {"0": 2e-3, "1": 1e-2}


@pytest.mark.parametrize("wino", ["1", "0"])
def test_engine_step_f32_per_tensor_damped(wino, monkeypatch):
    monkeypatch.setenv("PSX_TUNE", f"wino={wino}")
    from psx.models.engine import HipResNetEngine
    from psx.models.layout import ParamLayout
    from psx.models.resnet import ResNet18

    torch.manual_seed(5)
    B = 32
    model = ResNet18(100)
    with torch.no_grad():
        for name, m in model.named_modules():
            if name.endswith("bn2") or name.endswith("shortcut.1"):
                m.weight.fill_(0.2)
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    arena = arena.to(DEV)
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, dtype=torch.float32, deterministic=True)
    x = torch.randn(B, 3, 32, 32, device=DEV)
    y = torch.randint(0, 100, (B,), device=DEV)
    eng.unpack(arena)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 32, 32, eng.x0.shape[-1])
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(arena, train=True)
    eng.head(arena, backward=True)
    eng.backward(arena)
    torch.cuda.synchronize()
    ref = copy.deepcopy(model).to(DEV).double()
    m32 = model.to(DEV)
    m32.train()
    F.cross_entropy(m32(x), y).backward()
    ref.train()
    F.cross_entropy(ref(x.double()), y).backward()
    bad = []
    for name, p in ref.named_parameters():
        g = layout.grad_view(eng.grads, name).double()
        nrm = p.grad.norm().clamp_min(1e-30)
        err = ((g - p.grad).norm() / nrm).item()
        err32 = ((m32.get_parameter(name).grad.double() - p.grad).norm() / nrm).item()
        print(f"{name:32s} engine {err:.2e}  torch-fp32 {err32:.2e}")
        if err > max(PT_K * err32, PT_FLOOR[wino]):
            bad.append((name, err, err32))
    assert not bad, bad


@pytest.mark.parametrize("f32", [True, False])
def test_bn_statistics_large_mean_shifted_sums(f32):
    """BN variance from one-pass sums cancels when |mean| >> std. The conv
    epilogue sums (y - k) and (y - k)^2 around a per-channel shift k (the engine passes the
    previous batch mean) and the finalize recombines: the saved mean / invstd and the running
    variance of a conv output with mean 100 and std 1 per channel match float64 to ~1e-6, where
    the plain sums (k = 0) lose about three digits of the variance."""
    torch.manual_seed(3)
    B, hw, c = 64, 16, 64
    dt = torch.float32 if f32 else torch.bfloat16
    x = (100.0 + torch.randn(B, hw, hw, c, device=DEV) * (1.0 + torch.rand(c, device=DEV))).to(dt)
    w = torch.eye(c, device=DEV).to(dt).contiguous()  # 1x1 conv = identity: y = x
    y = torch.empty(B, hw, hw, c, dtype=dt, device=DEV)
    ref = x.double().reshape(-1, c)
    mean_ref, var_ref = ref.mean(0), ref.var(0, unbiased=False)
    errs = {}
    for name, k in (("plain", None), ("shifted", (mean_ref + 0.3 * var_ref.sqrt()).float())):
        stats = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
        K.conv_fwd2(x, w, y, stats, None, B, hw, hw, c, c, 1, 1, 0, 64, sshift=k)
        gamma, beta = torch.ones(c, device=DEV), torch.zeros(c, device=DEV)
        rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
        aff, saved = torch.empty(2, c, device=DEV), torch.empty(2, c, device=DEV)
        nxt = torch.zeros(c, device=DEV)
        K.bn_finalize(stats, K.STAT_SLOTS, c, B * hw * hw, gamma, beta, 1e-5, 0.1, rm, rv, aff, saved, sshift=k,
                      sshift_next=nxt)
        torch.cuda.synchronize()
        var = 1.0 / saved[1].double() ** 2 - 1e-5
        errs[name] = (((saved[0].double() - mean_ref).abs().max() / var_ref.sqrt().max()).item(),
                      ((var - var_ref).abs() / var_ref).max().item())
        assert torch.allclose(nxt.double(), mean_ref, rtol=1e-6, atol=1e-4)
        unb = var_ref * (B * hw * hw) / (B * hw * hw - 1)
        if k is not None:
            assert ((rv.double() - (0.9 + 0.1 * unb)).abs() / unb).max().item() < 1e-5
    print("bn statistics mean / variance error:", errs)
    assert errs["shifted"][0] < 1e-5 and errs["shifted"][1] < 2e-5, errs


@pytest.mark.parametrize("shape", [(16, 64, 128, 32), (128, 128, 256, 16), (16, 256, 512, 8), (4, 64, 128, 14)])
@pytest.mark.parametrize("stats", [False, True])
def test_conv_dgrad2_shortcut_fold_f32(shape, stats):
    """3x3/s2 data gradient with the block's 1x1/s2 shortcut data gradient folded into the (0, 0)
    parity class (conv_v2.hip psx_conv_dgrad2_sc) against torch fp64 of both convs summed."""
    torch.manual_seed(6)
    n, cin, cout, hw = shape
    w = torch.randn(cout, cin, 3, 3, device=DEV) / (cin * 9) ** 0.5
    w2 = torch.randn(cout, cin, 1, 1, device=DEV) / cin ** 0.5
    _, wd, cp, _, kgd = operands_f32(w)
    _, wd2, _, _, kgd2 = operands_f32(w2)
    oh = (hw - 1) // 2 + 1
    dy, dy2 = torch.randn(n, cout, oh, oh, device=DEV), torch.randn(n, cout, oh, oh, device=DEV)
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.double(), dy.double(), stride=2, padding=1)
    ref = (ref + torch.nn.grad.conv2d_input((n, cin, hw, hw), w2.double(), dy2.double(), stride=2)).permute(0, 2, 3, 1)
    dx = torch.full((n, hw, hw, cp), float("nan"), device=DEV)
    bst = None
    if stats:
        o = torch.randn(n, hw, hw, cp, device=DEV)
        y1 = torch.randn(n, hw, hw, cp, device=DEV)
        saved = torch.stack([0.1 * torch.randn(cp, device=DEV), 1.0 + torch.rand(cp, device=DEV)])
        part = torch.zeros(K.STAT_SLOTS, 2, cp, device=DEV)
        bst = K.bwd_stats_desc(part, o, y1, saved)
    assert K.conv_dgrad2_sc(nhwc(dy, cout), wd, dx, None, n, hw, hw, cp, cout, kgd, nhwc(dy2, cout), wd2, kgd2, bst=bst)
    assert _rel(dx[..., :cin], ref) < TOL, shape
    if stats:
        dz = (dx.double() * (o > 0)).reshape(-1, cp)
        xhat = (y1.double().reshape(-1, cp) - saved[0].double()) * saved[1].double()
        assert torch.allclose(part[:, 0].double().sum(0), dz.sum(0), rtol=1e-4, atol=1e-3)
        assert torch.allclose(part[:, 1].double().sum(0), (dz * xhat).sum(0), rtol=1e-4, atol=1e-3)
    # shapes the fold does not cover report False (the caller runs the two launches)
    w1 = torch.randn(cout, cin, 1, 1, device=DEV)
    _, wd1, _, _, kgd1 = operands_f32(w1)
    assert not K.conv_dgrad2_sc(nhwc(dy, cout), wd, dx, None, n, hw, hw, cp, cout, kgd, nhwc(dy2, cout), wd1,
                                kgd1 + 1)


@pytest.mark.parametrize("n", [128, 3])
def test_stem_conv_direct_f32(n):
    """The direct stem conv (csrc/kernels/stem.hip, 3 -> 64, 3x3/s1) and its shifted BN statistics
    against torch fp64; n = 3 leaves a partial last workgroup."""
    K.set_deterministic(None)  # an earlier engine test may have left the process in deterministic mode
    torch.manual_seed(10)
    x = torch.randn(n, 3, 32, 32, device=DEV)
    w = torch.randn(64, 3, 3, 3, device=DEV) / 27 ** 0.5
    wf, _, cp, kg, _ = operands_f32(w)
    y = torch.full((n, 32, 32, 64), float("nan"), device=DEV)
    st = torch.zeros(K.STAT_SLOTS, 2, 64, device=DEV)
    sh = 0.1 * torch.randn(64, device=DEV)
    assert K.stem_conv(nhwc(x, cp), wf, y, st, n, 32, 32, 3, cp, 64, kg, sshift=sh)
    ref = F.conv2d(x.double(), w.double(), padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < TOL
    d = y.double().reshape(-1, 64) - sh.double()
    assert torch.allclose(st[:, 0].double().sum(0), d.sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(st[:, 1].double().sum(0), (d * d).sum(0), rtol=1e-4, atol=1e-2)
    assert not K.stem_conv(nhwc(x, cp), wf, y, st, n, 32, 32, 4, cp, 64, kg)  # not the stem shape


@pytest.mark.parametrize("n", [2, 3])
def test_stem7_conv_f32(n):
    """The ImageNet stem on the MFMA (stem.hip stem7_fwd_kernel: 3 -> 64, 7x7 / stride 2 / pad 3,
    224 -> 112, input patch + weights in LDS) and its shifted BN statistics against torch fp64."""
    K.set_deterministic(None)  # an earlier engine test may have left the process in deterministic mode
    torch.manual_seed(12)
    x = torch.randn(n, 3, 224, 224, device=DEV)
    w = torch.randn(64, 3, 7, 7, device=DEV) / 147 ** 0.5
    wf, _, cp, kg, _ = operands_f32(w)
    y = torch.full((n, 112, 112, 64), float("nan"), device=DEV)
    st = torch.zeros(K.STAT_SLOTS, 2, 64, device=DEV)
    sh = 0.1 * torch.randn(64, device=DEV)
    assert K.stem_conv(nhwc(x, cp), wf, y, st, n, 224, 224, 3, cp, 64, kg, sshift=sh, k=7)
    ref = F.conv2d(x.double(), w.double(), stride=2, padding=3).permute(0, 2, 3, 1)
    assert _rel(y, ref) < TOL
    d = y.double().reshape(-1, 64) - sh.double()
    assert torch.allclose(st[:, 0].double().sum(0), d.sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(st[:, 1].double().sum(0), (d * d).sum(0), rtol=1e-4, atol=1e-2)
    assert not K.stem_conv(nhwc(x, cp), wf, y, st, n, 224, 224, 4, cp, 64, kg, k=7)  # not the stem shape


def test_stem7_wgrad_f32():
    """The ImageNet stem's weight gradient (stem.hip stem7_wgrad_kernel, reached through
    conv_wgrad2 + wgrad_reduce as the engine calls it) against torch fp64."""
    torch.manual_seed(13)
    n = 3
    x = torch.randn(n, 3, 224, 224, device=DEV)
    w = torch.randn(64, 3, 7, 7, device=DEV)
    _, _, cp, kg, _ = operands_f32(w)
    dy = torch.randn(n, 112, 112, 64, device=DEV)
    spl = K.conv_wgrad2_splits(n, 224, 224, cp, 64, 7, 2, 3, kg, True)
    part = torch.full((spl * 64 * kg,), float("nan"), device=DEV)
    out = torch.full((64 * 3 * 49,), float("nan"), device=DEV)
    assert K.conv_wgrad2(nhwc(x, cp), dy, part, n, 224, 224, cp, 64, 7, 2, 3, kg) == spl
    K.wgrad_reduce(part, spl, 64, kg, 3, cp, 7, 1.0, out.data_ptr(), False)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.double(), (64, 3, 7, 7), dy.double().permute(0, 3, 1, 2), stride=2, padding=3)
    assert _rel(out.view(64, 3, 7, 7), ref) < TOL
