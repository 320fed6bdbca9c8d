"""conv v2 (LDS-DMA pipelined, split-K) vs torch fp32 on every ResNet-18 conv shape at batch 128
and every ResNet-50 (224x224) conv shape at batch 8."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from psx.ops import kernels as K  # noqa: E402
from tests.test_kernels_gpu import _pow2, _rel, make_operands, to_nhwc  # noqa: E402

DEV = "cuda"
SHAPES = [(128, c, o, hw, k, s, p) for (_, c, o, hw, k, s, p) in [
    (8, 3, 64, 32, 3, 1, 1), (8, 64, 64, 32, 3, 1, 1), (8, 64, 128, 32, 3, 2, 1), (8, 64, 128, 32, 1, 2, 0),
    (8, 128, 128, 16, 3, 1, 1), (8, 128, 256, 16, 3, 2, 1), (8, 128, 256, 16, 1, 2, 0), (8, 256, 256, 8, 3, 1, 1),
    (8, 256, 512, 8, 3, 2, 1), (8, 256, 512, 8, 1, 2, 0), (8, 512, 512, 4, 3, 1, 1)]] + [(3, 64, 64, 8, 3, 1, 1)]
# every distinct ResNet-50 (ImageNet 224) conv: 7x7/s2 stem, bottleneck 1x1s, strided 3x3s, downsamples
SHAPES += [(4, 3, 64, 224, 7, 2, 3), (8, 64, 64, 56, 1, 1, 0), (8, 64, 64, 56, 3, 1, 1), (8, 64, 256, 56, 1, 1, 0),
           (8, 256, 64, 56, 1, 1, 0), (8, 256, 128, 56, 1, 1, 0), (8, 128, 128, 56, 3, 2, 1),
           (8, 128, 512, 28, 1, 1, 0), (8, 256, 512, 56, 1, 2, 0), (8, 512, 128, 28, 1, 1, 0),
           (8, 128, 128, 28, 3, 1, 1), (8, 256, 256, 28, 3, 2, 1), (8, 512, 1024, 28, 1, 2, 0),
           (8, 1024, 256, 14, 1, 1, 0), (8, 512, 512, 14, 3, 2, 1), (8, 1024, 2048, 14, 1, 2, 0),
           (8, 2048, 512, 7, 1, 1, 0), (8, 512, 512, 7, 3, 1, 1), (8, 512, 2048, 7, 1, 1, 0),
           (8, 256, 256, 14, 3, 1, 1)]


def _ws(nb, oh, ow, oc, kg):
    n = K.conv2_workspace_bytes(nb, oh, ow, oc, kg)
    return torch.empty(max(1, n // 4), dtype=torch.float32, device=DEV) if n else None


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd2(shape):
    torch.manual_seed(0)
    n, cin, cout, hw, k, s, p = shape
    x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).to(torch.bfloat16).float()
    wf, wd, cp, kg, kgd = make_operands(w)
    oh = (hw + 2 * p - k) // s + 1
    y = torch.empty(n, oh, oh, cout, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(K.STAT_SLOTS, 2, cout, device=DEV)
    K.conv_fwd2(to_nhwc(x, cp), wf, y, stats, _ws(n, oh, oh, cout, kg), n, hw, hw, cp, cout, k, s, p, kg)
    ref = F.conv2d(x, w, stride=s, padding=p).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2, shape
    yq = y.float().reshape(-1, cout)
    assert torch.allclose(stats[:, 0].sum(0), yq.sum(0), rtol=1e-3, atol=5e-2), shape
    assert torch.allclose(stats[:, 1].sum(0), (yq * yq).sum(0), rtol=1e-3, atol=5e-2), shape


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_wgrad2(shape):
    torch.manual_seed(2)
    n, cin, cout, hw, k, s, p = shape
    x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    oh = (hw + 2 * p - k) // s + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_weight(x, (cout, cin, k, k), dy, stride=s, padding=p)
    cp = _pow2(cin)
    kg = -(-(k * k * cp) // 64) * 64
    splits = K.conv_wgrad2_splits(n, hw, hw, cp, cout, k, s, p, kg)
    part = torch.full((splits * cout * kg,), float("nan"), device=DEV)  # every slab element must be written
    assert K.conv_wgrad2(to_nhwc(x, cp), to_nhwc(dy, cout), part, n, hw, hw, cp, cout, k, s, p, kg) == splits
    out = torch.zeros(cout * cin * k * k, device=DEV)
    K.wgrad_reduce(part, splits, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False)
    assert _rel(out.view_as(ref), ref) < 5e-3, shape


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[1] != 3])
def test_conv_dgrad2(shape):
    torch.manual_seed(1)
    n, cin, cout, hw, k, s, p = shape
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).to(torch.bfloat16).float()
    wf, wd, cp, kg, kgd = make_operands(w)
    oh = (hw + 2 * p - k) // s + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w, dy, stride=s, padding=p).permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.bfloat16, device=DEV)
    res = torch.randn(n, hw, hw, cp, device=DEV).to(torch.bfloat16)
    ws = _ws(n, hw, hw, cp, kgd)
    K.conv_dgrad2(to_nhwc(dy, cout), wd, dx, None, ws, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], ref) < 1e-2, shape
    K.conv_dgrad2(to_nhwc(dy, cout), wd, dx, res, ws, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], ref + res[..., :cin].float()) < 1e-2, shape


TILES = [(128, 128, 2), (64, 128, 2), (64, 64, 2), (64, 256, 1), (64, 128, 1), (128, 256, 2)]


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("shape", [(32, 64, 64, 32, 3, 1, 1), (32, 128, 128, 16, 3, 1, 1), (32, 64, 128, 32, 3, 2, 1),
                                   (32, 256, 256, 8, 3, 1, 1)])
def test_conv2_every_tile_config(shape, tile, monkeypatch):
    """Every (BM, BN, wave layout) instantiation of conv2_kernel, forced through the planner's
    experiment overrides, fwd (+ BN statistics) and dgrad (+ residual) against torch fp32."""
    bm, bn, wgm = tile
    n, cin, cout, hw, k, s, p = shape
    if cout % bm or cin % bm:
        pytest.skip("tile wider than the channel count")
    monkeypatch.setenv("PSX_TUNE", f"cv_bm={bm},cv_bn={bn},cv_wgm={wgm},cv_splits=1,cv_tapr=0")
    torch.manual_seed(3)
    x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).to(torch.bfloat16).float()
    wf, wd, cp, kg, kgd = make_operands(w)
    oh = (hw + 2 * p - k) // s + 1
    y = torch.empty(n, oh, oh, cout, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(K.STAT_SLOTS, 2, cout, device=DEV)
    K.conv_fwd2(to_nhwc(x, cp), wf, y, stats, None, n, hw, hw, cp, cout, k, s, p, kg)
    ref = F.conv2d(x, w, stride=s, padding=p).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2, (shape, tile)
    yq = y.float().reshape(-1, cout)
    assert torch.allclose(stats[:, 0].sum(0), yq.sum(0), rtol=1e-3, atol=5e-2), (shape, tile)
    dy = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    dref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w, dy, stride=s, padding=p).permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.bfloat16, device=DEV)
    res = torch.randn(n, hw, hw, cp, device=DEV).to(torch.bfloat16)
    K.conv_dgrad2(to_nhwc(dy, cout), wd, dx, res, None, n, hw, hw, cp, cout, k, s, p, kgd)
    assert _rel(dx[..., :cin], dref + res[..., :cin].float()) < 1e-2, (shape, tile)


@pytest.mark.parametrize("bn", [64, 128, 256, "halo"])
@pytest.mark.parametrize("shape", [(32, 64, 64, 32, 3, 1, 1), (16, 128, 128, 16, 3, 1, 1), (16, 256, 256, 8, 3, 1, 1),
                                   (16, 512, 512, 4, 3, 1, 1), (4, 64, 128, 64, 3, 1, 1), (3, 64, 64, 56, 3, 1, 1),
                                   (5, 128, 128, 28, 3, 1, 1), (3, 512, 512, 7, 3, 1, 1)])
def test_conv2_tap_reuse(shape, bn, monkeypatch):
    """The tap-reuse mainloop (conv2_kernel TAPR: one staged window per kernel row feeds its three
    taps, zero row at the image-row edges) at every tile width, and its halo mode (tiles that
    start mid-row, any width: the ResNet-50 56/28/14/7 layers; forced on the power-of-two shapes
    too): fwd (+ BN statistics) and dgrad (+ residual, + fused BN-backward sums) against torch fp32."""
    n, cin, cout, hw, k, s, p = shape
    extra = ""
    if bn == "halo":
        monkeypatch.setenv("PSX_TUNE", "cv_tapr_halo=1" + extra)
    elif (n * hw * hw) % bn or bn % hw:
        pytest.skip("tile does not hold whole image rows")
    else:
        monkeypatch.setenv("PSX_TUNE", f"cv_tapr_bn={bn}" + extra)
    torch.manual_seed(4)
    x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(cout, cin, k, k, device=DEV) / (cin * k * k) ** 0.5).to(torch.bfloat16).float()
    wf, wd, cp, kg, kgd = make_operands(w)
    y = torch.empty(n, hw, hw, cout, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(K.STAT_SLOTS, 2, cout, device=DEV)
    K.conv_fwd2(to_nhwc(x, cp), wf, y, stats, _ws(n, hw, hw, cout, kg), n, hw, hw, cp, cout, k, s, p, kg)
    ref = F.conv2d(x, w, stride=s, padding=p).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2, (shape, bn)
    yq = y.float().reshape(-1, cout)
    assert torch.allclose(stats[:, 0].sum(0), yq.sum(0), rtol=1e-3, atol=5e-2), (shape, bn)
    assert torch.allclose(stats[:, 1].sum(0), (yq * yq).sum(0), rtol=1e-3, atol=5e-2), (shape, bn)
    dy = torch.randn(n, cout, hw, hw, device=DEV).to(torch.bfloat16).float()
    dref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w, dy, stride=s, padding=p).permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.bfloat16, device=DEV)
    res = torch.randn(n, hw, hw, cp, device=DEV).to(torch.bfloat16)
    o = torch.randn(n, hw, hw, cp, device=DEV).to(torch.bfloat16)
    y1 = torch.randn(n, hw, hw, cp, device=DEV).to(torch.bfloat16)
    saved = torch.stack([0.1 * torch.randn(cp, device=DEV), 1.0 + torch.rand(cp, device=DEV)])
    part = torch.zeros(K.STAT_SLOTS, 2, cp, device=DEV)
    bst = K.bwd_stats_desc(part, o, y1, saved)
    K.conv_dgrad2(to_nhwc(dy, cout), wd, dx, res, _ws(n, hw, hw, cp, kgd), n, hw, hw, cp, cout, k, s, p, kgd, bst=bst)
    assert _rel(dx[..., :cin], dref + res[..., :cin].float()) < 1e-2, (shape, bn)
    dz = (dx.float() * (o.float() > 0)).reshape(-1, cp)
    xhat = ((y1.float().reshape(-1, cp) - saved[0]) * saved[1])
    assert torch.allclose(part[:, 0].sum(0), dz.sum(0), rtol=1e-3, atol=5e-2), (shape, bn)
    assert torch.allclose(part[:, 1].sum(0), (dz * xhat).sum(0), rtol=1e-3, atol=5e-2), (shape, bn)


@pytest.mark.parametrize("shape", [(128, 64, 128, 32), (128, 128, 256, 16), (128, 256, 512, 8), (8, 128, 256, 28)])
def test_conv_dgrad2_shortcut_fold(shape):
    """bf16: the 3x3/s2 data gradient + the folded 1x1/s2 shortcut data gradient in one launch
    (psx_conv_dgrad2_sc) against torch fp32 of both convs summed."""
    torch.manual_seed(7)
    n, cin, cout, hw = shape
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (cin * 9) ** 0.5).to(torch.bfloat16).float()
    w2 = (torch.randn(cout, cin, 1, 1, device=DEV) / cin ** 0.5).to(torch.bfloat16).float()
    _, wd, cp, _, kgd = make_operands(w)
    _, wd2, _, _, kgd2 = make_operands(w2)
    oh = (hw - 1) // 2 + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    dy2 = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w, dy, stride=2, padding=1)
    ref = (ref + torch.nn.grad.conv2d_input((n, cin, hw, hw), w2, dy2, stride=2)).permute(0, 2, 3, 1)
    dx = torch.empty(n, hw, hw, cp, dtype=torch.bfloat16, device=DEV)
    assert K.conv_dgrad2_sc(to_nhwc(dy, cout), wd, dx, None, n, hw, hw, cp, cout, kgd, to_nhwc(dy2, cout), wd2, kgd2)
    assert _rel(dx[..., :cin], ref) < 1e-2, shape


def test_stem_conv_direct():
    """bf16: the direct stem conv (stem.hip) and its BN statistics against torch fp32."""
    K.set_deterministic(None)  # an earlier engine test may have left the process in deterministic mode
    torch.manual_seed(11)
    n = 64
    x = torch.randn(n, 3, 32, 32, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(64, 3, 3, 3, device=DEV) / 27 ** 0.5).to(torch.bfloat16).float()
    wf, _, cp, kg, _ = make_operands(w)
    y = torch.empty(n, 32, 32, 64, dtype=torch.bfloat16, device=DEV)
    st = torch.zeros(K.STAT_SLOTS, 2, 64, device=DEV)
    assert K.stem_conv(to_nhwc(x, cp), wf, y, st, n, 32, 32, 3, cp, 64, kg)
    assert _rel(y, F.conv2d(x, w, padding=1).permute(0, 2, 3, 1)) < 1e-2
    q = y.float().reshape(-1, 64)
    assert torch.allclose(st[:, 0].sum(0), q.sum(0), rtol=1e-3, atol=5e-2)
    assert torch.allclose(st[:, 1].sum(0), (q * q).sum(0), rtol=1e-3, atol=5e-2)


@pytest.mark.parametrize("n", [2, 3])
def test_stem7_conv_bf16(n):
    """bf16: the ImageNet stem on the MFMA (stem.hip stem7_fwd_bf16_kernel: 3 -> 64, 7x7 / stride 2
    / pad 3, 224 -> 112, 4 taps x 8 channels per v_mfma_f32_16x16x32_bf16) and its shifted BN
    statistics of the stored bf16 values, against torch fp32 on the same bf16 operands."""
    torch.manual_seed(14)
    x = torch.randn(n, 3, 224, 224, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(64, 3, 7, 7, device=DEV) / 147 ** 0.5).to(torch.bfloat16).float()
    wf, _, cp, kg, _ = make_operands(w)
    assert cp == 8
    y = torch.full((n, 112, 112, 64), float("nan"), device=DEV).to(torch.bfloat16)
    st = torch.zeros(K.STAT_SLOTS, 2, 64, device=DEV)
    sh = 0.1 * torch.randn(64, device=DEV)
    assert K.stem_conv(to_nhwc(x, cp), wf, y, st, n, 224, 224, 3, cp, 64, kg, sshift=sh, k=7)
    ref = F.conv2d(x, w, stride=2, padding=3).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
    d = y.double().reshape(-1, 64) - sh.double()
    assert torch.allclose(st[:, 0].double().sum(0), d.sum(0), rtol=1e-3, atol=5e-2)
    assert torch.allclose(st[:, 1].double().sum(0), (d * d).sum(0), rtol=1e-3, atol=5e-2)
