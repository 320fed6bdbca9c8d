"""Fused fp32 Winograd weight gradient (csrc/kernels/wino_wgrad.hip: x / dy transformed in
registers, the 36 tile-reduction GEMMs on v_mfma_f32_16x16x4f32, partial slabs reduced by the
output transform) against torch float64 ``conv2d_weight``: every ResNet-18 / ResNet-50 Winograd
shape class, fp32 and fp16-wire outputs, the forward BN + ReLU folded into the x load (xaff), the
BN-backward apply folded into the dy load (bwd_in), and bit-reproducibility (fixed reduction
order). Bar: max-abs error <= 1e-4 of the reference's max-abs (the fp32 test bar; the
F(3x3,4x4) transforms measure ~1e-6..1e-5 there)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.ops import kernels as K  # noqa: E402

from .test_wino_fused_gpu import _bwd_case, _bwd_ref  # noqa: E402

DEV = "cuda"
TOL = 1e-4


def _rel(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _wref(x_nhwc, dy_nhwc, k, c):
    return torch.nn.grad.conv2d_weight(x_nhwc.double().permute(0, 3, 1, 2), (k, c, 3, 3),
                                       dy_nhwc.double().permute(0, 3, 1, 2), padding=1)


def _run(x, dy, nb, h, c, k, out_dtype=torch.float32, xaff=None, bwd_in=None):
    q = K.wino_wgrad_fused_q(nb, h, h, c, k)
    assert q > 0
    part = torch.full((36 * q * k * c,), float("nan"), device=DEV)
    out = torch.full((k * c * 9,), float("nan"), device=DEV, dtype=out_dtype)
    K.wino_wgrad_fused(x, dy, part, out, nb, h, h, c, k, xaff=xaff, bwd_in=bwd_in)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("nb,h,c,k", [(16, 32, 64, 64), (32, 16, 128, 128), (32, 8, 256, 256), (32, 4, 512, 512),
                                      (8, 8, 64, 128), (4, 16, 32, 16), (4, 56, 64, 64), (16, 28, 128, 128)])
def test_wgrad_fused_vs_fp64(nb, h, c, k):
    torch.manual_seed(nb * h + c + k)
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    dy = torch.randn(nb, h, h, k, device=DEV)
    out = _run(x, dy, nb, h, c, k)
    assert _rel(out, _wref(x, dy, k, c)) < TOL


def test_wgrad_fused_fp16_wire_and_scale():
    torch.manual_seed(3)
    nb, h, c, k = 16, 16, 128, 128
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    dy = torch.randn(nb, h, h, k, device=DEV) * 0.01
    q = K.wino_wgrad_fused_q(nb, h, h, c, k)
    part = torch.empty(36 * q * k * c, device=DEV)
    out = torch.empty(k * c * 9, device=DEV, dtype=torch.float16)
    K.wino_wgrad_fused(x, dy, part, out, nb, h, h, c, k, scale=0.5)
    torch.cuda.synchronize()
    ref = 0.5 * _wref(x, dy, k, c)
    assert _rel(out, ref) < 2e-3  # the fp16 wire's own rounding (2^-11)


@pytest.mark.parametrize("nb,h,c,k", [(16, 32, 64, 64), (16, 16, 128, 128), (32, 4, 512, 512)])
def test_wgrad_fused_bn_relu_fold(nb, h, c, k):
    """x = relu(scale * y + shift) of the stored pre-BN y (the forward folded that BN into the
    next conv's input transform, so the activation was never written); padding stays zero."""
    torch.manual_seed(c + 7)
    y = torch.randn(nb, h, h, c, device=DEV) * 2.0 + 0.5
    aff = torch.stack([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)]).contiguous()
    dy = torch.randn(nb, h, h, k, device=DEV)
    out = _run(y, dy, nb, h, c, k, xaff=aff)
    x = torch.relu(y.double() * aff[0].double() + aff[1].double())
    assert _rel(out, _wref(x, dy, k, c)) < TOL


@pytest.mark.parametrize("nb,h,c,k", [(8, 32, 64, 64), (4, 16, 128, 128)])
@pytest.mark.parametrize("aff", [False, True])
def test_wgrad_fused_bwd_fold(nb, h, c, k, aff):
    """dy = k1 dz + k2 y + k3 (the BN-backward apply folded into the load, the coefficients from
    the slot sums as wino_fused / wino_wgrad compute them) == the weight gradient of the float64
    BN backward; also with the x-side BN fold at the same time."""
    torch.manual_seed(k + c + aff)
    cnt = nb * h * h
    dz, yb, saved, gamma, part = _bwd_case(nb, h, k, seed=nb + h)
    coef = torch.full((3, k), float("nan"), device=DEV)
    dgb = torch.full((2, k), float("nan"), device=DEV)
    ctr = torch.zeros(4, dtype=torch.int32, device=DEV)
    fin = K.bn_bwd_fin(gamma, saved, coef, dgb[0].data_ptr(), dgb[1].data_ptr(), ctr.data_ptr(), cnt, 1.0, k, False)
    y = torch.randn(nb, h, h, c, device=DEV)
    xa = torch.stack([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV)]).contiguous() if aff else None
    out = _run(y, dz, nb, h, c, k, xaff=xa, bwd_in=(yb, part, fin))
    x = torch.relu(y.double() * xa[0].double() + xa[1].double()) if aff else y.double()
    dy_ref, _, _ = _bwd_ref(dz, yb, saved, gamma, part, cnt)
    assert _rel(out, _wref(x, dy_ref, k, c)) < TOL


def test_wgrad_fused_matches_three_launch_path():
    """Same layer through wino.hip's V / D / batched-GEMM path: the two Winograd weight gradients
    agree to fp32 transform rounding."""
    torch.manual_seed(11)
    nb, h, c, k = 32, 16, 128, 128
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    dy = torch.randn(nb, h, h, k, device=DEV)
    fused = _run(x, dy, nb, h, c, k)
    w = torch.randn(k, c, 3, 3, device=DEV)
    u = torch.empty(36 * k * c, device=DEV)
    K.wino_weights(w, u, k, c)
    v = torch.empty(K.wino_v_floats(nb, h, h, c), device=DEV)
    p = torch.empty(K.wino_p_floats(nb, h, h, c, k), device=DEV)
    K.wino_conv(x, u, torch.empty(nb, h, h, k, device=DEV), None, None, v, p, nb, h, h, c, k)
    q = K.wino_wgrad_q(nb, h, h, c, k)
    d = torch.empty(K.wino_v_floats(nb, h, h, k), device=DEV)
    wp = torch.empty(36 * q * k * c, device=DEV)
    g = torch.empty(k * c * 9, device=DEV)
    K.wino_wgrad(v, dy, d, wp, g, nb, h, h, c, k)
    torch.cuda.synchronize()
    assert _rel(fused, g) < 2e-5


def test_wgrad_fused_bit_reproducible():
    torch.manual_seed(5)
    nb, h, c, k = 16, 32, 64, 64
    x = torch.relu(torch.randn(nb, h, h, c, device=DEV))
    dy = torch.randn(nb, h, h, k, device=DEV)
    a = _run(x, dy, nb, h, c, k)
    b = _run(x, dy, nb, h, c, k)
    assert torch.equal(a, b)
