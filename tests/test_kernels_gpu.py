"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Runs on an MI355X only (``-m gpu``). Inputs are bf16-representable so the reference sees the
exact operands the kernel sees; tolerances are bf16-output level.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def _pow2(v):
    p = 8
    while p < v:
        p *= 2
    return p


def make_operands(w):
    """OIHW fp32 weight -> (wf [OC][Kg] bf16, wd [Cp][Kgd] bf16) through the unpack kernel."""
    oc, cin, k, _ = w.shape
    cp = _pow2(cin)
    kg = -(-(k * k * cp) // 64) * 64
    kgd = k * k * oc
    wbuf = torch.zeros(oc * kg + cp * kgd, dtype=torch.bfloat16, device=DEV)
    raw = np.zeros(1, dtype=np.dtype([("o", "<i8", 3), ("i", "<i4", 8)]))
    raw[0]["o"] = (0, 0, oc * kg)
    raw[0]["i"] = (oc, cin, k, k, cp, kg, kgd, 0)
    desc = torch.from_numpy(raw.view(np.uint8).copy()).to(DEV)
    K.param_unpack(w.contiguous().reshape(-1), desc, 1, wbuf)
    return wbuf[:oc * kg], wbuf[oc * kg:], cp, kg, kgd


def to_nhwc(x, cp):
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, cp, dtype=torch.bfloat16, device=DEV)
    out[..., :c] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return out


# (batch, cin, cout, hw, k, stride, pad): every distinct ResNet-18 CIFAR conv + the stem
R18_SHAPES = [
    (8, 3, 64, 32, 3, 1, 1),
    (8, 64, 64, 32, 3, 1, 1),
    (8, 64, 128, 32, 3, 2, 1),
    (8, 64, 128, 32, 1, 2, 0),
    (8, 128, 128, 16, 3, 1, 1),
    (8, 128, 256, 16, 3, 2, 1),
    (8, 128, 256, 16, 1, 2, 0),
    (8, 256, 256, 8, 3, 1, 1),
    (8, 256, 512, 8, 3, 2, 1),
    (8, 256, 512, 8, 1, 2, 0),
    (8, 512, 512, 4, 3, 1, 1),
    (128, 64, 64, 32, 3, 1, 1),
]


@pytest.mark.parametrize("shape", R18_SHAPES)
def test_conv_wgrad(shape):
    torch.manual_seed(2)
    n, cin, cout, hw, k, s, p = shape
    x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    oh = (hw + 2 * p - k) // s + 1
    dy = torch.randn(n, cout, oh, oh, device=DEV).to(torch.bfloat16).float()
    ref = torch.nn.grad.conv2d_weight(x, (cout, cin, k, k), dy, stride=s, padding=p)
    cp = _pow2(cin)
    kg = -(-(k * k * cp) // 64) * 64
    # the split slabs of the weight-gradient mainloop (conv v2, tests/test_conv_v2_gpu.py for the
    # kernel itself) through both reductions: fp32 and the fp16 wire
    splits = K.conv_wgrad2_splits(n, hw, hw, cp, cout, k, s, p, kg)
    part = torch.zeros(splits * cout * kg, device=DEV)
    got = K.conv_wgrad2(to_nhwc(x, cp), to_nhwc(dy, cout), part, n, hw, hw, cp, cout, k, s, p, kg)
    assert got == splits
    out = torch.zeros(cout * cin * k * k, device=DEV)
    part2 = part.clone()  # the reduce consumes its partials (in-place pre-sum of many-split layers)
    K.wgrad_reduce(part, splits, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False)
    assert _rel(out.view_as(ref), ref) < 5e-3, shape
    out16 = torch.zeros(cout * cin * k * k, dtype=torch.float16, device=DEV)
    K.wgrad_reduce(part2, splits, cout, kg, cin, cp, k, 0.5, out16.data_ptr(), True)
    assert _rel(out16.view_as(ref).float(), 0.5 * ref) < 5e-3, shape


@pytest.mark.parametrize("c,hw,mode", [(64, 32, 0), (128, 16, 1), (256, 8, 2), (512, 4, 1)])
def test_bn_forward(c, hw, mode):
    torch.manual_seed(3)
    n = 16
    y = (torch.randn(n, hw, hw, c, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    yf = y.float().reshape(-1, c)
    part = torch.stack([yf.sum(0), (yf * yf).sum(0)]).reshape(1, 2, c).contiguous()
    gamma = torch.rand(c, device=DEV) + 0.5
    beta = torch.randn(c, device=DEV)
    rm = torch.zeros(c, device=DEV)
    rv = torch.ones(c, device=DEV)
    aff = torch.zeros(2, c, device=DEV)
    saved = torch.zeros(2, c, device=DEV)
    K.bn_finalize(part, 1, c, yf.shape[0], gamma, beta, 1e-5, 0.1, rm, rv, aff, saved)
    ynchw = y.float().permute(0, 3, 1, 2)
    rm_ref = torch.zeros(c, device=DEV)
    rv_ref = torch.ones(c, device=DEV)
    ref = F.batch_norm(ynchw, rm_ref, rv_ref, gamma, beta, training=True, momentum=0.1, eps=1e-5)
    assert torch.allclose(rm, rm_ref, atol=1e-4, rtol=1e-4)
    assert torch.allclose(rv, rv_ref, atol=1e-3, rtol=1e-3)
    out = torch.empty_like(y)
    if mode == 0:
        K.bn_apply(y, aff, out, c, relu=True)
        ref = F.relu(ref)
    elif mode == 1:
        res = torch.randn_like(y.float()).to(torch.bfloat16)
        K.bn_apply(y, aff, out, c, relu=True, res=res)
        ref = F.relu(ref + res.float().permute(0, 3, 1, 2))
    else:
        res = torch.randn_like(y.float()).to(torch.bfloat16)
        aff2 = torch.stack([torch.rand(c, device=DEV), torch.randn(c, device=DEV)])
        K.bn_apply(y, aff, out, c, relu=True, res=res, affine2=aff2)
        ref = F.relu(ref + (res.float() * aff2[0] + aff2[1]).permute(0, 3, 1, 2))
    assert _rel(out, ref.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("c,hw,two", [(64, 32, False), (128, 16, True), (512, 4, False)])
def test_bn_backward(c, hw, two):
    torch.manual_seed(4)
    n = 16
    y = (torch.randn(n, c, hw, hw, device=DEV) * 1.5).to(torch.bfloat16).float().requires_grad_(True)
    y2 = (torch.randn(n, c, hw, hw, device=DEV)).to(torch.bfloat16).float().requires_grad_(True)
    gamma = (torch.rand(c, device=DEV) + 0.5).requires_grad_(True)
    beta = torch.randn(c, device=DEV).requires_grad_(True)
    g2 = (torch.rand(c, device=DEV) + 0.5).requires_grad_(True)
    b2 = torch.randn(c, device=DEV).requires_grad_(True)
    z = F.batch_norm(y, None, None, gamma, beta, training=True, eps=1e-5)
    if two:
        z = z + F.batch_norm(y2, None, None, g2, b2, training=True, eps=1e-5)
    o = F.relu(z)
    go = torch.randn_like(o).to(torch.bfloat16).float()
    o.backward(go)
    nhwc = lambda t: t.detach().permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)  # noqa: E731
    npix = n * hw * hw
    saved = torch.stack([y.detach().mean((0, 2, 3)), y.detach().var((0, 2, 3), unbiased=False).add(1e-5).rsqrt()])
    saved2 = torch.stack([y2.detach().mean((0, 2, 3)), y2.detach().var((0, 2, 3), unbiased=False).add(1e-5).rsqrt()])
    T = K.bn_bwd_reduce_T(npix, c)
    part = torch.zeros(T * 3 * c, device=DEV)
    oh = nhwc(o)
    Tg = K.bn_bwd_reduce(nhwc(go), oh, nhwc(y), saved, part, npix, c, y2=nhwc(y2) if two else None,
                         saved2=saved2 if two else None)
    ns = 3 if two else 2
    coef = torch.zeros(3, c, device=DEV)
    coef2 = torch.zeros(3, c, device=DEV)
    dgb = torch.zeros(2, c, device=DEV)
    dgb2 = torch.zeros(2, c, device=DEV)
    K.bn_bwd_finalize(part, Tg, ns, 1, c, npix, gamma.detach(), saved, coef, dgb.data_ptr(), dgb.data_ptr() + 4 * c,
                      1.0, False)
    assert torch.allclose(dgb[0], gamma.grad, rtol=2e-2, atol=2e-2)
    assert torch.allclose(dgb[1], beta.grad, rtol=2e-2, atol=2e-2)
    dx = torch.empty(n, hw, hw, c, dtype=torch.bfloat16, device=DEV)
    dx2 = torch.empty_like(dx)
    dz = torch.empty_like(dx)
    if two:
        K.bn_bwd_finalize(part, Tg, ns, 2, c, npix, g2.detach(), saved2, coef2, dgb2.data_ptr(),
                          dgb2.data_ptr() + 4 * c, 1.0, False)
        assert torch.allclose(dgb2[0], g2.grad, rtol=2e-2, atol=2e-2)
        K.bn_bwd_apply(nhwc(go), oh, nhwc(y), coef, dx, c, y2=nhwc(y2), coef2=coef2, dx2=dx2, dzout=dz)
        assert _rel(dx2, y2.grad.permute(0, 2, 3, 1)) < 3e-2
    else:
        K.bn_bwd_apply(nhwc(go), oh, nhwc(y), coef, dx, c, dzout=dz)
    assert _rel(dx, y.grad.permute(0, 2, 3, 1)) < 3e-2
    assert _rel(dz, (go * (o > 0)).permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("b,hw,c,k", [(32, 16, 512, 100), (40, 49, 2048, 1000)])
def test_head_fwd_bwd(b, hw, c, k):
    """Fused per-sample head (ResNet-18) and the split pool/GEMM/softmax path (ResNet-50 2048 ->
    1000, batch not a multiple of the 32-sample tile) against torch fp32 autograd."""
    torch.manual_seed(5)
    side = int(hw ** 0.5)
    act = torch.rand(b, side, side, c, device=DEV).to(torch.bfloat16)
    w = (torch.randn(k, c, device=DEV) * 0.05).requires_grad_(True)
    bias = torch.randn(k, device=DEV).requires_grad_(True)
    lab = torch.randint(0, k, (b,), device=DEV, dtype=torch.int32)
    a = act.float().requires_grad_(True)
    pooled_ref = a.mean((1, 2))
    logits = pooled_ref @ w.t() + bias
    loss = F.cross_entropy(logits, lab.long())
    loss.backward()
    pooled = torch.zeros(b, c, device=DEV)
    dlog = torch.zeros(b, k, device=DEV)
    dact = torch.empty_like(act)
    lossv = torch.zeros(b, device=DEV)
    correct = torch.zeros(1, dtype=torch.int32, device=DEV)
    y1 = torch.randn(b, side, side, c, device=DEV).to(torch.bfloat16)
    saved = torch.stack([0.1 * torch.randn(c, device=DEV), 1.0 + torch.rand(c, device=DEV)])
    part = torch.zeros(K.STAT_SLOTS, 2, c, device=DEV)
    fused = K.head_fwd_bwd(act, b, hw, c, w.detach(), bias.detach(), k, lab, pooled, dlog, dact, lossv, correct,
                           bst=K.bwd_stats_desc(part, act, y1, saved))
    assert fused == (k * c <= (1 << 18))  # the per-sample head also produces the BN-backward sums
    if fused:
        dz = (dact.float() * (act.float() > 0)).reshape(-1, c)
        xhat = (y1.float().reshape(-1, c) - saved[0]) * saved[1]
        assert torch.allclose(part[:, 0].sum(0), dz.sum(0), rtol=1e-3, atol=1e-5)
        assert torch.allclose(part[:, 1].sum(0), (dz * xhat).sum(0), rtol=1e-3, atol=1e-5)
    else:
        assert not part.any()
    assert _rel(pooled, pooled_ref) < 1e-5
    assert abs(lossv.mean().item() - loss.item()) < 1e-3
    assert correct.item() == int((logits.argmax(1) == lab.long()).sum())
    assert _rel(dact, a.grad) < 1e-2
    dw = torch.zeros(k, c, device=DEV)
    db = torch.zeros(k, device=DEV)
    K.head_wgrad(dlog, pooled, b, k, c, dw.data_ptr(), db.data_ptr(), 1.0, False)
    assert _rel(dw, w.grad) < 1e-3 and _rel(db, bias.grad) < 1e-3


def test_sgd_and_codec():
    torch.manual_seed(6)
    n = 1 << 20
    p = torch.randn(n, device=DEV)
    g = torch.randn(n, device=DEV)
    g16 = torch.empty(n, dtype=torch.float16, device=DEV)
    K.fp16_pack(g, g16, 1.0)
    assert torch.equal(g16, g.half())
    back = torch.empty(n, device=DEV)
    K.fp16_unpack(g16, back, 2.0)
    assert torch.equal(back, g.half().float() * 2)
    ref = p - 0.1 * 0.25 * g16.float()
    p1 = p.clone()
    K.sgd_apply(p1, g16, 0.1, gscale=0.25)
    assert torch.allclose(p1, ref, atol=1e-6)
    # momentum + weight decay (baseline optimizer semantics of torch.optim.SGD)
    p2 = p.clone().requires_grad_(False)
    buf = torch.zeros(n, device=DEV)
    tp = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([tp], lr=0.1, momentum=0.9, weight_decay=5e-4)
    for it in range(3):
        tp.grad = g.clone()
        opt.step()
        K.sgd_apply(p2, g, 0.1, momentum=0.9, wd=5e-4, buf=buf, first=(it == 0))
    assert torch.allclose(p2, tp.detach(), atol=1e-5)


def test_grad_aggregate():
    torch.manual_seed(7)
    n = 100003
    srcs = [torch.randn(n, device=DEV).half() for _ in range(3)]
    ptrs = torch.tensor([s.data_ptr() for s in srcs], dtype=torch.int64, device=DEV)
    dst = torch.zeros(n, device=DEV)
    K.grad_aggregate(ptrs, 3, True, dst, n, scale=1 / 3)
    ref = sum(s.float() for s in srcs) / 3
    assert torch.allclose(dst, ref, atol=1e-5)


def test_augment_matches_torchvision_semantics():
    n, b = 64, 16
    img = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labels = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    idx = torch.randperm(n, device=DEV)[:b].to(torch.int32)
    out = torch.empty(b, 32, 32, 8, dtype=torch.bfloat16, device=DEV)
    olab = torch.empty(b, dtype=torch.int32, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    mean, std = (0.5071, 0.4867, 0.4408), (0.2675, 0.2565, 0.2761)
    K.augment(img, labels, idx, out, olab, b, 32, 32, 4, 7, step, False, mean, std)
    ref = (img[idx.long()].float() / 255 - torch.tensor(mean, device=DEV)) / torch.tensor(std, device=DEV)
    assert torch.equal(olab, labels[idx.long()])
    assert _rel(out[..., :3], ref) < 1e-2
    assert out[..., 3:].abs().max().item() == 0
    K.augment(img, labels, idx, out, olab, b, 32, 32, 4, 7, step, True, mean, std)
    # every augmented image is a shifted (and maybe flipped) window of the normalized original
    pad_val = (0 - torch.tensor(mean, device=DEV)) / torch.tensor(std, device=DEV)
    for i in range(b):
        src = torch.empty(40, 40, 3, device=DEV)
        src[:] = pad_val
        src[4:36, 4:36] = ref[i]
        found = False
        for flip in (False, True):
            o = out[i, :, :, :3].float()
            o = o.flip(1) if flip else o
            for dy in range(9):
                for dx in range(9):
                    if (src[dy:dy + 32, dx:dx + 32] - o).abs().max() < 0.05:
                        found = True
        assert found, i
