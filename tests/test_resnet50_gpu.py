"""ResNet-50 (ImageNet shape) on the HIP engine: max-pool kernels and one whole training step
vs torch fp32 autograd (same acceptance rule as the ResNet-18 test: per-tensor gradient cosine
no worse than torch's own bf16-autocast path, minus a margin)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import ResNet50  # noqa: E402
from psx.ops import kernels as K  # noqa: E402

from .test_engine_gpu import _bf16_round_, _cos  # noqa: E402

DEV = "cuda"


@pytest.mark.parametrize("shape", [(4, 112, 112, 64), (2, 7, 9, 16)])
def test_maxpool_fwd_bwd_matches_torch(shape):
    torch.manual_seed(0)
    B, H, W, C = shape
    x = torch.randn(B, H, W, C, device=DEV).to(torch.bfloat16)
    x[0, 0, 0, :8] = x[0, 0, 1, :8]  # exact ties: first maximum in window order wins (torch rule)
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y = torch.empty(B, OH, OW, C, dtype=torch.bfloat16, device=DEV)
    arg = torch.empty(B, OH, OW, C, dtype=torch.uint8, device=DEV)
    K.maxpool3s2_fwd(x, y, arg)
    xr = x.permute(0, 3, 1, 2).float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.permute(0, 3, 1, 2).float(), yr.detach())
    dy = torch.randn(B, OH, OW, C, device=DEV).to(torch.bfloat16)
    dx = torch.empty_like(x)
    K.maxpool3s2_bwd(dy, arg, dx)
    yr.backward(dy.permute(0, 3, 1, 2).float())
    ref = xr.grad.permute(0, 2, 3, 1)
    assert torch.allclose(dx.float(), ref, atol=2e-2, rtol=1e-2)


@pytest.fixture(scope="module")
def r50():
    torch.manual_seed(0)
    B = 16
    model = ResNet50(1000)
    # damp the residual branches (cf. torchvision's zero_init_residual) so a random-init
    # 50-layer net's gradients are not chaotic and a gradient comparison is meaningful
    with torch.no_grad():
        for name, m in model.named_modules():
            if name.endswith("bn3"):
                m.weight.fill_(0.2)
    _bf16_round_(model)
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    model = model.to(DEV)
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, in_hw=(224, 224))
    x = torch.randn(B, 3, 224, 224, device=DEV).to(torch.bfloat16).float()
    y = torch.randint(0, 1000, (B,), device=DEV)
    return model, layout, arena.to(DEV), eng, x, y


def test_resnet50_train_step_matches_torch(r50):
    model, layout, arena, eng, x, y = r50
    assert layout.param_numel == 25_557_032
    a = arena.clone()
    eng.unpack(a)
    K.nchw_to_nhwc(x, eng.x0, x.shape[0], 3, 224, 224, 8)
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(a, train=True)
    eng.head(a, backward=True)
    eng.backward(a)
    torch.cuda.synchronize()
    model.train()
    model.zero_grad()
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    ref32 = {n: p.grad.clone() for n, p in model.named_parameters()}
    model.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        F.cross_entropy(model(x), y).backward()
    ref16 = {n: p.grad.clone() for n, p in model.named_parameters()}
    assert abs(eng.loss.mean().item() - loss.item()) < 0.02 * max(1.0, loss.item())
    ce, cb = [], []
    for name in ref32:
        g = layout.grad_view(eng.grads, name)
        c_eng, c_bf16 = _cos(g, ref32[name]), _cos(ref16[name], ref32[name])
        ce.append(c_eng)
        cb.append(c_bf16)
        # relative to torch's own bf16 path; where even that is far from fp32 the tensor's
        # gradient is chaotic and only the median check below applies
        if c_bf16 > 0.5:
            assert c_eng > c_bf16 - 0.1, (name, c_eng, c_bf16)
    ce.sort()
    cb.sort()
    assert ce[len(ce) // 2] > cb[len(cb) // 2] - 0.02, (ce[:5], cb[:5])
    fcw = layout.grad_view(eng.grads, "fc.weight")
    assert _cos(fcw, ref32["fc.weight"]) > 0.99


def test_resnet50_graph_step(r50):
    model, layout, arena, eng, x, y = r50
    n = 64
    imgs = torch.randint(0, 256, (n, 224, 224, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 1000, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    a = arena.clone()
    eng.capture(a, imgs, labs, warmup=1)
    a.copy_(arena)
    eng.step_graph()
    torch.cuda.synchronize()
    assert torch.isfinite(eng.grads).all() and eng.grads.abs().sum() > 0
    assert 5.0 < eng.loss.mean().item() < 9.0  # ~ln(1000) at random init


def test_resnet50_fp32_step_matches_torch_fp64():
    """The fp32 ResNet-50 engine step (the BASELINE config-5 path: ImageNet stem on the MFMA with
    its patch in LDS, Winograd on every 3x3 / stride-1 layer including the 14x14 / 7x7 stages'
    partial edge tiles, BN folded into their input transforms) against float64 autograd: loss, and
    per-parameter gradient error no worse than torch's own fp32 autograd (x3, floor 8e-3) at the
    worst tensor and the median (residual branches damped as in the r50 fixture)."""
    import copy

    torch.manual_seed(3)
    B = 4
    model = ResNet50(1000)
    with torch.no_grad():
        for name, m in model.named_modules():
            if name.endswith("bn3"):
                m.weight.fill_(0.2)
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    arena = arena.to(DEV)
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, in_hw=(224, 224), dtype=torch.float32,
                          deterministic=True)
    assert {"layer1.0.conv2", "layer3.1.conv2", "layer4.1.conv2"} <= set(eng.wino_layers), sorted(eng.wino_layers)
    x = torch.randn(B, 3, 224, 224, device=DEV)
    y = torch.randint(0, 1000, (B,), device=DEV)
    eng.unpack(arena)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 224, 224, eng.x0.shape[-1])
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
    loss = F.cross_entropy(ref(x.double()), y)
    loss.backward()
    assert abs(eng.loss.double().mean().item() - loss.item()) < 1e-4 * max(1.0, loss.item())
    rows = []
    for name, p in ref.named_parameters():
        g = layout.grad_view(eng.grads, name).double()
        nrm = p.grad.norm().clamp_min(1e-30)
        rows.append((name, ((g - p.grad).norm() / nrm).item(),
                     ((m32.get_parameter(name).grad.double() - p.grad).norm() / nrm).item()))
    errs, errs32 = sorted(r[1] for r in rows), sorted(r[2] for r in rows)
    print("r50 fp32 engine: worst %.2e median %.2e; torch fp32 worst %.2e median %.2e"
          % (errs[-1], errs[len(errs) // 2], errs32[-1], errs32[len(errs32) // 2]))
    assert errs[-1] <= max(3 * errs32[-1], 8e-3), max(rows, key=lambda r: r[1])
    assert errs[len(errs) // 2] <= max(3 * errs32[len(errs32) // 2], 5e-3)
