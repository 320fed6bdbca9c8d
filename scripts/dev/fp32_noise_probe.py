"""Diagnostic: run-to-run spread of the fp32 engine's gradients vs fp64 references (GPU and CPU)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F

import psx  # noqa: F401
from psx.models.engine import HipResNetEngine
from psx.models.layout import ParamLayout
from psx.models.resnet import ResNet18
from psx.ops import kernels as K

torch.manual_seed(0)
B = int(os.environ.get("B", "16"))
model = ResNet18(100)
layout = ParamLayout.from_module(model)
arena0, _ = layout.pack(model)
arena0 = arena0.cuda()
eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, dtype=torch.float32)
x = torch.randn(B, 3, 32, 32, device="cuda")
y = torch.randint(0, 100, (B,), device="cuda")


def run_engine():
    a = arena0.clone()
    eng.unpack(a)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 32, 32, eng.x0.shape[-1])
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(a, train=True)
    eng.head(a, backward=True)
    eng.backward(a)
    torch.cuda.synchronize()
    return {n: layout.grad_view(eng.grads, n).double().cpu().clone() for n, _ in model.named_parameters()}


def run_ref(dev, dtype):
    m = copy.deepcopy(model).to(dev).to(dtype)
    m.train()
    F.cross_entropy(m(x.to(dev, dtype)), y.to(dev)).backward()
    return {n: p.grad.double().cpu() for n, p in m.named_parameters()}


e1, e2 = run_engine(), run_engine()
g64 = run_ref("cuda", torch.float64)
g64b = run_ref("cuda", torch.float64)
c64 = run_ref("cpu", torch.float64)
g32 = run_ref("cuda", torch.float32)


def err(a, b, n):
    return ((a[n] - b[n]).norm() / b[n].norm().clamp_min(1e-30)).item()


print(f"{'tensor':28s} {'e1-e2':>9s} {'e1-cpu64':>9s} {'g64-cpu64':>9s} {'g64-g64b':>9s} {'t32-cpu64':>9s}")
for n, _ in model.named_parameters():
    if n.endswith("weight") and ("conv" in n or "fc" in n or "shortcut.0" in n):
        print(f"{n:28s} {err(e1, e2, n):9.2e} {err(e1, c64, n):9.2e} {err(g64, c64, n):9.2e} {err(g64, g64b, n):9.2e} "
              f"{err(g32, c64, n):9.2e}")
