"""Per-tensor gradient agreement: HIP engine vs torch fp32, torch bf16-autocast vs fp32, engine run-to-run."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
import psx
from psx.models.engine import HipResNetEngine
from psx.models.layout import ParamLayout
from psx.models.resnet import ResNet18
from psx.ops import kernels as K
DEV = 'cuda'
def cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()
torch.manual_seed(0)
B = int(os.environ.get('B', '32'))
model = ResNet18(100)
with torch.no_grad():
    for m in model.modules():
        if isinstance(m, torch.nn.Conv2d): m.weight.copy_(m.weight.to(torch.bfloat16).float())
layout = ParamLayout.from_module(model)
arena, _ = layout.pack(model)
arena = arena.to(DEV)
model = model.to(DEV)
eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32)
x = torch.randn(B, 3, 32, 32, device=DEV).to(torch.bfloat16).float()
y = torch.randint(0, 100, (B,), device=DEV)
def run_engine():
    a = arena.clone()
    eng.unpack(a)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 32, 32, 8)
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(a, train=True); eng.head(a, backward=True); eng.backward(a)
    torch.cuda.synchronize()
    return eng.grads.clone(), eng.loss.mean().item()
g1, l1 = run_engine()
g2, l2 = run_engine()
model.train(); model.zero_grad()
loss = F.cross_entropy(model(x), y); loss.backward()
ref = {n: p.grad.clone() for n, p in model.named_parameters()}
model.zero_grad()
with torch.autocast('cuda', dtype=torch.bfloat16):
    lb = F.cross_entropy(model(x), y)
lb.backward()
refb = {n: p.grad.clone() for n, p in model.named_parameters()}
print(f"loss engine {l1:.5f} {l2:.5f} torch32 {loss.item():.5f} torch_bf16 {lb.item():.5f}")
print(f"{'param':32s} {'eng~t32':>8s} {'eng~eng':>8s} {'tbf~t32':>8s}")
for n in ref:
    a = layout.grad_view(g1, n); b = layout.grad_view(g2, n)
    print(f"{n:32s} {cos(a, ref[n]):8.4f} {cos(a, b):8.5f} {cos(refb[n], ref[n]):8.4f}")
