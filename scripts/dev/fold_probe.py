# which gradient tensors differ between PSX_WINO_BNFOLD=1/0 (deterministic fp32 engine step)
import os, sys
sys.path.insert(0, os.getcwd())
import torch
import psx  # noqa
from psx.models.engine import HipResNetEngine
from psx.models.layout import ParamLayout
from psx.models.resnet import ResNet18

torch.manual_seed(1)
model = ResNet18(100)
layout = ParamLayout.from_module(model)
arena0, _ = layout.pack(model)
arena0 = arena0.cuda()
B = 32
imgs = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device="cuda")
labs = torch.randint(0, 100, (64,), dtype=torch.int32, device="cuda")
out = {}
for fold in ("1", "0"):
    os.environ["PSX_WINO_BNFOLD"] = fold
    eng = HipResNetEngine(model, layout, B, dtype=torch.float32, deterministic=True)
    eng.index.copy_(torch.arange(B, dtype=torch.int32, device="cuda"))
    a = arena0.clone()
    eng.train_step(a, imgs, labs)
    torch.cuda.synchronize()
    out[fold] = eng.grads.double().clone()
g1, g0 = out["1"], out["0"]
for name, e in layout.entries.items():
    if e.region != "param":
        continue
    v1, v0 = layout.grad_view(g1, name), layout.grad_view(g0, name)
    if not torch.equal(v1, v0):
        d = (v1 - v0).abs().max().item() / max(v0.abs().max().item(), 1e-30)
        print(f"{name}: rel {d:.3e} ndiff {(v1 != v0).sum().item()} / {v1.numel()}")
print("done")
