# fold vs unfolded: is the folded x operand bit-identical to the activation the apply writes?
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
eng = {}
for fold in ("1", "0"):
    os.environ["PSX_WINO_BNFOLD"] = fold
    e = HipResNetEngine(model, layout, B, dtype=torch.float32, deterministic=True)
    e.index.copy_(torch.arange(B, dtype=torch.int32, device="cuda"))
    a = arena0.clone()
    e.train_step(a, imgs, labs)
    torch.cuda.synchronize()
    eng[fold] = e
e1, e0 = eng["1"], eng["0"]
for j, b in enumerate(e1.spec.blocks[:4]):
    bs = b.bns[0]
    af1, af0 = e1.bn[bs.name]["affine"], e0.bn[bs.name]["affine"]
    y1, y0 = e1.blk[j]["y"][0], e0.blk[j]["y"][0]
    a0 = e0.blk[j]["a"][0]
    C = bs.c
    sc, sh = af0.view(-1)[:C].double(), af0.view(-1)[C:2 * C].double()
    xf = torch.relu((y0.double() * sc + sh).float())  # correctly rounded fma
    xm = torch.relu(y0 * af0.view(-1)[:C] + af0.view(-1)[C:2 * C])  # two roundings
    print(bs.name, "affine equal", torch.equal(af1, af0), "y equal", torch.equal(y1, y0),
          "a==fma", torch.equal(a0, xf), "a==mul+add", torch.equal(a0, xm),
          "ndiff fma", (a0 != xf).sum().item(), "ndiff mul+add", (a0 != xm).sum().item())
