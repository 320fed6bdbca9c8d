"""Where do two identical engine steps diverge? Per-tensor differences of forward activations
and backward gradients between two runs on the same input (fp32-atomic BN statistics are the
only intended source of run-to-run differences)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import build_model  # noqa: E402
from psx.utils.data import DeviceDataset  # noqa: E402

model = build_model("resnet18", None, seed=0)
lay = ParamLayout.from_module(model)
arena, _ = lay.pack(model)
arena = arena.cuda()
ds = DeviceDataset.synthetic(256, 32, 100, seed=3, device="cuda")
snaps = []
for run in range(2):
    eng = HipResNetEngine(model, lay, 64, in_hw=(32, 32))
    eng.index.copy_(torch.arange(64, dtype=torch.int32))
    a = arena.clone()
    eng.train_step(a, ds.images, ds.labels)
    torch.cuda.synchronize()
    s = {"x0": eng.x0.clone(), "y0": eng.y0.clone(), "a0": eng.a0.clone()}
    for j, d in enumerate(eng.blk):
        for i, t in enumerate(d["y"]):
            s[f"b{j}.y{i}"] = t.clone()
        for i, t in enumerate(d["a"]):
            s[f"b{j}.a{i}"] = t.clone()
        s[f"b{j}.out"] = d["out"].clone()
    s["pooled"] = eng.pooled.clone()
    s["dlogits"] = eng.dlogits.clone()
    s["dfinal"] = eng.dfinal.clone()
    for j in range(len(eng.blk) - 1, -1, -1):
        d = eng.blk[j]
        for i, t in enumerate(d["dy"]):
            s[f"b{j}.dy{i}"] = t.clone()
        s[f"b{j}.gin"] = d["gin"].clone()
    s["dy0"] = eng.dy0.clone()
    for name in list(eng.bn)[:4]:
        s[f"saved:{name}"] = eng.bn[name]["saved"].clone()
    snaps.append(s)
for k in snaps[0]:
    x, y = snaps[0][k].float(), snaps[1][k].float()
    nd = (x != y).sum().item()
    print(f"{k:24s} n={x.numel():9d} ndiff={nd:9d} maxdiff={(x - y).abs().max().item():.3e} max={x.abs().max().item():.3e}")
