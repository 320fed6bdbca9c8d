"""Per-tensor gradient differences: batched vs per-layer wgrad reduction (and run-to-run noise)."""
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
g = {}
for tag in ("1a", "1b", "0a", "0b"):
    os.environ["PSX_WGRAD_RBATCH"] = tag[0]
    eng = HipResNetEngine(model, lay, 64, in_hw=(32, 32))
    eng.index.copy_(torch.arange(64, dtype=torch.int32))
    a = arena.clone()
    eng.train_step(a, ds.images, ds.labels)
    torch.cuda.synchronize()
    g[tag] = eng.grads[: lay.param_numel].float().clone()
for name, e in lay.entries.items():
    if e.region != "param":
        continue
    sl = slice(e.offset, e.offset + e.numel)
    m = g["0a"][sl].abs().max().item()
    print(f"{name:28s} max {m:9.3e}  0a-0b {(g['0a'][sl]-g['0b'][sl]).abs().max().item():9.3e}  "
          f"1a-1b {(g['1a'][sl]-g['1b'][sl]).abs().max().item():9.3e}  1a-0a {(g['1a'][sl]-g['0a'][sl]).abs().max().item():9.3e}")
