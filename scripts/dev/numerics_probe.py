"""Per-tensor gradient error of one fp32 ResNet-18 engine step vs float64 autograd under PSX_TUNE
variants (diagnostic for test_fp32_gpu.py::test_engine_step_f32_per_tensor_damped): prints, per
variant, the median / worst relative error over all tensors and over layer4's."""
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import psx  # noqa: E402,F401
from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import ResNet18  # noqa: E402
from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"
torch.manual_seed(5)
B = 32
model = ResNet18(100)
with torch.no_grad():
    for name, m in model.named_modules():
        if name.endswith("bn2") or name.endswith("shortcut.1"):
            m.weight.fill_(0.2)
layout = ParamLayout.from_module(model)
arena0, _ = layout.pack(model)
arena0 = arena0.to(DEV)
x = torch.randn(B, 3, 32, 32, device=DEV)
y = torch.randint(0, 100, (B,), device=DEV)
ref = copy.deepcopy(model).to(DEV).double()
ref.train()
F.cross_entropy(ref(x.double()), y).backward()
for variant in sys.argv[1:] or [""]:
    det = "nodet" not in variant
    os.environ["PSX_TUNE"] = variant.replace("nodet", "").strip(",")
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32, dtype=torch.float32, deterministic=det)
    a = arena0.clone()
    eng.unpack(a)
    K.nchw_to_nhwc(x, eng.x0, B, 3, 32, 32, eng.x0.shape[-1])
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(a, train=True)
    eng.head(a, backward=True)
    eng.backward(a)
    torch.cuda.synchronize()
    errs = {}
    for name, p in ref.named_parameters():
        g = layout.grad_view(eng.grads, name).double()
        errs[name] = ((g - p.grad).norm() / p.grad.norm().clamp_min(1e-30)).item()
    v = sorted(errs.values())
    l4 = sorted(e for n, e in errs.items() if n.startswith("layer4"))
    worst = max(errs, key=errs.get)
    print(json.dumps({"variant": variant or "default", "median": f"{v[len(v) // 2]:.2e}", "worst": f"{v[-1]:.2e}",
                      "worst_tensor": worst, "layer4_median": f"{l4[len(l4) // 2]:.2e}",
                      "conv1.weight": f"{errs['conv1.weight']:.2e}",
                      "layer4.1.conv2.weight": f"{errs['layer4.1.conv2.weight']:.2e}"}), flush=True)
    K.set_deterministic(None)
