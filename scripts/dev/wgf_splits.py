"""fp32 weight-gradient split sweep of one layer in one process (PSX_WGF_SPLITS is read per call)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import psx  # noqa: E402,F401
sys.path.insert(0, os.path.join(ROOT, "bench"))
from conv_layers_f32 import t_us  # noqa: E402
from psx.ops import kernels as K  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402

B = 128
for cin, cout, hw in [(64, 64, 32), (128, 128, 16), (256, 256, 8), (512, 512, 4)]:
    x = torch.randn(B, cin, hw, hw, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda")
    wf, wd, cp, kg, kgd = operands_f32(w)
    xh = nhwc(x, cp)
    dy = torch.randn(B, hw, hw, cout, device="cuda")
    res = {}
    for sp in ["", "2", "4", "6", "8", "16", "22", "28", "42", "56", "84", "85", "86", "87", "88", "112", "128"]:
        os.environ["PSX_WGF_SPLITS"] = sp
        spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, 3, 1, 1, kg, True)
        part = torch.empty(spl * cout * kg, device="cuda")
        res[f"{sp or 'plan'}:{spl}"] = round(t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, 3, 1, 1, kg)), 1)
    print(json.dumps({"layer": [cin, cout, hw], "us": res}), flush=True)
