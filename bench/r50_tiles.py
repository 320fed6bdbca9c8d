"""Conv tile sweep on ResNet-50's 1x1 and strided layers (batch 128, bf16 and fp32): psx conv_v2
forward (with BN slot sums) and data gradient (with the residual on 1x1 stride-1 layers, as the
engine runs conv1's) per tile plan (PSX_TUNE cv_bm / cv_bn; "plan" = the default plan_for choice).
One JSON line per (dtype, shape): us per tile.

  python bench/r50_tiles.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from bench.r50_1x1_bf16 import t_us  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402

# (cin, cout, hw, k, stride, pad)
SHAPES = [(64, 256, 56, 1, 1, 0), (256, 64, 56, 1, 1, 0), (64, 64, 56, 1, 1, 0), (256, 128, 56, 1, 1, 0),
          (256, 512, 56, 1, 2, 0), (128, 128, 56, 3, 2, 1), (128, 512, 28, 1, 1, 0), (512, 128, 28, 1, 1, 0),
          (512, 256, 28, 1, 1, 0), (512, 1024, 28, 1, 2, 0), (256, 256, 28, 3, 2, 1), (256, 1024, 14, 1, 1, 0),
          (1024, 256, 14, 1, 1, 0), (1024, 512, 14, 1, 1, 0), (1024, 2048, 14, 1, 2, 0), (512, 512, 14, 3, 2, 1),
          (512, 2048, 7, 1, 1, 0), (2048, 512, 7, 1, 1, 0)]
TILES = {"plan": "", "64x64": "cv_bm=64,cv_bn=64", "64x128": "cv_bm=64,cv_bn=128", "128x128": "cv_bm=128,cv_bn=128"}


def main():
    B = int(os.environ.get("B", "128"))
    torch.manual_seed(0)
    for dt in ("bf16", "fp32"):
        f32 = dt == "fp32"
        for cin, cout, hw, k, s, p in SHAPES:
            x = torch.randn(B, cin, hw, hw, device="cuda")
            w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
            if f32:
                wf, wd, cp, kg, kgd = operands_f32(w)
                xh = nhwc(x, cp)
                adt = torch.float32
            else:
                wf, wd, cp, kg, kgd = make_operands(w)
                xh = to_nhwc(x, cp)
                adt = torch.bfloat16
            del x
            oh = (hw + 2 * p - k) // s + 1
            y = torch.empty(B, oh, oh, cout, dtype=adt, device="cuda")
            dy = torch.randn(B, oh, oh, cout, device="cuda").to(adt)
            dx = torch.empty(B, hw, hw, cp, dtype=adt, device="cuda")
            res = torch.randn(B, hw, hw, cp, device="cuda").to(adt) if (k == 1 and s == 1) else None
            stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
            n1 = K.conv2_workspace_bytes(B, oh, oh, cout, kg, f32)
            n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd, f32)
            ws = torch.empty(max(n1, n2, 4) // 4 * 4, device="cuda")
            r = {"dtype": dt, "shape": [cin, cout, hw, k, s]}
            for name, tv in TILES.items():
                os.environ["PSX_TUNE"] = tv
                try:
                    fw = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg), iters=10)
                    dg = t_us(lambda: K.conv_dgrad2(dy, wd, dx, res, ws, B, hw, hw, cp, cout, k, s, p, kgd), iters=10)
                    r[name] = [round(fw, 1), round(dg, 1)]
                except Exception as e:  # noqa: BLE001
                    r[name] = str(e)[:50]
            os.environ.pop("PSX_TUNE", None)
            print(json.dumps(r), flush=True)
            del xh, y, dy, dx, res, ws


if __name__ == "__main__":
    main()
