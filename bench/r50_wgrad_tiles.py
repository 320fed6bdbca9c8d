"""Weight-gradient tile sweep on ResNet-50's 1x1 / strided layers (batch 128, bf16 and fp32):
conv_wgrad2 + its split reduction per tile (PSX_TUNE wg_br / wg_bc for bf16, wgf_br / wgf_bc for
fp32; "plan" = the cost-model choice). One JSON line per (dtype, shape): [kernel us, with reduce us,
splits] per tile.

  python bench/r50_wgrad_tiles.py
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
from bench.r50_tiles import SHAPES  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402


def main():
    B = int(os.environ.get("B", "128"))
    torch.manual_seed(0)
    for dt in ("bf16", "fp32"):
        f32 = dt == "fp32"
        pre = "wgf_" if f32 else "wg_"
        tiles = {"plan": ""}
        for br in (64, 128):
            for bc in (64, 128):
                tiles[f"{br}x{bc}"] = f"{pre}br={br},{pre}bc={bc}"
        for cin, cout, hw, k, s, p in SHAPES:
            if k == 3:
                continue  # the strided 3x3s: same kernel family, sweep the 1x1s
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
            dy = torch.randn(B, oh, oh, cout, device="cuda").to(adt)
            out = torch.empty(cout * cin * k * k, device="cuda")
            r = {"dtype": dt, "shape": [cin, cout, hw, k, s]}
            for name, tv in tiles.items():
                os.environ["PSX_TUNE"] = tv
                try:
                    spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg, f32)
                    part = torch.empty(spl * cout * kg, device="cuda")
                    kern = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg), iters=10)
                    full = t_us(lambda: (K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg),
                                         K.wgrad_reduce(part, spl, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False)),
                                iters=10)
                    r[name] = [round(kern, 1), round(full, 1), spl]
                    del part
                except Exception as e:  # noqa: BLE001
                    r[name] = str(e)[:50]
            os.environ.pop("PSX_TUNE", None)
            print(json.dumps(r), flush=True)
            del xh, dy


if __name__ == "__main__":
    main()
