"""Run only the wgrad v2 kernel on chosen ResNet-18 (B=128) layers — a clean target for
`rocprofv3 --pmc` (one row per dispatch) and for A/B timing of wgrad variants.

  python bench/wgrad_probe.py [--layers 1,4,7,10] [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "bench"))
from conv_layers import SHAPES, t_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="1,4,7,10")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    B = a.batch
    for li in (int(x) for x in a.layers.split(",")):
        cin, cout, hw, k, s, p = SHAPES[li]
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
        w = torch.randn(cout, cin, k, k, device="cuda")
        wf, wd, cp, kg, kgd = make_operands(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = to_nhwc(x, cp)
        dy = torch.randn(B, oh, oh, cout, device="cuda").to(torch.bfloat16)
        spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg)
        part = torch.empty(spl * cout * kg, device="cuda")
        us = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg), iters=a.iters)
        gf = 2.0 * B * oh * oh * cout * cin * k * k / 1e9
        print(f"layer {li} {cin}->{cout} {hw}x{hw} k{k} s{s}: splits {spl}  {us:7.1f} us  "
              f"{gf / us * 1e3:6.1f} TFLOP/s  partial {spl * cout * kg * 4 / 1e6:.1f} MB", flush=True)


if __name__ == "__main__":
    main()
