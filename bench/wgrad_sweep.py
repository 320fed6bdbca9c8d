"""Sweep wgrad v2 tile shape x split count per ResNet-18 layer (B=128) in one process, using the
PSX_TUNE wg_* experiment overrides read by psx_conv_wgrad2. Prints the planner's pick and the best."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from psx.utils.tune import set_tune  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402
from conv_layers import SHAPES, t_us  # noqa: E402


def main():
    B = 128
    layers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,5,7,8,10").split(",")]
    for li in layers:
        cin, cout, hw, k, s, p = SHAPES[li]
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
        w = torch.randn(cout, cin, k, k, device="cuda")
        wf, wd, cp, kg, kgd = make_operands(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = to_nhwc(x, cp)
        dy = torch.randn(B, oh, oh, cout, device="cuda").to(torch.bfloat16)
        part = torch.empty(64 * cout * kg, device="cuda")
        set_tune()
        spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg)
        base = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg), iters=20)
        res = []
        for br, bc in ((128, 128), (64, 128), (128, 64), (64, 64)):
            if kg % br or cout % bc:
                continue
            for sp in (1, 2, 4, 6, 8, 12, 16, 24, 28, 32, 48, 56, 64):
                set_tune(wg_br=br, wg_bc=bc, wg_splits=sp)
                if oh * oh * B // 64 < sp:
                    continue
                us = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg), iters=20)
                res.append((us, br, bc, sp))
        res.sort()
        print(f"layer {li} {cin}->{cout} {hw} k{k}s{s}: planner splits={spl} {base:.1f} us | best "
              + "  ".join(f"{br}x{bc}/s{sp}:{us:.1f}" for us, br, bc, sp in res[:4]), flush=True)
    set_tune()


if __name__ == "__main__":
    main()
