"""Sweep conv v2 fwd / dgrad tile shape x split-K per ResNet-18 layer (B=128) in one process,
using the PSX_TUNE cv_* experiment overrides read by plan_for (csrc/kernels/conv_v2.hip)."""
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



def clear():
    set_tune()


def main():
    B = 128
    layers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3,4,5,6,7,8,9,10").split(",")]
    ws = torch.empty(64 << 20, device="cuda")  # 256 MB scratch covers every split plan
    for li in layers:
        cin, cout, hw, k, s, p = SHAPES[li]
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = make_operands(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = to_nhwc(x, cp)
        y = torch.empty(B, oh, oh, cout, dtype=torch.bfloat16, device="cuda")
        dy = torch.randn(B, oh, oh, cout, device="cuda").to(torch.bfloat16)
        dx = torch.empty(B, hw, hw, cp, dtype=torch.bfloat16, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
        ops = {"fwd": lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg)}
        if cin != 3:
            ops["dgrad"] = lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd)
        for name, fn in ops.items():
            clear()
            base = t_us(fn, iters=20)
            res = []
            for bm, bn, wgm in ((128, 128, 2), (64, 128, 2), (64, 64, 2), (64, 256, 1), (64, 128, 1), (128, 256, 2)):
                for sp in (1, 2, 3, 4, 6, 8):
                    set_tune(cv_bm=bm, cv_bn=bn, cv_splits=sp, cv_wgm=wgm)
                    try:
                        res.append((t_us(fn, iters=20), bm, bn, sp, wgm))
                    except RuntimeError:
                        pass
            res.sort()
            print(f"layer {li} {name:5s} {cin}->{cout} {hw} k{k}s{s}: planner {base:.1f} us | best "
                  + "  ".join(f"{bm}x{bn}w{wgm}/s{sp}:{us:.1f}" for us, bm, bn, sp, wgm in res[:4]), flush=True)
    clear()


if __name__ == "__main__":
    main()
