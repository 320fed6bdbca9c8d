"""fp32 conv tile A/B (conv_v2.hip conv2_kernel): the planner's tiles against forced 128 x 128
(PSX_TUNE cv_bm / cv_bn, read per call) on ResNet-50's 1x1 layers and ResNet-18's strided layers,
batch 128, forward and data gradient; numerics of the forced tile against torch fp64. One JSON
line per layer: microseconds and TFLOP/s per tile.

  python bench/f32_tiles.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from psx.utils.tune import set_tune  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402

# (cin, cout, hw, k, stride, pad)
SHAPES = [(64, 64, 56, 1, 1, 0), (64, 256, 56, 1, 1, 0), (256, 64, 56, 1, 1, 0), (256, 128, 56, 1, 1, 0),
          (128, 512, 28, 1, 1, 0), (512, 128, 28, 1, 1, 0), (512, 256, 28, 1, 1, 0), (256, 1024, 14, 1, 1, 0),
          (1024, 256, 14, 1, 1, 0), (1024, 512, 14, 1, 1, 0), (512, 2048, 7, 1, 1, 0), (2048, 512, 7, 1, 1, 0),
          (256, 512, 8, 1, 2, 0), (128, 256, 16, 3, 2, 1)]
TILES = [None, (128, 128), (64, 128), (64, 64)]


def t_us(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / iters


def force(t):
    set_tune()
    if t:
        set_tune(cv_bm=t[0], cv_bn=t[1])


def main():
    B = int(os.environ.get("B", "128"))
    torch.manual_seed(0)
    for cin, cout, hw, k, s, p in SHAPES:
        x = torch.randn(B, cin, hw, hw, device="cuda")
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = operands_f32(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = nhwc(x, cp)
        y = torch.empty(B, oh, oh, cout, device="cuda")
        dy = torch.randn(B, oh, oh, cout, device="cuda")
        dx = torch.empty(B, hw, hw, cp, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
        n1 = K.conv2_workspace_bytes(B, oh, oh, cout, kg, True)
        n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd, True)
        ws = torch.empty(max(n1, n2, 4) // 4, device="cuda")
        fl = 2.0 * B * oh * oh * cout * cin * k * k
        r = {"shape": [cin, cout, hw, k, s]}
        yref = F.conv2d(x.double(), w.double(), stride=s, padding=p).permute(0, 2, 3, 1)
        for t in TILES:
            force(t)
            tag = "plan" if t is None else f"{t[0]}x{t[1]}"
            try:
                K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg)
                torch.cuda.synchronize()
                err = ((y.double() - yref).abs().max() / yref.abs().max()).item()
                us = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg))
                ud = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd))
                r[tag] = {"fwd": [round(us, 1), round(fl / us / 1e6, 1), f"{err:.1e}"],
                          "dgrad": [round(ud, 1), round(fl / ud / 1e6, 1)]}
            except Exception as e:  # noqa: BLE001
                r[tag] = str(e)[:80]
        force(None)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
