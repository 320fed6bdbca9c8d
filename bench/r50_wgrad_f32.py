"""fp32 weight-gradient timing on ResNet-50's layers (ImageNet shape, batch 128): the planner's
wgrad2f / wgrad3f choice and forced tiles (PSX_TUNE wgf_br / wgf_bc, read per call), mainloop and
split-K reduction separately, TFLOP/s against the 157 TF fp32 MFMA peak. One JSON line per layer.

  python bench/r50_wgrad_f32.py            # all layers
  ONE=1 python bench/r50_wgrad_f32.py      # the 56x56 256->64 1x1 layer only, 5 launches (PMC runs)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from psx.utils.tune import set_tune  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402

# (cin, cout, hw, k, stride, pad): the 1x1 reduce / expand layers and the 3x3 layers of each stage
SHAPES = [(256, 64, 56, 1, 1, 0), (64, 256, 56, 1, 1, 0), (64, 64, 56, 1, 1, 0), (64, 64, 56, 3, 1, 1),
          (512, 128, 28, 1, 1, 0), (128, 512, 28, 1, 1, 0), (128, 128, 28, 3, 1, 1), (1024, 256, 14, 1, 1, 0),
          (256, 1024, 14, 1, 1, 0), (256, 256, 14, 3, 1, 1), (2048, 512, 7, 1, 1, 0), (512, 2048, 7, 1, 1, 0),
          (512, 512, 7, 3, 1, 1)]
TILES = [None, (128, 128), (128, 64), (64, 128), (64, 64)]


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
    set_tune(**({"wgf_br": t[0], "wgf_bc": t[1]} if t else {}))


def main():
    B = int(os.environ.get("B", "128"))
    one = os.environ.get("ONE") == "1"
    torch.manual_seed(0)
    for cin, cout, hw, k, s, p in SHAPES[:1] if one else SHAPES:
        x = torch.randn(B, cin, hw, hw, device="cuda")
        w = torch.randn(cout, cin, k, k, device="cuda")
        _, _, cp, kg, _ = operands_f32(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = nhwc(x, cp)
        dy = torch.randn(B, oh, oh, cout, device="cuda")
        fl = 2.0 * B * oh * oh * cout * cin * k * k
        r = {"shape": [cin, cout, hw, k, s]}
        ref = None
        for t in [None] if one else TILES:
            force(t)
            tag = "plan" if t is None else f"{t[0]}x{t[1]}"
            try:
                spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg, True)
                part = torch.empty(spl * cout * kg, device="cuda")
                out = torch.empty(cout * cin * k * k, device="cuda")
                if one:
                    for _ in range(5):
                        K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg)
                    torch.cuda.synchronize()
                    continue
                K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg)
                K.wgrad_reduce(part, spl, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False)
                torch.cuda.synchronize()
                if ref is None:
                    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, k, k), dy.double().permute(0, 3, 1, 2),
                                                      stride=s, padding=p).reshape(-1)
                err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
                us = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg))
                ur = t_us(lambda: K.wgrad_reduce(part, spl, cout, kg, cin, cp, k, 1.0, out.data_ptr(), False), iters=3)
                r[tag] = [spl, round(us, 1), round(ur, 1), round(fl / us / 1e6, 1), f"{err:.1e}"]
            except Exception as e:  # noqa: BLE001
                r[tag] = str(e)[:80]
        force(None)
        if not one:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
