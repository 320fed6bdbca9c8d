"""Run only conv v2 fwd / dgrad on chosen ResNet-18 layers (B=128): a clean rocprofv3 --pmc target."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402
from conv_layers import SHAPES, t_us  # noqa: E402


def main():
    B = 128
    layers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,7,10").split(",")]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ws = torch.empty(64 << 20, device="cuda")
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
        f = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg), iters=iters)
        d = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd), iters=iters) \
            if cin != 3 else float("nan")
        print(f"layer {li} {cin}->{cout} {hw} k{k}s{s}: fwd {f:6.1f} us  dgrad {d:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
