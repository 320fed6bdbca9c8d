"""Cost of the fused BN statistics in the conv epilogues (tap-reuse path, ResNet-18 B=128):
fwd with/without statistics, dgrad with/without the BN-backward sums (+ residual)."""
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
    for li in (1, 4, 7, 10):
        cin, cout, hw, k, s, p = SHAPES[li]
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = make_operands(w)
        x = to_nhwc(torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float(), cp)
        y = torch.empty(B, hw, hw, cout, dtype=torch.bfloat16, device="cuda")
        stats = torch.zeros(256, 2, cout, device="cuda")  # room for the A/B builds (<= 256 slot rows)
        dy = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
        dx = torch.empty(B, hw, hw, cp, dtype=torch.bfloat16, device="cuda")
        res = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
        o = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
        y1 = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
        saved = torch.ones(2, cp, device="cuda")
        part = torch.zeros(256, 3, cp, device="cuda")
        b2 = K.bwd_stats_desc(part, o, y1, saved)
        b3 = K.bwd_stats_desc(part, o, y1, saved, y1, saved)
        r = {
            "fwd+st": t_us(lambda: K.conv_fwd2(x, wf, y, stats, None, B, hw, hw, cp, cout, k, s, p, kg), iters=40),
            "fwd": t_us(lambda: K.conv_fwd2(x, wf, y, None, None, B, hw, hw, cp, cout, k, s, p, kg), iters=40),
            "dg": t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, None, B, hw, hw, cp, cout, k, s, p, kgd), iters=40),
            "dg+bst": t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, None, B, hw, hw, cp, cout, k, s, p, kgd, bst=b2),
                           iters=40),
            "dg+res+bst": t_us(lambda: K.conv_dgrad2(dy, wd, dx, res, None, B, hw, hw, cp, cout, k, s, p, kgd, bst=b2),
                               iters=40),
            "dg+res+bst3": t_us(lambda: K.conv_dgrad2(dy, wd, dx, res, None, B, hw, hw, cp, cout, k, s, p, kgd,
                                                      bst=b3), iters=40),
        }
        print(f"layer {li} {cin}->{cout} {hw}: " + "  ".join(f"{k_} {v:5.1f}" for k_, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
