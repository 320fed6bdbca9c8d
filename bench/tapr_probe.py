"""Layer-1/4/7 conv fwd timing decomposition: tap reuse on/off, BN stats on/off, batch 128/256."""
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
    ws = torch.empty(64 << 20, device="cuda")
    for li in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,4,7,10").split(",")]:
        cin, cout, hw, k, s, p = SHAPES[li]
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = make_operands(w)
        for B in (128,):
            x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
            xh = to_nhwc(x, cp)
            y = torch.empty(B, hw, hw, cout, dtype=torch.bfloat16, device="cuda")
            stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
            dy = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
            dx = torch.empty(B, hw, hw, cp, dtype=torch.bfloat16, device="cuda")
            row = []
            for tapr in ("256", "128", "64", "0"):
                set_tune(cv_tapr="0" if tapr == "0" else "1", cv_tapr_bn=tapr)
                t = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg), iters=40)
                td = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd), iters=40)
                row.append(f"bn{tapr} fwd {t:5.1f} dgrad {td:5.1f}")
            fl = 2.0 * B * hw * hw * cout * cin * 9
            print(f"layer {li} B={B} ({fl / 1e9:.1f} GF): " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
