"""Sweep the tap-reuse weight-gradient kernel (wgrad3: 3x3 stride-1 layers) over tile width x
split count per ResNet-18 layer (B=128), timing wgrad + the split reduction together (the split
count sets the partial-sum volume the reduction reads). Compares against wgrad2 (PSX_TUNE wg3=0).
One line per layer: planner picks and the best (BC, splits) found."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from psx.utils.tune import set_tune  # noqa: E402
from tests.test_kernels_gpu import to_nhwc  # noqa: E402
from conv_layers import SHAPES, t_us  # noqa: E402



def main():
    B = 128
    layers = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,4,7,10").split(",")]
    for li in layers:
        cin, cout, hw, k, s, p = SHAPES[li]
        kg = k * k * cin
        xh = to_nhwc(torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float(), cin)
        dy = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
        part = torch.empty(256 * cout * kg, device="cuda")
        out = torch.empty(cout * kg, dtype=torch.float16, device="cuda")

        def run():
            n = K.conv_wgrad2(xh, dy, part, B, hw, hw, cin, cout, k, s, p, kg)
            K.wgrad_reduce(part, n, cout, kg, cin, cin, k, 1.0, out.data_ptr(), True)

        def timed(**env):
            set_tune(**env)
            spl = K.conv_wgrad2_splits(B, hw, hw, cin, cout, k, s, p, kg)
            return spl, t_us(run, iters=20)

        if os.environ.get("SPLIT_ONLY"):
            for env in ({"wg3": 0}, {}):
                set_tune(**env)
                n = K.conv_wgrad2_splits(B, hw, hw, cin, cout, k, s, p, kg)
                tw = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cin, cout, k, s, p, kg), iters=20)
                tr = t_us(lambda: K.wgrad_reduce(part, n, cout, kg, cin, cin, k, 1.0, out.data_ptr(), True), iters=20)
                print(f"layer {li} {'wgrad2' if env else 'wgrad3'} splits={n} wgrad {tw:.1f} us reduce {tr:.1f} us "
                      f"partial {n * cout * kg * 4 / 1e6:.1f} MB", flush=True)
            continue
        s2, t2 = timed(wg3=0)
        s3, t3 = timed()
        best = (t3, 0, 0, s3)
        allr = []
        steps = B * hw * hw // 64
        for bc in (64, 128):
            if cout % bc:
                continue
            for ns in (3, 6):
                for sp in (3, 6, 10, 16, 24, 32, 43, 64, 86, 128, 171, 256):
                    if sp > steps:
                        continue
                    _, t = timed(wg_bc=bc, wg_ns=ns, wg_splits=sp)
                    best = min(best, (t, bc, ns, sp))
                    allr.append((round(t, 1), bc, ns, sp))
        set_tune()
        print(f"layer {li} {cin}->{cout} {hw}x{hw}: wgrad2 plan splits={s2} {t2:.1f} us | "
              f"wgrad3 plan splits={s3} {t3:.1f} us | best BC={best[1]} NS={best[2]} splits={best[3]} {best[0]:.1f} us",
              flush=True)
        print("   top:", sorted(allr)[:5], flush=True)


if __name__ == "__main__":
    main()
