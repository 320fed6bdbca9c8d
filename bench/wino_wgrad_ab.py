"""Same-process A/B of the fp32 Winograd weight gradient per ResNet-18 layer class (batch 128):
the three-launch path (wino.hip: dy transform -> D, batched TN GEMM over the forward's V, output
transform) vs the fused launch (wino_wgrad.hip: x and dy transformed in registers, no V / D) +
its output transform. Also the fused kernel alone (PSX_TUNE wino_wgf_q sweeps its tile ranges).
One JSON line per layer, microseconds.

  python bench/wino_wgrad_ab.py            # Q="8,16,32" sweeps q where it applies
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

from bench.wino_fused_ab import t_us  # noqa: E402

SHAPES = [(64, 32), (128, 16), (256, 8), (512, 4)]  # (channels, image side)


def main():
    B = int(os.environ.get("B", "128"))
    qs = [int(q) for q in os.environ.get("Q", "").split(",") if q]
    for c, hw in SHAPES:
        x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
        dy = torch.randn(B, hw, hw, c, device="cuda")
        g = torch.empty(c * c * 9, device="cuda", dtype=torch.float16)
        r = {"layer": f"{hw}x{hw}x{c}", "B": B}
        q3 = K.wino_wgrad_q(B, hw, hw, c, c)
        if q3:
            v = torch.empty(K.wino_v_floats(B, hw, hw, c), device="cuda")
            p = torch.empty(K.wino_v_floats(B, hw, hw, c), device="cuda")
            u = torch.empty(36 * c * c, device="cuda")
            K.wino_weights(torch.randn(c, c, 3, 3, device="cuda"), u, c, c)
            K.wino_conv(x, u, torch.empty_like(dy), None, None, v, p, B, hw, hw, c, c)
            d = torch.empty(K.wino_v_floats(B, hw, hw, c), device="cuda")
            wp = torch.empty(36 * q3 * c * c, device="cuda")
            r["three_launch_us"] = round(t_us(lambda: K.wino_wgrad(v, dy, d, wp, g, B, hw, hw, c, c)), 2)
        qf = K.wino_wgrad_fused_q(B, hw, hw, c, c)
        r["fused_q"] = qf
        part = torch.empty(36 * max([qf] + qs) * c * c, device="cuda")
        r["fused_us"] = round(t_us(lambda: K.wino_wgrad_fused(x, dy, part, g, B, hw, hw, c, c)), 2)
        aff = torch.stack([torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")]).contiguous()
        r["fused_aff_us"] = round(t_us(lambda: K.wino_wgrad_fused(x, dy, part, g, B, hw, hw, c, c, xaff=aff)), 2)
        r["wout_us"] = round(t_us(lambda: K.kernels().psx_wino_wout(K.ptr(part), K.ptr(g), 1, 1.0, c, c, qf,
                                                                     K.stream_ptr())), 2)
        for q in qs:
            set_tune(wino_wgf_q=q)
            if K.wino_wgrad_fused_q(B, hw, hw, c, c) == q:
                r[f"fused_q{q}_us"] = round(t_us(lambda: K.wino_wgrad_fused(x, dy, part, g, B, hw, hw, c, c)), 2)
            set_tune()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
