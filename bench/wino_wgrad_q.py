"""Winograd weight-gradient split sweep (tile ranges q per batch, PSX_TUNE wino_wq) on ResNet-18's
stride-1 3x3 layers at batch 128: dy transform + batched TN GEMM + inverse transform to the
fp16 wire, microseconds. One JSON line per layer.

  python bench/wino_wgrad_q.py
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


def main():
    B = int(os.environ.get("B", "128"))
    for c, hw in [(64, 32), (128, 16), (256, 8), (512, 4)]:
        x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
        dy = torch.randn(B, hw, hw, c, device="cuda")
        w = torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5
        u = torch.empty(36 * c * c, device="cuda")
        K.wino_weights(w, u, c, c)
        nv = K.wino_v_floats(B, hw, hw, c)
        v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
        K.wino_conv(x, u, torch.empty(B, hw, hw, c, device="cuda"), None, None, v1, v2, B, hw, hw, c, c)
        gout = torch.empty(c * c * 9, dtype=torch.float16, device="cuda")
        r = {"layer": f"{hw}x{hw}x{c}", "B": B, "q_default": K.wino_wgrad_q(B, hw, hw, c, c)}
        T = B * (hw // 4) ** 2
        for q in (1, 2, 4, 8, 16, 32, 64):
            if T % (32 * q) or T // q < 32:
                continue
            set_tune(wino_wq=q)
            if K.wino_wgrad_q(B, hw, hw, c, c) != q:
                continue
            wpart = torch.empty(36 * q * c * c, device="cuda")
            r[f"q{q}_us"] = round(t_us(lambda: K.wino_wgrad(v1, dy, v2, wpart, gout, B, hw, hw, c, c)), 2)
        set_tune()
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
