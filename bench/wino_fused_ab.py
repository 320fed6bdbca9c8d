"""Same-process A/B of the Winograd forward on the ResNet-18 3x3 stride-1 layers (batch 128):
unfused (input transform + batched GEMM + output transform, PSX_WINO_FUSED=0) vs the GEMM with
the output transform fused into its epilogue (conv_v2.hip WOUT, PSX_WINO_FUSED=2). Forward with
BN statistics, the data gradient without fused sums. One JSON line per layer, microseconds.

  python bench/wino_fused_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402


def t_us(fn, iters=20, warm=3):
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

SHAPES = [(64, 32), (128, 16), (256, 8), (512, 4)]  # (channels, image side)


def main():
    B = int(os.environ.get("B", "128"))
    for c, hw in SHAPES:
        x = torch.randn(B, hw, hw, c, device="cuda")
        dy = torch.randn(B, hw, hw, c, device="cuda")
        w = torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5
        u = torch.empty(36 * c * c, device="cuda")
        ud = torch.empty(36 * c * c, device="cuda")
        K.wino_weights(w, u, c, c)
        K.wino_weights(w, ud, c, c, True)
        nv = K.wino_v_floats(B, hw, hw, c)
        v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
        y = torch.empty(B, hw, hw, c, device="cuda")
        dx = torch.empty(B, hw, hw, c, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
        r = {"layer": f"{hw}x{hw}x{c}", "B": B}
        outs = {}
        for mode in ("0", "2"):
            os.environ["PSX_WINO_FUSED"] = mode
            r[f"fwd_f{mode}_us"] = round(t_us(lambda: K.wino_conv(x, u, y, None, stats, v1, v2, B, hw, hw, c, c)), 2)
            r[f"dgrad_f{mode}_us"] = round(t_us(lambda: K.wino_conv(dy, ud, dx, None, None, v2, v1, B, hw, hw, c, c)), 2)
            K.wino_conv(x, u, y, None, None, v1, v2, B, hw, hw, c, c)
            torch.cuda.synchronize()
            outs[mode] = y.clone()
        os.environ["PSX_WINO_FUSED"] = "0"
        r["max_rel_diff"] = float((outs["2"] - outs["0"]).abs().max() / outs["0"].abs().max())
        # weight gradient: tile-range splits q of the batched TN GEMM (PSX_WINO_WQ)
        K.wino_conv(x, u, y, None, None, v1, v2, B, hw, hw, c, c)
        gout = torch.empty(c * c * 9, dtype=torch.float16, device="cuda")
        for q in (1, 2, 4, 8, 16, 32):
            T = B * (hw // 4) ** 2
            if T % (32 * q) or T // q < 32:
                continue
            os.environ["PSX_WINO_WQ"] = str(q)
            if K.wino_wgrad_q(B, hw, hw, c, c) != q:
                continue
            wpart = torch.empty(36 * q * c * c, device="cuda")
            r[f"wgrad_q{q}_us"] = round(t_us(lambda: K.wino_wgrad(v1, dy, v2, wpart, gout, B, hw, hw, c, c)), 2)
        os.environ.pop("PSX_WINO_WQ", None)
        r["wgrad_q_default"] = K.wino_wgrad_q(B, hw, hw, c, c)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
