"""Same-process A/B of the fp32 Winograd conv on ResNet-18's 32x32x64 / 16x16x128 layers (batch
128): the three-launch path (wino.hip: input transform + 36 batched GEMMs + output transform) vs
the single fused launch (wino_fused.hip), forward with BN statistics (+ V side output, as the
engine runs it for the weight gradient) and the data gradient with the consumer BN's sums.
One JSON line per layer, microseconds.

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


SHAPES = [(64, 32), (128, 16)]  # (channels, image side)


def main():
    B = int(os.environ.get("B", "128"))
    for c, hw in SHAPES:
        x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
        dy = torch.randn(B, hw, hw, c, device="cuda")
        w = torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5
        u, ud = (torch.empty(36 * c * c, device="cuda") for _ in range(2))
        uf, ufd = (torch.empty(40 * c * c, device="cuda") for _ in range(2))
        K.WinoWeightBatch([(w, u, c, c, False, 0), (w, ud, c, c, True, 0), (w, uf, c, c, False, 1),
                           (w, ufd, c, c, True, 1)])()
        nv = max(K.wino_v_floats(B, hw, hw, c), K.wino_p_floats(B, hw, hw, c, c))
        v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
        y, y2 = torch.empty(B, hw, hw, c, device="cuda"), torch.empty(B, hw, hw, c, device="cuda")
        dx = torch.empty(B, hw, hw, c, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
        o, y1 = torch.randn(B, hw, hw, c, device="cuda"), torch.randn(B, hw, hw, c, device="cuda")
        saved = torch.stack([torch.randn(c, device="cuda"), torch.rand(c, device="cuda") + 0.5])
        part = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
        bst = K.bwd_stats_desc(part, o, y1, saved, mask_store=True)
        r = {"layer": f"{hw}x{hw}x{c}", "B": B}
        r["fwd_split_us"] = round(t_us(lambda: K.wino_conv(x, u, y, None, stats, v1, v2, B, hw, hw, c, c)), 2)
        r["fwd_fused_us"] = round(t_us(lambda: K.wino_fused(x, uf, y2, None, stats, None, B, hw, hw, c, c)), 2)
        r["fwd_fused_v_us"] = round(t_us(lambda: K.wino_fused(x, uf, y2, None, stats, v1, B, hw, hw, c, c)), 2)
        r["dgrad_split_us"] = round(t_us(lambda: K.wino_conv(dy, ud, dx, None, None, v2, v1, B, hw, hw, c, c,
                                                             bst=bst)), 2)
        r["dgrad_fused_us"] = round(t_us(lambda: K.wino_fused(dy, ufd, dx, None, None, None, B, hw, hw, c, c,
                                                              bst=bst)), 2)
        K.wino_conv(x, u, y, None, None, v1, v2, B, hw, hw, c, c)
        K.wino_fused(x, uf, y2, None, None, None, B, hw, hw, c, c)
        torch.cuda.synchronize()
        r["max_rel_diff"] = float((y2 - y).abs().max() / y.abs().max())
        gf = 2.0 * 36 * B * (hw // 4) ** 2 * c * c / 1e3  # GEMM MFLOP -> TF/s at us
        r["fused_fwd_tflops"] = round(gf / r["fwd_fused_us"] / 1e3, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
