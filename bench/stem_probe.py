"""The CIFAR stem conv (3 -> 64, 3x3, 32x32, batch 128) in isolation: the planner's tile and
forced tiles (PSX_TUNE cv_bm / cv_bn / cv_wgm, read per call) on the gathered 4-channel
operand, against the same GEMM as a 1x1 conv over a pre-built 32-channel im2col operand, and
the output-store floor (a 128 x 32 x 32 x 64 tensor copy). One JSON line per variant.

  python bench/stem_probe.py
  BF16=1 python bench/stem_probe.py   # bf16 operands: conv_v2 tiles and the direct kernel only
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


def force(t):
    set_tune()
    if t:
        set_tune(cv_bm=t[0], cv_bn=t[1], cv_wgm=t[2])


def main():
    B, hw, cout = int(os.environ.get("B", "128")), 32, 64
    dt = torch.bfloat16 if os.environ.get("BF16") == "1" else torch.float32
    torch.manual_seed(0)
    x = torch.randn(B, 3, hw, hw, device="cuda")
    w = torch.randn(cout, 3, 3, 3, device="cuda") / 27 ** 0.5
    if dt == torch.bfloat16:  # BF16=1: the bf16 operands (8-channel chunks)
        from tests.test_kernels_gpu import make_operands, to_nhwc
        wf, _, cp, kg, _ = make_operands(w)
        xh = to_nhwc(x, cp)
    else:
        wf, _, cp, kg, _ = operands_f32(w)
        xh = nhwc(x, cp)
    y = torch.empty(B, hw, hw, cout, device="cuda", dtype=dt)
    stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
    ws = torch.empty(max(4, K.conv2_workspace_bytes(B, hw, hw, cout, kg, True)) // 4, device="cuda")
    for t in [None, (64, 128, 2), (64, 64, 2), (64, 256, 1), (64, 128, 1)]:
        force(t)
        try:
            us = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, 3, 1, 1, kg))
            print(json.dumps({"variant": "gather4", "tile": t or "plan", "us": round(us, 1)}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": "gather4", "tile": t, "err": str(e)[:80]}), flush=True)
    force(None)
    us = t_us(lambda: K.stem_conv(xh, wf, y, stats, B, hw, hw, 3, cp, cout, kg))
    print(json.dumps({"variant": "direct (stem.hip)", "us": round(us, 1)}), flush=True)
    us = t_us(lambda: K.stem_conv(xh, wf, y, None, B, hw, hw, 3, cp, cout, kg))
    print(json.dumps({"variant": "direct, no statistics", "us": round(us, 1)}), flush=True)
    if dt == torch.bfloat16:
        return
    # the same GEMM as a 1x1 conv over an im2col operand [B][32][32][32] (27 taps x 3 ch + pad)
    xc = torch.randn(B, hw, hw, 32, device="cuda")
    w1 = torch.randn(cout, 32, 1, 1, device="cuda")
    wf1, _, cp1, kg1, _ = operands_f32(w1)
    for t in [None, (64, 128, 2), (64, 64, 2), (64, 256, 1)]:
        force(t)
        try:
            us = t_us(lambda: K.conv_fwd2(xc, wf1, y, stats, ws, B, hw, hw, cp1, cout, 1, 1, 0, kg1))
            print(json.dumps({"variant": "im2col32_1x1", "tile": t or "plan", "us": round(us, 1)}), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"variant": "im2col32_1x1", "tile": t, "err": str(e)[:80]}), flush=True)
    force(None)
    y2 = torch.empty_like(y)
    print(json.dumps({"variant": "copy_floor", "us": round(t_us(lambda: y2.copy_(y)), 1),
                      "bytes_each_way": y.numel() * 4}), flush=True)
    print(json.dumps({"variant": "fill_floor", "us": round(t_us(lambda: y2.fill_(1.0)), 1)}), flush=True)


if __name__ == "__main__":
    main()
