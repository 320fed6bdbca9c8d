"""ResNet-50 stem max-pool (3x3 / stride 2 / pad 1, 112x112x64, batch 128) forward and backward
time, fp32 and bf16, against the bytes each pass must move. One JSON line per dtype.

  python bench/pool_probe.py
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


def main():
    B, H, C = int(os.environ.get("B", "128")), 112, 64
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(B, H, H, C, device="cuda").to(dt)
        y = torch.empty(B, H // 2, H // 2, C, device="cuda", dtype=dt)
        arg = torch.empty(B, H // 2, H // 2, C, device="cuda", dtype=torch.uint8)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        f = t_us(lambda: K.maxpool3s2_fwd(x, y, arg))
        b = t_us(lambda: K.maxpool3s2_bwd(dy, arg, dx))
        es = x.element_size()
        fb = x.numel() * es + y.numel() * (es + 1)
        print(json.dumps({"dtype": str(dt), "fwd_us": round(f, 1), "bwd_us": round(b, 1),
                          "fwd_TBps": round(fb / f / 1e6, 2), "bwd_TBps": round(fb / b / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
