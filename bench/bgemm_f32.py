"""fp32 batched-GEMM throughput of the Winograd layers (the 36 per-point GEMMs of ResNet-18's
8x8x256 / 4x4x512 layers and ResNet-50's 3x3 stages at B=128): psx's conv_v2 mainloop (every
tile config) and torch.bmm (hipBLASLt / rocBLAS fp32) on the same operands. One JSON line per shape: microseconds and TFLOP/s.

  python bench/bgemm_f32.py
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


# (M = tiles, N = out channels, Kd = in channels); batch 36
SHAPES = [(512, 256, 256), (128, 512, 512), (2048, 128, 128), (6272, 128, 128), (25088, 64, 64),
          (2048, 256, 256), (512, 512, 512)]  # the last two: ResNet-50's 14x14 / 7x7 (partial tiles)


def main():
    torch.manual_seed(0)
    nb = 36
    for m, n, kd in SHAPES:
        a = torch.randn(nb, m, kd, device="cuda")
        b = torch.randn(n, nb, kd, device="cuda")
        p = torch.empty(nb, m, n, device="cuda")
        ref = torch.bmm(a, b.permute(1, 2, 0))
        fl = 2.0 * nb * m * n * kd
        r = {"m": m, "n": n, "kd": kd, "nb": nb}
        for cfg in range(4):
            try:
                K.bgemm_f32(a, b, p, m, n, kd, nb, cfg)
                torch.cuda.synchronize()
                err = ((p - ref).abs().max() / ref.abs().max()).item()
                us = t_us(lambda: K.bgemm_f32(a, b, p, m, n, kd, nb, cfg))
                r[f"cfg{cfg}"] = [round(us, 1), round(fl / us / 1e6, 1), f"{err:.1e}"]
            except Exception as e:  # noqa: BLE001
                r[f"cfg{cfg}"] = str(e)[:60]
        bt = b.permute(1, 2, 0).contiguous()
        us = t_us(lambda: torch.bmm(a, bt, out=p))
        r["torch_bmm"] = [round(us, 1), round(fl / us / 1e6, 1)]
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
