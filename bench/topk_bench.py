"""Top-k encode/decode timing (csrc/kernels/topk.hip) on ResNet-18/50-sized gradients.

  python bench/topk_bench.py [--n 11220132] [--ratio 0.01]
Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel import topk as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=11_220_132)
    ap.add_argument("--ratio", type=float, default=0.01)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", choices=["both", "fp32", "fp16"], default="both")
    a = ap.parse_args()
    dts = {"both": (torch.float32, torch.float16), "fp32": (torch.float32,), "fp16": (torch.float16,)}[a.dtype]
    for dt in dts:
        g = (torch.randn(a.n, device="cuda") * 1e-3).to(dt)
        c = T.TopKCodec(a.n, a.ratio, "cuda")
        for _ in range(3):
            c.encode(g)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            c.encode(g)
        torch.cuda.synchronize()
        enc = (time.perf_counter() - t0) / a.iters * 1e6
        dst = torch.zeros(a.n, device="cuda")
        t0 = time.perf_counter()
        for _ in range(a.iters):
            T.decode_add(c.payload, dst, 1.0, c.kcap)
        torch.cuda.synchronize()
        dec = (time.perf_counter() - t0) / a.iters * 1e6
        nc = int(c.ws[3])  # candidates of the last encode (topk.hip state word TK_NC)
        print(f"{str(dt):14s} n={a.n} k={c.k}: encode {enc:8.1f} us  decode {dec:6.1f} us  "
              f"payload {c.nbytes / 1e6:.2f} MB  candidates {nc}", flush=True)


if __name__ == "__main__":
    main()
