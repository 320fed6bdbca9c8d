"""Per-layer conv kernel timing (ResNet-18 CIFAR shapes, batch 128): fwd / dgrad / wgrad (+ reduce)
and MIOpen (torch channels_last bf16) for reference. Prints one JSON line per layer."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402

SHAPES = [(3, 64, 32, 3, 1, 1), (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (64, 128, 32, 1, 2, 0),
          (128, 128, 16, 3, 1, 1), (128, 256, 16, 3, 2, 1), (128, 256, 16, 1, 2, 0), (256, 256, 8, 3, 1, 1),
          (256, 512, 8, 3, 2, 1), (256, 512, 8, 1, 2, 0), (512, 512, 4, 3, 1, 1)]


def t_us(fn, iters=30, warm=5):
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
    B = int(os.environ.get("B", "128"))
    for cin, cout, hw, k, s, p in SHAPES:
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
        w = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16).float()
        wf, wd, cp, kg, kgd = make_operands(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = to_nhwc(x, cp)
        y = torch.empty(B, oh, oh, cout, dtype=torch.bfloat16, device="cuda")
        dy = torch.randn(B, oh, oh, cout, device="cuda").to(torch.bfloat16)
        dx = torch.empty(B, hw, hw, cp, dtype=torch.bfloat16, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
        n1 = K.conv2_workspace_bytes(B, oh, oh, cout, kg)
        n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd)
        ws = torch.empty(max(n1, n2, 4) // 4, device="cuda")
        flops = 2.0 * B * oh * oh * cout * cin * k * k
        r = {"shape": [cin, cout, hw, k, s], "gflop": round(flops / 1e9, 3)}
        r["fwd_v2_us"] = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg))
        if cin != 3:
            r["dgrad_v2_us"] = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd))
            # as the step runs it: the consumer BN's backward sums in the epilogue + the masked store
            o = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
            y1 = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
            saved = torch.stack([torch.randn(cp, device="cuda"), torch.rand(cp, device="cuda") + 0.5]).contiguous()
            part = torch.zeros(K.STAT_SLOTS, 2, cp, device="cuda")
            bst = K.bwd_stats_desc(part, o, y1, saved, mask_store=True)
            r["dgrad_bst_v2_us"] = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd,
                                                             bst=bst))
        out16 = torch.empty(cout * cin * k * k, dtype=torch.float16, device="cuda")
        spl2 = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg)
        part2 = torch.empty(spl2 * cout * kg, device="cuda")

        def wg2():
            K.conv_wgrad2(xh, dy, part2, B, hw, hw, cp, cout, k, s, p, kg)
            K.wgrad_reduce(part2, spl2, cout, kg, cin, cp, k, 1.0, out16.data_ptr(), True)

        r["wgrad_v2_us"] = t_us(wg2)
        r["wgrad_v2_splits"] = spl2
        r["wgrad_v2_kernel_us"] = t_us(lambda: K.conv_wgrad2(xh, dy, part2, B, hw, hw, cp, cout, k, s, p, kg))
        r["wgrad_reduce_us"] = t_us(
            lambda: K.wgrad_reduce(part2, spl2, cout, kg, cin, cp, k, 1.0, out16.data_ptr(), True))
        xt = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r["miopen_fwd_us"] = t_us(lambda: F.conv2d(xt, wt, stride=s, padding=p))
        for key in list(r):
            if key.endswith("_us"):
                r[key] = round(r[key], 2)
        r["fwd_v2_tflops"] = round(flops / r["fwd_v2_us"] / 1e6, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
