"""Per-layer timing of the fp32 conv kernels (ResNet-18 CIFAR shapes, batch 128) against MIOpen fp32
(torch channels_last fp32 conv forward / input-grad / weight-grad on the same box): the library
baseline for the fp32 headline. One JSON line per layer; TFLOP/s of each pass against the 157 TF
fp32 peak (MI355X_MICROARCH.md, f32 MFMA = f32 VALU rate).

  python bench/conv_layers_f32.py              # all layers
  ONLY=wgrad python bench/conv_layers_f32.py   # one pass (profiling)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402

SHAPES = [(3, 64, 32, 3, 1, 1), (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (64, 128, 32, 1, 2, 0),
          (128, 128, 16, 3, 1, 1), (128, 256, 16, 3, 2, 1), (128, 256, 16, 1, 2, 0), (256, 256, 8, 3, 1, 1),
          (256, 512, 8, 3, 2, 1), (256, 512, 8, 1, 2, 0), (512, 512, 4, 3, 1, 1)]
# occurrences of each shape in one ResNet-18 step (fwd; dgrad skips the stem)
COUNT = [1, 4, 1, 1, 3, 1, 1, 3, 1, 1, 3]


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
    B = int(os.environ.get("B", "128"))
    only = os.environ.get("ONLY", "")
    miopen = os.environ.get("MIOPEN", "1") == "1" and not only
    tot = {"psx": 0.0, "miopen": 0.0}
    for (cin, cout, hw, k, s, p), cnt in zip(SHAPES, COUNT):
        x = torch.randn(B, cin, hw, hw, device="cuda")
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = operands_f32(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = nhwc(x, cp)
        y = torch.empty(B, oh, oh, cout, device="cuda")
        dy = torch.randn(B, oh, oh, cout, device="cuda")
        dx = torch.empty(B, hw, hw, cp, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
        n1 = K.conv2_workspace_bytes(B, oh, oh, cout, kg, True)
        n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd, True)
        ws = torch.empty(max(n1, n2, 4) // 4, device="cuda")
        flops = 2.0 * B * oh * oh * cout * cin * k * k
        r = {"shape": [cin, cout, hw, k, s], "gflop": round(flops / 1e9, 3)}
        if only in ("", "fwd"):
            r["fwd_us"] = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg))
        if cin != 3 and only in ("", "dgrad"):
            r["dgrad_us"] = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd))
        if only in ("", "wgrad"):
            spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg, True)
            part = torch.empty(spl * cout * kg, device="cuda")
            out = torch.empty(cout * cin * k * k, dtype=torch.float16, device="cuda")
            r["wgrad_splits"] = spl
            r["wgrad_us"] = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg))
            r["wreduce_us"] = t_us(lambda: K.wgrad_reduce(part, spl, cout, kg, cin, cp, k, 1.0, out.data_ptr(), True))
        if k == 3 and s == 1 and cin >= 64 and K.wino_ok(hw, hw, cin, cout) and not only:
            # Winograd F(4x4,3x3) (csrc/kernels/wino.hip): forward / data gradient per GEMM tile
            # config, and the per-step weight transforms (forward + flipped)
            u = torch.empty(36 * cout * cin, device="cuda")
            ud = torch.empty(36 * cout * cin, device="cuda")
            nv = max(K.wino_v_floats(B, hw, hw, cin), K.wino_v_floats(B, hw, hw, cout), K.wino_p_floats(B, hw, hw, cin, cout),
                     K.wino_p_floats(B, hw, hw, cout, cin))
            v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
            xw = x.permute(0, 2, 3, 1).contiguous()
            r["wino_wt_us"] = t_us(lambda: (K.wino_weights(w, u, cout, cin), K.wino_weights(w, ud, cout, cin, True)))
            for cfg in range(4):
                r[f"wino_fwd_c{cfg}_us"] = t_us(lambda: K.wino_conv(xw, u, y, None, stats, v1, v2, B, hw, hw, cin,
                                                                    cout, cfg=cfg))
                r[f"wino_dgrad_c{cfg}_us"] = t_us(lambda: K.wino_conv(dy, ud, dx, None, None, v2, v1, B, hw, hw, cout,
                                                                      cin, cfg=cfg))
            K.wino_conv(xw, u, y, None, stats, v1, v2, B, hw, hw, cin, cout)
            q = K.wino_wgrad_q(B, hw, hw, cin, cout)
            if q > 0:
                wpart = torch.empty(36 * q * cout * cin, device="cuda")
                gout = torch.empty(cout * cin * 9, dtype=torch.float16, device="cuda")
                r["wino_wgrad_q"] = q
                r["wino_wgrad_us"] = t_us(lambda: K.wino_wgrad(v1, dy, v2, wpart, gout, B, hw, hw, cin, cout))
        psx_us = sum(r.get(key, 0.0) for key in ("fwd_us", "dgrad_us", "wgrad_us", "wreduce_us"))
        tot["psx"] += cnt * psx_us
        if miopen:
            xt = x.contiguous(memory_format=torch.channels_last)
            wt = w.contiguous(memory_format=torch.channels_last)
            dyt = dy.permute(0, 3, 1, 2)  # NHWC storage = channels_last view
            r["miopen_fwd_us"] = t_us(lambda: F.conv2d(xt, wt, stride=s, padding=p))
            if cin != 3:
                r["miopen_dgrad_us"] = t_us(lambda: torch.ops.aten.convolution_backward(
                    dyt, xt, wt, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (True, False, False)))
            r["miopen_wgrad_us"] = t_us(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wt, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (False, True, False)))
            tot["miopen"] += cnt * sum(r.get(key, 0.0) for key in ("miopen_fwd_us", "miopen_dgrad_us", "miopen_wgrad_us"))
        for key in list(r):
            if key.endswith("_us"):
                r[key] = round(r[key], 2)
        for key in ("fwd", "dgrad", "wgrad"):
            if f"{key}_us" in r:
                r[f"{key}_tflops"] = round(flops / r[f"{key}_us"] / 1e6, 1)
        print(json.dumps(r), flush=True)
    print(json.dumps({"step_conv_us": {k: round(v, 1) for k, v in tot.items()},
                      "note": "sum over the 20 convs of one ResNet-18 step (fwd + dgrad + wgrad [+ reduce])"}))


if __name__ == "__main__":
    main()
