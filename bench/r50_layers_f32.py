"""Isolated per-layer timing of every ResNet-50 conv (ImageNet shape, batch 128, fp32) on the path
the engine plans for it: forward (+ BN statistics epilogue), data gradient, weight gradient
(+ split-K reduction), or the fused Winograd kernels where the engine uses them. One JSON line
per unique layer shape with its count per step, TFLOP/s against the measured 155 TF f32 MFMA
ceiling (profiles/r2s3_mfma_ceiling.jsonl), and a final line with the count-weighted sums —
compared against the in-step kernel times of a serial (PSX_TUNE wgrad_stream=0) step profile.

  python bench/r50_layers_f32.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from psx.utils.tune import tune_flag  # noqa: E402
from tests.test_fp32_gpu import nhwc, operands_f32  # noqa: E402

# (cin, cout, hw_in, k, stride, pad, count per step) — torchvision ResNet-50 v1.5 (stride in the 3x3)
SHAPES = [
    (3, 64, 224, 7, 2, 3, 1),
    (64, 64, 56, 1, 1, 0, 1), (64, 64, 56, 3, 1, 1, 3), (64, 256, 56, 1, 1, 0, 4), (256, 64, 56, 1, 1, 0, 2),
    (256, 128, 56, 1, 1, 0, 1), (128, 128, 56, 3, 2, 1, 1), (256, 512, 56, 1, 2, 0, 1),
    (128, 512, 28, 1, 1, 0, 4), (512, 128, 28, 1, 1, 0, 3), (128, 128, 28, 3, 1, 1, 3),
    (512, 256, 28, 1, 1, 0, 1), (256, 256, 28, 3, 2, 1, 1), (512, 1024, 28, 1, 2, 0, 1),
    (256, 1024, 14, 1, 1, 0, 6), (1024, 256, 14, 1, 1, 0, 5), (256, 256, 14, 3, 1, 1, 5),
    (1024, 512, 14, 1, 1, 0, 1), (512, 512, 14, 3, 2, 1, 1), (1024, 2048, 14, 1, 2, 0, 1),
    (512, 2048, 7, 1, 1, 0, 3), (2048, 512, 7, 1, 1, 0, 2), (512, 512, 7, 3, 1, 1, 2),
]
PEAK_TF = 155.0


def t_us(fn, iters=10, warm=2):
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
    torch.manual_seed(0)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "reduce": 0.0}
    for cin, cout, hw, k, s, p, cnt in SHAPES:
        if only and only != f"{cin}x{cout}x{hw}x{k}s{s}":
            continue
        x = torch.randn(B, cin, hw, hw, device="cuda")
        w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
        wf, wd, cp, kg, kgd = operands_f32(w)
        oh = (hw + 2 * p - k) // s + 1
        xh = nhwc(x, cp)
        del x
        y = torch.empty(B, oh, oh, cout, device="cuda")
        dy = torch.randn(B, oh, oh, cout, device="cuda")
        dx = torch.empty(B, hw, hw, cp, device="cuda") if cin != 3 else None
        stats = torch.zeros(K.STAT_SLOTS, 2, cout, device="cuda")
        n1 = K.conv2_workspace_bytes(B, oh, oh, cout, kg, True)
        n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd, True)
        ws = torch.empty(max(n1, n2, 4) // 4, device="cuda")
        fl = 2.0 * B * oh * oh * cout * cin * k * k
        r = {"shape": [cin, cout, hw, k, s], "count": cnt, "gflop": round(fl / 1e9, 2)}
        wino = k == 3 and s == 1 and hw <= 64 and K.wino_ok(hw, hw, cp, cout) and tune_flag("wino", True)
        if wino:
            u = torch.empty(40 * cout * cp, device="cuda")
            ud = torch.empty(40 * cout * cp, device="cuda")
            wc = w.contiguous()
            K.WinoWeightBatch([(wc, u, cout, cp, False, int(K.wino_fused_ok(B, hw, hw, cp, cout))),
                               (wc, ud, cout, cp, True, int(K.wino_fused_ok(B, hw, hw, cout, cp)))])()
            nv = max(K.wino_v_floats(B, hw, hw, cp), K.wino_v_floats(B, hw, hw, cout), K.wino_p_floats(B, hw, hw, cp, cout),
                     K.wino_p_floats(B, hw, hw, cout, cp))
            v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
            if K.wino_fused_ok(B, hw, hw, cp, cout):
                r["path"] = "wino_fused"
                r["fwd_us"] = t_us(lambda: K.wino_fused(xh, u, y, None, stats, None, B, hw, hw, cp, cout))
                r["dgrad_us"] = t_us(lambda: K.wino_fused(dy, ud, dx, None, None, None, B, hw, hw, cout, cp))
            else:
                r["path"] = "wino"
                r["fwd_us"] = t_us(lambda: K.wino_conv(xh, u, y, None, stats, v1, v2, B, hw, hw, cp, cout))
                r["dgrad_us"] = t_us(lambda: K.wino_conv(dy, ud, dx, None, None, v2, v1, B, hw, hw, cout, cp))
            q = K.wino_wgrad_fused_q(B, hw, hw, cp, cout)
            q3 = K.wino_wgrad_q(B, hw, hw, cp, cout)
            gout = torch.empty(cout * cin * 9, dtype=torch.float16, device="cuda")
            if q > 0 and hw >= 16:
                wpart = torch.empty(36 * q * cout * cp, device="cuda")
                r["wgrad_us"] = t_us(lambda: K.wino_wgrad_fused(xh, dy, wpart, gout, B, hw, hw, cp, cout))
                r["reduce_us"] = 0.0
            elif q3 > 0:  # three launches: dy transform, batched TN GEMM, output transform; V from the forward
                r["path"] += "+wino_wgrad"
                K.wino_conv(xh, u, y, None, stats, v1, v2, B, hw, hw, cp, cout)
                d = torch.empty(K.wino_v_floats(B, hw, hw, cout), device="cuda")
                wpart = torch.empty(36 * q3 * cout * cp, device="cuda")
                r["wgrad_us"] = t_us(lambda: K.wino_wgrad(v1, dy, d, wpart, gout, B, hw, hw, cp, cout))
                r["reduce_us"] = 0.0
                del d
            del v1, v2
        elif cin == 3 and k == 7 and K.stem_conv(xh, wf, y, stats, B, hw, hw, cin, cp, cout, kg, k=7):
            r["path"] = "stem7"  # csrc/kernels/stem.hip (the weight gradient: conv_wgrad2 -> stem7_wgrad)
            r["fwd_us"] = t_us(lambda: K.stem_conv(xh, wf, y, stats, B, hw, hw, cin, cp, cout, kg, k=7))
        else:
            r["path"] = "conv_v2"
            r["fwd_us"] = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, k, s, p, kg))
            if dx is not None:
                r["dgrad_us"] = t_us(lambda: K.conv_dgrad2(dy, wd, dx, None, ws, B, hw, hw, cp, cout, k, s, p, kgd))
        if "wgrad_us" not in r:
            spl = K.conv_wgrad2_splits(B, hw, hw, cp, cout, k, s, p, kg, True)
            part = torch.empty(spl * cout * kg, device="cuda")
            out = torch.empty(cout * cin * k * k, dtype=torch.float16, device="cuda")
            r["wgrad_splits"] = spl
            r["wgrad_us"] = t_us(lambda: K.conv_wgrad2(xh, dy, part, B, hw, hw, cp, cout, k, s, p, kg))
            r["reduce_us"] = t_us(lambda: K.wgrad_reduce(part, spl, cout, kg, cin, cp, k, 1.0, out.data_ptr(), True),
                                  iters=3)
        for key in ("fwd", "dgrad", "wgrad"):
            if f"{key}_us" in r:
                r[f"{key}_tf"] = round(fl / r[f"{key}_us"] / 1e6, 1)
                r[f"{key}_pct_peak"] = round(100 * fl / r[f"{key}_us"] / 1e6 / PEAK_TF, 1)
        for key in tot:
            tot[key] += cnt * r.get(f"{key}_us", 0.0)
        for key in list(r):
            if key.endswith("_us"):
                r[key] = round(r[key], 1)
        print(json.dumps(r), flush=True)
        del xh, y, dy, dx, ws
        torch.cuda.empty_cache()
    print(json.dumps({"step_conv_us": {k: round(v, 1) for k, v in tot.items()}, "total_us": round(sum(tot.values()), 1),
                      "note": "count-weighted sum over ResNet-50's convs, isolated launches, batch %d" % B}))


if __name__ == "__main__":
    main()
