"""Sweep of the fp32 tap-reuse weight gradient (wgrad3f_kernel) on the ResNet-18 3x3 stride-1
layers at batch 128: output-channel tile (PSX_TUNE wg_bc) x split count (wgf_splits), time of the
kernel + its split-K reduction, against the planner's choice and the wgrad2f path (wg3=0).
One JSON line per layer. The knobs are read per launch, so one process sweeps them all.

  python bench/wgrad3f_sweep.py
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

LAYERS = [(64, 32), (128, 16), (256, 8), (512, 4)]  # (channels, hw)


def env(**kv):
    set_tune(**kv)


def main():
    B = 128
    for c, hw in LAYERS:
        kg = 9 * c
        x = torch.randn(B, hw, hw, c, device="cuda")
        dy = torch.randn(B, hw, hw, c, device="cuda")
        out = torch.empty(c * c * 9, dtype=torch.float16, device="cuda")
        flops = 2.0 * B * hw * hw * c * c * 9

        def run():
            spl = K.conv_wgrad2_splits(B, hw, hw, c, c, 3, 1, 1, kg, True)
            part = torch.empty(spl * c * kg, device="cuda")
            tw = t_us(lambda: K.conv_wgrad2(x, dy, part, B, hw, hw, c, c, 3, 1, 1, kg))
            tr = t_us(lambda: K.wgrad_reduce(part, spl, c, kg, c, c, 3, 1.0, out.data_ptr(), True))
            return {"splits": spl, "wgrad_us": round(tw, 2), "reduce_us": round(tr, 2),
                    "tflops": round(flops / tw / 1e6, 1)}

        r = {"layer": [c, hw], "gflop": round(flops / 1e9, 3)}
        env(wg3=0)
        r["wgrad2f"] = run()
        env()
        r["plan"] = run()
        sweep = []
        steps = B * hw * hw // 32
        for bc in (64, 128):
            for spl in (8, 16, 32, 48, 64, 96, 128, 192, 256, 384, 512):
                if spl > steps or c % bc:
                    continue
                env(wg_bc=bc, wgf_splits=spl)
                sweep.append(dict(bc=bc, **run()))
        env()
        best = min(sweep, key=lambda d: d["wgrad_us"] + d["reduce_us"])
        r["best"] = best
        r["sweep"] = sweep
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
