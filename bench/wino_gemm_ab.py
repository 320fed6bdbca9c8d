"""Same-process A/B of the three-launch fp32 Winograd conv (wino.hip: input transform + 36 batched
GEMMs on the conv_v2 mainloop + output transform) on ResNet-18's 8x8x256 / 4x4x512 layers and
ResNet-50's 14x14x256 / 7x7x512 (batch 128), forward with BN sums in microseconds, per PSX_TUNE
setting given on the command line ("" = defaults; round 6 measured the batched GEMMs' LDS ring
depth this way, profiles/r6_wino_gemm_stages_ab.jsonl). One JSON line per layer and setting; the
settings alternate per layer (same box, interleaved).

  python bench/wino_gemm_ab.py "" "some_key=1"
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402

SHAPES = [(256, 8), (512, 4), (256, 14), (512, 7)]


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
    settings = sys.argv[1:] or [""]
    B = int(os.environ.get("B", "128"))
    for c, hw in SHAPES:
        x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
        w = torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5
        u = torch.empty(36 * c * c, device="cuda")
        K.wino_weights(w, u, c, c)
        nv = max(K.wino_v_floats(B, hw, hw, c), K.wino_p_floats(B, hw, hw, c, c))
        v1, v2 = torch.empty(nv, device="cuda"), torch.empty(nv, device="cuda")
        y = torch.empty(B, hw, hw, c, device="cuda")
        stats = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
        ref = None
        for rep in range(2):
            for st in settings:
                os.environ["PSX_TUNE"] = st
                us = t_us(lambda: K.wino_conv(x, u, y, None, stats, v1, v2, B, hw, hw, c, c))
                if ref is None:
                    ref = y.clone()
                diff = float((y - ref).abs().max() / ref.abs().max())
                print(json.dumps({"layer": f"{hw}x{hw}x{c}", "B": B, "tune": st, "rep": rep, "fwd_us": round(us, 2),
                                  "max_rel_diff_vs_first": diff}), flush=True)
        os.environ.pop("PSX_TUNE", None)


if __name__ == "__main__":
    main()
