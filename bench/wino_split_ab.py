"""Winograd forward / data gradient (wino.hip psx_wino_conv: input transform, 36 batched GEMMs,
output transform) per reduction split s2 of the GEMMs (PSX_TUNE wino_s2): the 3-launch layers of
ResNet-18 (8x8x256, 4x4x512) and ResNet-50 (14x14x256, 7x7x512) at batch 128. One JSON line per
layer: microseconds per s2.

  python bench/wino_split_ab.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from bench.bgemm_f32 import t_us  # noqa: E402

SHAPES = [(8, 256), (4, 512), (14, 256), (7, 512)]  # (h = w, channels in = out)


def main():
    torch.manual_seed(0)
    B = int(os.environ.get("B", "128"))
    for hw, c in SHAPES:
        x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
        w = torch.randn(c, c, 3, 3, device="cuda") * (2.0 / (9 * c)) ** 0.5
        u = torch.empty(36 * c * c, device="cuda")
        ud = torch.empty(36 * c * c, device="cuda")
        K.wino_weights(w, u, c, c)
        K.wino_weights(w, ud, c, c, True)
        y = torch.empty(B, hw, hw, c, device="cuda")
        dx = torch.empty_like(y)
        stats = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
        r = {"hw": hw, "c": c, "B": B}
        ref = None
        for s2 in (1, 2, 4):
            os.environ["PSX_TUNE"] = f"wino_s2={s2}"
            n = max(K.wino_v_floats(B, hw, hw, c), K.wino_p_floats(B, hw, hw, c, c))
            v, p = torch.empty(n, device="cuda"), torch.empty(n, device="cuda")
            K.wino_conv(x, u, y, None, stats, v, p, B, hw, hw, c, c)
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            err = ((y - ref).abs().max() / ref.abs().max()).item()
            fw = t_us(lambda: K.wino_conv(x, u, y, None, stats, v, p, B, hw, hw, c, c))
            dg = t_us(lambda: K.wino_conv(x, ud, dx, None, None, v, p, B, hw, hw, c, c))
            r[f"s2_{s2}"] = {"fwd_us": round(fw, 1), "dgrad_us": round(dg, 1), "rel_vs_s2_1": f"{err:.1e}"}
        os.environ.pop("PSX_TUNE", None)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
