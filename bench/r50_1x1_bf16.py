"""ResNet-50's 1x1 convolutions in bf16 (batch 128): psx's conv_v2 forward (with the BN slot sums)
and data gradient (with the residual, as the block's conv1 runs it) against the same GEMMs on
torch.mm (hipBLASLt) and their HBM byte floor. One JSON line per shape: us, TB/s of the psx launch.

  python bench/r50_1x1_bf16.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402
from tests.test_kernels_gpu import make_operands, to_nhwc  # noqa: E402

# (cin, cout, hw) stride 1
SHAPES = [(64, 256, 56), (256, 64, 56), (128, 512, 28), (512, 128, 28), (256, 1024, 14), (1024, 256, 14),
          (512, 2048, 7), (2048, 512, 7)]


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
    torch.manual_seed(0)
    only = os.environ.get("ONLY", "")  # "cinxcoutxhw": that layer only (profiling)
    for cin, cout, hw in SHAPES:
        if only and only != f"{cin}x{cout}x{hw}":
            continue
        npix = B * hw * hw
        x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).float()
        w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16).float()
        wf, wd, cp, kg, kgd = make_operands(w)
        xh = to_nhwc(x, cp)
        y = torch.empty(B, hw, hw, cout, dtype=torch.bfloat16, device="cuda")
        dy = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
        dx = torch.empty(B, hw, hw, cp, dtype=torch.bfloat16, device="cuda")
        res = torch.randn(B, hw, hw, cp, device="cuda").to(torch.bfloat16)
        stats = torch.zeros(64, 2, cout, device="cuda")  # >= any slot count a variant build uses
        stats_det = torch.zeros(K.STAT_SLOTS * K.det_slot_scale(), 2, cout, device="cuda")
        n1 = K.conv2_workspace_bytes(B, hw, hw, cout, kg)
        n2 = K.conv2_workspace_bytes(B, hw, hw, cp, kgd)
        ws = torch.empty(max(n1, n2, 4) // 4, device="cuda")
        r = {"cin": cin, "cout": cout, "hw": hw}
        fwd = t_us(lambda: K.conv_fwd2(xh, wf, y, stats, ws, B, hw, hw, cp, cout, 1, 1, 0, kg))
        fwd_ns = t_us(lambda: K.conv_fwd2(xh, wf, y, None, ws, B, hw, hw, cp, cout, 1, 1, 0, kg))
        K.set_deterministic(True)
        fwd_det = t_us(lambda: K.conv_fwd2(xh, wf, y, stats_det, ws, B, hw, hw, cp, cout, 1, 1, 0, kg))
        K.set_deterministic(False)
        dg = t_us(lambda: K.conv_dgrad2(dy, wd, dx, res, ws, B, hw, hw, cp, cout, 1, 1, 0, kgd))
        a2 = xh.view(npix, cp)
        wm = wf.view(cout, -1)[:, :cp].contiguous().t().contiguous()  # [cin][cout]
        yo = torch.empty(npix, cout, dtype=torch.bfloat16, device="cuda")
        mm_f = t_us(lambda: torch.mm(a2, wm, out=yo))
        st_f = t_us(lambda: (yo.float().sum(0), (yo.float() ** 2).sum(0)))
        g2 = dy.view(npix, cout)
        wdm = wm.t().contiguous()
        xo = torch.empty(npix, cp, dtype=torch.bfloat16, device="cuda")
        mm_d = t_us(lambda: torch.mm(g2, wdm, out=xo))
        by = 2
        floor_f = (npix * cin + npix * cout) * by / 5.0e6  # us at 5 TB/s
        floor_d = (npix * cout + 2 * npix * cin) * by / 5.0e6
        r.update({"psx_fwd_us": round(fwd, 1), "psx_fwd_nostats_us": round(fwd_ns, 1), "psx_fwd_det_us": round(fwd_det, 1), "psx_fwd_tbs": round((npix * (cin + cout) * by) / fwd / 1e6, 2),
                  "hipblaslt_fwd_us": round(mm_f, 1), "torch_stats_pass_us": round(st_f, 1),
                  "psx_dgrad_res_us": round(dg, 1), "hipblaslt_dgrad_us": round(mm_d, 1),
                  "floor_fwd_us": round(floor_f, 1), "floor_dgrad_res_us": round(floor_d, 1)})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
