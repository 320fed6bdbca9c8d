"""Microbenchmark of the conv-operand unpack kernels (csrc/kernels/optim.hip) on the ResNet-18
table: per-tap kernel (fp32 source), flat-grid kernel (fp32 / bf16 image source), against a
plain device copy of the same byte volume.

usage: python bench/unpack_probe.py [--iters 200]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import build_model  # noqa: E402
from psx.ops import kernels as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(5):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--model", default="resnet18")
    a = ap.parse_args()
    model = build_model(a.model, None, seed=0)
    lay = ParamLayout.from_module(model)
    arena, _ = lay.pack(model)
    arena = arena.cuda()
    hw = (32, 32) if a.model == "resnet18" else (224, 224)
    eng = HipResNetEngine(model, lay, 2, in_hw=hw)
    img = arena[: lay.param_numel].to(torch.bfloat16)
    out = {"ntiles": eng.ntiles, "ndesc": eng.ndesc, "wbuf_MB": eng.wbuf.numel() * 2 / 1e6}
    out["tap_fp32_us"] = timeit(lambda: K.param_unpack(arena, eng.descs, eng.ndesc, eng.wbuf), a.iters)
    out["tiles_fp32_us"] = timeit(lambda: K.param_unpack_tiles(arena, eng.descs, eng.ndesc, eng.ntiles, eng.wbuf),
                                  a.iters)
    out["tiles_bf16_us"] = timeit(lambda: K.param_unpack_tiles(img, eng.descs, eng.ndesc, eng.ntiles, eng.wbuf),
                                  a.iters)
    dst = torch.empty_like(eng.wbuf)
    out["copy_wbuf_us"] = timeit(lambda: dst.copy_(eng.wbuf), a.iters)
    print(json.dumps({k: round(v, 2) if isinstance(v, float) else v for k, v in out.items()}))


if __name__ == "__main__":
    main()
