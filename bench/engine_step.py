"""Single-GPU micro-benchmark of the worker training step.

Compares (a) the psx HIP engine (eager launches), (b) the same step replayed from a HIP graph,
and (c) a PyTorch-ROCm reference step (channels_last, MIOpen convs, autograd, SGD; bf16 autocast
for --dtype bf16, plain fp32 with TF32 off for --dtype fp32) on the same ResNet-18 / batch — the
library baseline our kernels must beat.

    python bench/engine_step.py --batch 128 --iters 50 [--dtype fp32] [--model resnet50]

--model resnet50: the ImageNet-shaped ResNet-50 (224x224, 1000 classes; BASELINE config 5's
model) on the same terms.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import psx  # noqa: E402,F401
from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import ResNet18, ResNet50  # noqa: E402
from psx.ops import kernels as K  # noqa: E402


def timeit(fn, iters, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--model", choices=["resnet18", "resnet50"], default="resnet18")
    a = ap.parse_args()
    r50 = a.model == "resnet50"
    mk = (lambda: ResNet50(1000)) if r50 else (lambda: ResNet18(100))
    hw, ncls = (224, 1000) if r50 else (32, 100)
    f32 = a.dtype == "fp32"
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    B = a.batch
    torch.manual_seed(0)
    model = mk()
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    arena = arena.cuda()
    kw = {}
    if r50:  # ImageNet-shaped input and normalisation, as parallel/compute.py builds it
        from psx.models.engine import IMAGENET_MEAN, IMAGENET_STD
        kw = dict(in_hw=(hw, hw), mean=IMAGENET_MEAN, std=IMAGENET_STD)
    eng = HipResNetEngine(model, layout, B, dtype=torch.float32 if f32 else torch.bfloat16, **kw)
    n = 1024 if r50 else 50000
    imgs = torch.empty(n, hw, hw, 3, dtype=torch.uint8, device="cuda")
    labs = torch.empty(n, dtype=torch.int32, device="cuda")
    K.synth_gen(imgs, labs, n, hw, hw, ncls, 1)
    eng.index.copy_(torch.randperm(n, device="cuda")[:B].to(torch.int32))
    res = {"model": a.model, "batch": B, "dtype": a.dtype}

    def step():
        eng.train_step(arena, imgs, labs)
        K.sgd_apply(arena, eng.grads, 0.0, n=layout.param_numel)  # lr 0: keep weights fixed

    if a.only in ("", "eager"):
        t = timeit(step, a.iters)
        res["hip_eager_ms"] = t * 1e3
        res["hip_eager_img_s"] = B / t
    if a.only in ("", "graph"):
        eng.capture(arena, imgs, labs)

        def gstep():
            eng.step_graph()
            K.sgd_apply(arena, eng.grads, 0.0, n=layout.param_numel)

        t = timeit(gstep, a.iters)
        res["hip_graph_ms"] = t * 1e3
        res["hip_graph_img_s"] = B / t
    if not a.no_torch and a.only in ("", "torch"):
        m = mk().cuda().to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(m.parameters(), lr=0.1)
        x = torch.randn(B, 3, hw, hw, device="cuda").to(memory_format=torch.channels_last)
        y = torch.randint(0, ncls, (B,), device="cuda")

        def tstep():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=not f32):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()

        t = timeit(tstep, a.iters)
        res[f"torch_{a.dtype}_ms"] = t * 1e3
        res[f"torch_{a.dtype}_img_s"] = B / t
    print(json.dumps(res))


if __name__ == "__main__":
    main()
