"""Debug: per-parameter gradient differences between BN-finalize paths (folded vs separate)
and between two identical runs (atomic-order noise baseline)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from tests.test_engine_gpu import setup as _setup  # noqa: E402

DEV = "cuda"
model, layout, arena, eng, x, y = _setup.__wrapped__() if hasattr(_setup, "__wrapped__") else _setup()
n = 256
torch.manual_seed(1)
imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
step0 = eng.step_dev.clone()


def run(fold):
    eng.fin_apply, eng.fuse_fin, eng.fuse_bnbwd = fold, False, False
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    eng.step_dev.copy_(step0)
    a = arena.clone()
    eng.train_step(a, imgs, labs)
    torch.cuda.synchronize()
    return eng.grads.float().clone(), eng.final.float().clone()


g0, f0 = run(False)
g0b, f0b = run(False)
g1, f1 = run(True)
print("final act diff noise", (f0b - f0).norm().item() / f0.norm().item(), "fold", (f1 - f0).norm().item() / f0.norm().item())
print("total grad noise", ((g0b - g0).norm() / g0.norm()).item(), "fold", ((g1 - g0).norm() / g0.norm()).item())
for name in layout.entries:
    try:
        a, b, c = (layout.grad_view(t, name).float() for t in (g0, g0b, g1))
    except Exception:
        continue
    d_noise = ((b - a).norm() / (a.norm() + 1e-12)).item()
    d_fold = ((c - a).norm() / (a.norm() + 1e-12)).item()
    if d_fold > 0.01 or d_noise > 0.01:
        print(f"{name:40s} noise {d_noise:.4f} fold {d_fold:.4f}")
