"""Run one fused Winograd launch shape in a loop (for rocprofv3 counter collection)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402

B, c, hw = int(os.environ.get("B", "128")), int(os.environ.get("C", "64")), int(os.environ.get("HW", "32"))
x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
w = torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5
uf = torch.empty(40 * c * c, device="cuda")
K.WinoWeightBatch([(w, uf, c, c, False, 1)])()
y = torch.empty(B, hw, hw, c, device="cuda")
stats = torch.zeros(K.STAT_SLOTS, 2, c, device="cuda")
for _ in range(int(os.environ.get("ITERS", "20"))):
    K.wino_fused(x, uf, y, None, stats, None, B, hw, hw, c, c)
torch.cuda.synchronize()
print("ok")
