# one fused Winograd weight-gradient shape (default ResNet-18 32x32x64, B=128), 5 launches, for PMC runs
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402

B, hw, c = int(os.environ.get("B", "128")), int(os.environ.get("HW", "32")), int(os.environ.get("C", "64"))
x = torch.relu(torch.randn(B, hw, hw, c, device="cuda"))
dy = torch.randn(B, hw, hw, c, device="cuda")
q = K.wino_wgrad_fused_q(B, hw, hw, c, c)
part = torch.empty(36 * q * c * c, device="cuda")
g = torch.empty(c * c * 9, device="cuda", dtype=torch.float16)
for _ in range(5):
    K.wino_wgrad_fused(x, dy, part, g, B, hw, hw, c, c)
torch.cuda.synchronize()
print("ok", q)
