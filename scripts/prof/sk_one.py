"""5 launches of the stream-K GEMM on the 8x8x256 Winograd shape (PMC runs)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402

m, n, kd, nb = 512, 256, 256, 36
a = torch.randn(nb, m, kd, device="cuda")
b = torch.randn(n, nb, kd, device="cuda")
c = torch.empty(nb, m, n, device="cuda")
for _ in range(5):
    assert K.sk_gemm_nt(a, b, c, m, n, kd, nb, (kd, m * kd), (nb * kd, kd), (n, m * n), bn=int(os.environ.get("BN", "0"))) == 0
torch.cuda.synchronize()
