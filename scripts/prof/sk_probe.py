"""Stream-K GEMM timing on the 8x8x256 Winograd shape (diagnostic modes: build a kernel variant
with -D PSX_SK_PROBE=<bits>, csrc/build.py --variant, and load it with PSX_KERNELS_LIB)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.ops import kernels as K  # noqa: E402

m, n, kd, nb = [int(v) for v in os.environ.get("SHAPE", "512,256,256,36").split(",")]
a = torch.randn(nb, m, kd, device="cuda")
b = torch.randn(n, nb, kd, device="cuda")
c = torch.empty(nb, m, n, device="cuda")
f = lambda: K.sk_gemm_nt(a, b, c, m, n, kd, nb, (kd, m * kd), (nb * kd, kd), (n, m * n), bn=int(os.environ.get("BN", "0")))
for _ in range(3):
    f()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
s.record()
for _ in range(20):
    f()
e.record()
torch.cuda.synchronize()
print(os.environ.get("PSX_SK_PROBE", "0"), os.environ.get("BN", "0"), "%.1f us" % (s.elapsed_time(e) * 1e3 / 20))
