"""Candidate counts of the top-k encoder (state words of the workspace) over repeated encodes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import psx  # noqa: E402,F401
from psx.parallel import topk as T  # noqa: E402

n = 11_220_132
g = torch.randn(n, device="cuda") * 1e-3
c = T.TopKCodec(n, 0.01, "cuda")
for it in range(12):
    c.encode(g)
    torch.cuda.synchronize()
    st = c.ws[4096:4096 + 6].cpu().tolist()
    print(f"iter {it}: b0={st[1]} cnt_gt={st[2]} krem={st[0]} n_c={st[3]} ({100 * st[3] / n:.2f}% of n) need={st[5]}")
