import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import psx
from psx.ops import kernels as K
torch.manual_seed(0)
DEV='cuda'
n, cin, cout, hw, k = 1, 64, 64, 8, 1
x = torch.randn(n, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
dy = torch.randn(n, cout, hw, hw, device=DEV).to(torch.bfloat16).float()
X = x.permute(0,2,3,1).reshape(-1, cin)   # [pix][c]
D = dy.permute(0,2,3,1).reshape(-1, cout) # [pix][oc]
ref = D.t() @ X   # [oc][c]
part = torch.zeros(4 * cout * 64, device=DEV)
splits = K.conv_wgrad_splits(n, hw, hw, cin, cout, 1, 1, 0, 64)
print('splits', splits)
K.conv_wgrad(X.to(torch.bfloat16).contiguous(), D.to(torch.bfloat16).contiguous(), part, n, hw, hw, cin, cout, 1, 1, 0, 64, splits)
torch.cuda.synchronize()
got = part[:cout*64].view(cout, 64)
print('rel', ((got-ref).abs().max()/ref.abs().max()).item())
# try candidate permutations
cands = {'T': ref.t()}
for name, c in cands.items():
    print(name, ((got-c).abs().max()/ref.abs().max()).item())
# single-pixel probes: X = e_pix_a * e_c, D = e_pix * e_oc
for (pa, ca, pb, ob) in [(0,0,0,0),(0,1,0,0),(0,0,0,1),(1,0,1,0),(5,3,5,7),(17,9,17,2),(40,33,40,50)]:
    Xs = torch.zeros(64, cin, device=DEV); Ds = torch.zeros(64, cout, device=DEV)
    Xs[pa, ca] = 1; Ds[pb, ob] = 1
    part.zero_()
    K.conv_wgrad(Xs.to(torch.bfloat16).contiguous(), Ds.to(torch.bfloat16).contiguous(), part, n, hw, hw, cin, cout, 1, 1, 0, 64, splits)
    torch.cuda.synchronize()
    g = part[:cout*64].view(cout, 64)
    nz = (g != 0).nonzero().tolist()
    print((pa,ca,pb,ob), 'expect (oc,c)=', (ob, ca), 'got', nz[:6])
