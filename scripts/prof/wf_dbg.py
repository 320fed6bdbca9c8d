import torch, sys
sys.path.insert(0, '/root/repo')
import psx
from psx.ops import kernels as K
import torch.nn.functional as F
DEV='cuda'
def nhwc(t): return t.permute(0,2,3,1).contiguous()
for (nb,h,c,k,res,vout) in [(8,16,64,128,True,True),(8,16,64,128,True,False),(8,16,64,128,False,True),(8,16,64,128,False,False),(8,16,64,64,True,True)]:
    torch.manual_seed(0)
    x = torch.relu(torch.randn(nb, c, h, h, device=DEV, dtype=torch.float64))
    w = torch.randn(k, c, 3, 3, device=DEV, dtype=torch.float64) * (2.0 / (9 * c)) ** 0.5
    r = torch.randn(nb, k, h, h, device=DEV, dtype=torch.float64) if res else None
    ref = nhwc(F.conv2d(x, w, padding=1) + (r if res else 0))
    uf = torch.full((40*k*c,), float('nan'), device=DEV)
    K.WinoWeightBatch([(w.float().contiguous(), uf, k, c, False, 1)])()
    y = torch.full((nb,h,h,k), float('nan'), device=DEV)
    stats = torch.zeros(K.STAT_SLOTS,2,k,device=DEV)
    v = torch.full((K.wino_v_floats(nb,h,h,c),), float('nan'), device=DEV) if vout else None
    K.wino_fused(nhwc(x.float()), uf, y, nhwc(r.float()) if res else None, stats, v, nb,h,h,c,k)
    torch.cuda.synchronize()
    err = (y.double()-ref).abs()
    bad = err > 1e-3
    print((nb,h,c,k,res,vout), 'maxerr', err.max().item(), 'nbad', bad.sum().item(), 'nan', torch.isnan(y).sum().item())
    if bad.any():
        idx = bad.nonzero()
        print(' bad n', idx[:,0].unique().tolist()[:10], 'rows', idx[:,1].unique().tolist()[:16], 'cols', idx[:,2].unique().tolist()[:16], 'ch', idx[:,3].unique().tolist()[:20], len(idx[:,3].unique()))
