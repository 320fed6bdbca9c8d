"""Top-k codec HIP kernels (csrc/kernels/topk.hip) vs the PyTorch fp32 reference path."""
import time

import pytest
import torch

from psx.parallel import topk as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(n, ratio, gs):
    c = T.TopKCodec(n, ratio, "cpu")
    outs = []
    for g in gs:
        outs.append((c.encode(g.cpu().float()).clone(), c.resid.clone()))
    return outs


def _entries(p):
    p = p.cpu()
    cnt, kcap = int(p[0]), int(p[1])
    idx = p[4:4 + cnt].long()
    val = p[4 + kcap:].view(torch.float16)[:cnt].float()
    order = torch.argsort(idx)
    return idx[order], val[order]


@pytest.mark.parametrize("n,ratio,dtype", [(1_000_003, 0.01, torch.float32), (11_220_132, 0.01, torch.float16),
                                           (4097, 0.3, torch.float32)])
def test_encode_is_topk_with_error_feedback(n, ratio, dtype):
    """Property check (valid for any tie-breaking): exactly k entries, every sent |acc| >= every
    unsent |acc|, values = fp16(acc), residual + sent == acc."""
    torch.manual_seed(0)
    c = T.TopKCodec(n, ratio, DEV)
    for step in range(3):
        g = torch.randn(n, device=DEV).to(dtype)
        acc = c.resid + g.float()
        p = c.encode(g)
        torch.cuda.synchronize()
        assert int(p[0]) == c.k
        idx, val = _entries(p)
        assert idx.unique().numel() == c.k
        a = acc.cpu()
        mask = torch.zeros(n, dtype=torch.bool)
        mask[idx] = True
        assert a[mask].abs().min() >= a[~mask].abs().max()
        assert torch.equal(val, a[idx].half().float())
        sent = torch.zeros(n, device=DEV)
        T.decode_add(p, sent, 1.0, c.kcap)
        assert torch.allclose(c.resid + sent, acc, atol=1e-6)


def test_encode_matches_reference_without_ties():
    torch.manual_seed(0)
    n = 1_000_003
    gs = [torch.randn(n, device=DEV) for _ in range(3)]
    refs = _ref(n, 0.01, gs)
    c = T.TopKCodec(n, 0.01, DEV)
    for g, (pr, rres) in zip(gs, refs):
        p = c.encode(g)
        i1, v1 = _entries(p)
        i2, v2 = _entries(pr)
        assert torch.equal(i1, i2) and torch.equal(v1, v2)
        assert torch.allclose(c.resid.cpu(), rres, atol=1e-6)


def test_ties_at_zero_and_decode():
    n = 100_000
    g = torch.zeros(n, device=DEV)
    nz = torch.randperm(n, device=DEV)[:50]
    g[nz] = torch.randn(50, device=DEV)
    c = T.TopKCodec(n, 0.001, DEV)  # k = 100 > 50 nonzeros: 50 zero ties fill the payload
    p = c.encode(g)
    torch.cuda.synchronize()
    assert int(p[0]) == 100
    idx, val = _entries(p)
    assert set(nz.cpu().tolist()) <= set(idx.tolist())
    dst = torch.zeros(n, device=DEV)
    T.decode_add(p, dst, 2.0, c.kcap)
    want = torch.zeros(n)
    T.decode_add(p.cpu(), want, 2.0, c.kcap)
    assert torch.equal(dst.cpu(), want)
    assert torch.allclose(dst.cpu(), 2 * g.cpu().half().float())


def test_encode_speed_resnet18():
    n = 11_220_132
    g = torch.randn(n, device=DEV).half()
    c = T.TopKCodec(n, 0.01, DEV)
    for _ in range(3):
        c.encode(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        c.encode(g)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 20 * 1e6
    print(f"topk encode n={n} k={c.k}: {us:.1f} us")
    assert us < 2000


def test_encode_without_gradient_selects_from_resid():
    """g = NULL (tk_pass_a<float, false>): selection straight from the residual equals the encode of
    the same values pushed as a gradient onto a zero residual, including an n that leaves a
    partial last tile and empty chunks."""
    from psx.ops import kernels as K

    torch.manual_seed(1)
    for n in (1_000_003, 5000):
        g = torch.randn(n, device=DEV)
        a = T.TopKCodec(n, 0.01, DEV)
        pa = a.encode(g).clone()
        b = T.TopKCodec(n, 0.01, DEV)
        b.resid.copy_(g)
        K.topk_encode(None, b.resid, b.k, b.kcap, b.payload, b.ws)
        torch.cuda.synchronize()
        assert torch.equal(b.payload, pa)
        assert torch.equal(b.resid, a.resid)
