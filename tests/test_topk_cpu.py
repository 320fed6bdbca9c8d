"""Top-k gradient codec (parallel/topk.py) on the CPU path: selection, error feedback, wire
format, server decode, and end-to-end PS runs (loopback + gloo) with --codec topk."""
import pytest
import torch

from psx.models.layout import ParamLayout
from psx.models.resnet import TinyResNet
from psx.parallel import topk as T
from psx.parallel.runner import run_local
from psx.parallel.server import ParameterServer
from psx.utils.config import PSConfig

from .test_ps_cpu import TINY, _spawn, tiny_cfg


def test_encode_selects_exact_topk_with_error_feedback():
    torch.manual_seed(0)
    n, ratio = 10_000, 0.01
    c = T.TopKCodec(n, ratio)
    assert c.k == 100 and c.nbytes == 4 * T.payload_words(100)
    g = torch.randn(n)
    p = c.encode(g.clone())
    cnt, kcap, nn = int(p[0]), int(p[1]), int(p[2])
    assert (cnt, kcap, nn) == (100, 100, n)
    idx = p[4:4 + cnt].long()
    want = torch.topk(g.abs(), 100).indices
    assert set(idx.tolist()) == set(want.tolist())
    sent = torch.zeros(n)
    T.decode_add(p, sent, 1.0, kcap)
    # error feedback: residual + sent == accumulated gradient (exact up to fp32 rounding)
    assert torch.allclose(c.resid + sent, g, atol=1e-6)
    assert torch.allclose(sent[idx], g[idx].half().float())
    # second step selects from resid + g2: large unsent entries eventually go out
    g2 = torch.zeros(n)
    p2 = c.encode(g2)
    idx2 = p2[4:4 + int(p2[0])].long()
    assert torch.allclose(c.resid[idx2].abs(), torch.zeros(len(idx2)), atol=1e-3)


def test_server_sparse_apply_matches_dense():
    torch.manual_seed(1)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    for mom in (0.0, 0.9):
        cfg = tiny_cfg(mode="async", workers=1, codec="topk", topk_ratio=0.05, momentum=mom)
        s1 = ParameterServer(cfg, lay, arena.clone(), counters, total_workers=1, log=lambda *a: None)
        s2 = ParameterServer(cfg, lay, arena.clone(), counters, total_workers=1, log=lambda *a: None)
        for s in (s1, s2):
            s.register_worker("w", 0)
        enc = T.TopKCodec(lay.param_numel, 0.05)
        p = enc.encode(torch.randn(lay.param_numel))
        dense = T.decode_add(p, torch.zeros(lay.param_numel), 1.0, enc.kcap)
        assert s1.push_gradients(0, p, 0)
        assert s2.push_gradients(0, dense, 0)
        assert torch.allclose(s1.arena, s2.arena, atol=1e-6)


@pytest.mark.parametrize("mode,workers", [("sync", 2), ("async", 3)])
def test_run_local_topk(mode, workers):
    cfg = tiny_cfg(mode=mode, workers=workers, codec="topk", topk_ratio=0.02, eval_every=0)
    res = run_local(cfg, log=lambda *a, **k: None)
    srv = res["server"]
    steps = -(-(96 // workers) // 8)
    assert srv["gradients_processed"] == workers * steps
    # compressed push: far fewer bytes than the fp16 wire
    dense = workers * steps * 2 * ParamLayout.from_module(TinyResNet(10)).param_numel
    assert 0 < srv["bytes_pushed"] < 0.1 * dense


def test_topk_multi_epoch_run():
    cfg = tiny_cfg(mode="sync", workers=1, codec="topk", topk_ratio=0.05, eval_every=0, epochs=4,
                   train_samples=64, lr=0.05)
    res = run_local(cfg, log=lambda *a, **k: None)
    assert res["server"]["global_steps_completed"] == 4 * 8


@pytest.mark.parametrize("args", [["--mode", "sync"], ["--mode", "sync", "--topology", "dedicated"],
                                  ["--mode", "async", "--staleness-bound", "50"]])
def test_dist_topk_gloo(args):
    recs, _ = _spawn(3, args + ["--codec", "topk", "--topk-ratio", "0.02"] + TINY)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"][0]
    assert srv["global_steps_completed"] > 0 and srv["gradients_processed"] > 0
