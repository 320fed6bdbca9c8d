"""Deterministic mode (engine ``deterministic=True`` / PSX_DETERMINISTIC=1 / --deterministic): every
BN statistic is reduced in a fixed order (csrc/kernels/bnfin.hpp DetRed), so a training step is
bit-reproducible. With that, paths that must compute the same step are compared with
``torch.equal``: two runs, graph replay vs eager, the weight gradients on the side stream vs the
main stream, segmented vs single graphs — and the SURVEY §4.2 equivalence row: a W=1, K=1 sync PS
run equals plain single-process SGD bit for bit over 5 steps (fp32 path, fp32 wire)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import ResNet18  # noqa: E402
from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"


def _setup(dtype, B=32, **kw):
    torch.manual_seed(0)
    model = ResNet18(100)
    lay = ParamLayout.from_module(model)
    arena, _ = lay.pack(model)
    eng = HipResNetEngine(model, lay, B, grad_dtype=torch.float32, dtype=dtype, deterministic=True, **kw)
    imgs = torch.randint(0, 256, (256, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (256,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(B, dtype=torch.int32, device=DEV))
    return model, lay, arena.to(DEV), eng, imgs, labs


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_two_runs_and_graph_replay_bit_identical(dtype):
    model, lay, arena, eng, imgs, labs = _setup(dtype)
    outs = []
    for _ in range(2):
        a = arena.clone()
        eng.reset_stat_shift()  # engine state besides the arena: the BN statistic shifts
        eng.train_step(a, imgs, labs)
        torch.cuda.synchronize()
        outs.append((eng.grads.clone(), a.clone()))
    assert torch.equal(outs[0][0], outs[1][0])  # gradients
    assert torch.equal(outs[0][1], outs[1][1])  # running statistics in the local arena
    a = arena.clone()
    eng.reset_stat_shift()
    eng.capture(a, imgs, labs, warmup=1)
    a.copy_(arena)
    eng.step_graph()
    torch.cuda.synchronize()
    assert torch.equal(eng.grads, outs[0][0])
    assert torch.equal(a, outs[0][1])


def test_side_stream_and_segments_bit_identical(monkeypatch):
    """the weight gradients on the side stream (default) equal the main-stream ones,
    eager and graph, and a segmented backward (per-bucket graphs) equals the single graph."""
    from psx.parallel.overlap import plan_buckets

    monkeypatch.setenv("PSX_TUNE", "wgrad_stream=0")
    _, lay, arena, main, imgs, labs = _setup(torch.float32)
    monkeypatch.setenv("PSX_TUNE", "wgrad_stream=1")
    _, _, _, side, _, _ = _setup(torch.float32)
    assert main.wg_stream is None and side.wg_stream is not None
    grads = []
    for eng in (main, side):
        a = arena.clone()
        eng.train_step(a, imgs, labs)
        torch.cuda.synchronize()
        grads.append(eng.grads.clone())
    assert torch.equal(grads[0], grads[1])
    a = arena.clone()
    side.reset_stat_shift()
    side.capture(a, imgs, labs, warmup=1)
    a.copy_(arena)
    side.step_graph()
    torch.cuda.synchronize()
    assert torch.equal(side.grads, grads[0])
    side.set_segments([b.keys for b in plan_buckets(lay, 2 << 20)])
    a = arena.clone()
    side.reset_stat_shift()
    side.capture(a, imgs, labs, warmup=1)
    a.copy_(arena)
    seen = []
    side.step_graph(on_segment=seen.append)
    torch.cuda.synchronize()
    assert len(seen) == 4 and torch.equal(side.grads, grads[0])


def test_sync_w1_equals_single_process_sgd():
    """SURVEY §4.2 'Equivalence': sync mode, W = 1, K = 1, same lr — the parameter server's master
    state after 5 rounds is bit-identical to plain single-process SGD with the same engine, data
    order and fp32 gradients (fp32 compute, fp32 wire, fp32 fetch)."""
    from psx.parallel.compute import HipCompute
    from psx.parallel.runner import build_state, make_datasets, make_local_channel
    from psx.parallel.server import ParameterServer
    from psx.parallel.worker import Worker
    from psx.utils.config import PSConfig

    cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=1024, eval_every=0, verbose=0, lr=0.1,
                   max_steps=5, mode="sync", workers=1, codec="none", deterministic=True).validate()
    model, lay, arena, counters = build_state(cfg)
    train, _ = make_datasets(cfg, torch.device(DEV), 100)
    srv = ParameterServer(cfg, lay, arena.clone(), counters, device=DEV, total_workers=1, log=lambda *a, **k: None)
    comp = HipCompute(model, lay, 64, DEV, grad_dtype=torch.float32, use_graph=True, dtype="fp32", deterministic=True)
    wk = Worker(cfg, comp, make_local_channel(cfg, srv, lay, DEV), train, None, worker_name="w", rank=0,
                log=lambda *a, **k: None, requested_id=0)
    wk.connect_to_server()
    wk.setup_data()
    wk.run_training()
    assert srv.core.global_step == 5
    # plain SGD: the same engine settings, data order and augmentation seed, no server
    ref = HipCompute(model, lay, 64, DEV, grad_dtype=torch.float32, use_graph=True, dtype="fp32", deterministic=True)
    ref.local_arena.copy_(arena.to(DEV))
    batches = wk.sampler.epoch_indices(0)
    n = lay.param_numel
    for i in range(5):
        ref.train_step(train, batches[i])
        K.sgd_apply(ref.local_arena[:n], ref.grads, 0.1, n=n)
    torch.cuda.synchronize()
    assert torch.equal(srv.arena[:n], ref.local_arena[:n])
