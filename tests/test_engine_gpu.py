"""Whole-network check: one ResNet-18 training step on the HIP engine vs torch fp32 autograd."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import ResNet18  # noqa: E402
from psx.ops import kernels as K  # noqa: E402

DEV = "cuda"


def _bf16_round_(model):
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, torch.nn.Conv2d):
                m.weight.copy_(m.weight.to(torch.bfloat16).float())


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def _slot_sums(buf, c, det):
    """Per-channel sums of the 2-row slot layout [STAT_SLOTS][2][c] (deterministic mode: the
    fixed-point pairs, csrc/kernels/bnfin.hpp DetRed)."""
    if det:
        return K.det_slot_values(buf, (K.STAT_SLOTS, 2, c)).sum(0).float()
    return buf[:K.STAT_SLOTS * 2 * c].view(K.STAT_SLOTS, 2, c).sum(0)


@pytest.fixture(scope="module")
def setup():
    torch.manual_seed(0)
    B = 32
    model = ResNet18(100)
    _bf16_round_(model)
    layout = ParamLayout.from_module(model)
    arena, _ = layout.pack(model)
    model = model.to(DEV)
    eng = HipResNetEngine(model, layout, B, grad_dtype=torch.float32)
    x = torch.randn(B, 3, 32, 32, device=DEV).to(torch.bfloat16).float()
    y = torch.randint(0, 100, (B,), device=DEV)
    return model, layout, arena.to(DEV), eng, x, y


def test_train_step_matches_torch(setup):
    model, layout, arena, eng, x, y = setup
    arena_k = arena.clone()
    eng.unpack(arena_k)
    K.nchw_to_nhwc(x, eng.x0, x.shape[0], 3, 32, 32, 8)
    eng.labels.copy_(y.to(torch.int32))
    eng.forward(arena_k, train=True)
    eng.head(arena_k, backward=True)
    eng.backward(arena_k)
    torch.cuda.synchronize()

    sd_init = {k: v.clone() for k, v in model.state_dict().items()}
    model.train()
    model.zero_grad()
    out = model(x)
    loss = F.cross_entropy(out, y)
    loss.backward()
    ref32 = {n: p.grad.clone() for n, p in model.named_parameters()}
    sd32 = {k: v.clone() for k, v in model.state_dict().items()}  # running stats after ONE forward
    # torch's own bf16 autocast path sets the precision bar: a randomly initialised ResNet's
    # early-layer gradients are chaotic, so bf16 activations alone move them by a few percent.
    model.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        F.cross_entropy(model(x), y).backward()
    ref16 = {n: p.grad.clone() for n, p in model.named_parameters()}
    assert abs(eng.loss.mean().item() - loss.item()) < 0.02 * max(1.0, loss.item())
    ce, cb = [], []
    for name in ref32:
        g = layout.grad_view(eng.grads, name)
        c_eng, c_bf16 = _cos(g, ref32[name]), _cos(ref16[name], ref32[name])
        ce.append(c_eng)
        cb.append(c_bf16)
        assert c_eng > 0.85 and c_eng > c_bf16 - 0.06, (name, c_eng, c_bf16)
    ce.sort()
    cb.sort()
    assert ce[len(ce) // 2] > cb[len(cb) // 2] - 0.01, (ce, cb)  # median agreement >= torch bf16's
    assert _cos(eng.grads[-5000:], torch.cat([ref32["fc.weight"].flatten(), ref32["fc.bias"]])[-5000:]) > 0.999
    model.load_state_dict(sd_init)
    # running statistics were updated in the worker-local arena exactly like torch's
    for name in ("bn1.running_mean", "layer2.0.bn1.running_var", "layer4.1.bn2.running_mean"):
        got = layout.view(arena_k, name)
        assert torch.allclose(got, sd32[name], rtol=2e-2, atol=2e-3), name


def test_graph_replay_matches_eager(setup):
    model, layout, arena, eng, x, y = setup
    n = 256
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    a1 = arena.clone()
    eng.train_step(a1, imgs, labs)
    torch.cuda.synchronize()
    eager = eng.grads.clone()
    a2 = arena.clone()
    eng.capture(a2, imgs, labs, warmup=1)
    a2.copy_(arena)
    eng.step_graph()
    torch.cuda.synchronize()
    # BN statistics use fp32 atomics (order-dependent last bits) which the chaotic backward of a
    # random-init ResNet amplifies to ~1e-2; the head gradients must agree tightly.
    assert _cos(eng.grads.float(), eager.float()) > 0.97
    fc = layout.entries["fc.weight"].offset
    assert _cos(eng.grads[fc:].float(), eager[fc:].float()) > 0.9999


@pytest.mark.parametrize("mode", ["conv_epilogue", "apply", "apply_bnbwd"])
def test_fused_bn_finalize_matches_separate_kernels(setup, mode):
    """Folded BN finalize gives exactly what the separate finalize kernels compute from the same
    slot sums (every BN layer, two consecutive steps). conv_epilogue: last workgroup of the
    producing launch (engine.fuse_fin); apply (default): every workgroup of the consuming apply
    launch (bnfin.hpp bn_fin_lds), with the backward sums from bn_bwd_reduce or from the dgrad
    epilogue (apply_bnbwd). Also: running statistics updated exactly once per step, and the
    block-internal apply outputs equal bn_apply with the recomputed affine.
    (Whole-step gradients are not compared across paths: at random init two runs of the SAME
    path already differ by ~20% through the atomic-order noise in the statistics.)"""
    model, layout, arena, eng, x, y = setup
    n = 256
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    before = (eng.fin_apply, eng.fuse_fin, eng.fuse_bnbwd)
    eng.fin_apply = mode != "conv_epilogue"
    eng.fuse_fin = mode == "conv_epilogue"
    eng.fuse_bnbwd = mode == "apply_bnbwd"
    a = arena.clone()
    for step in range(2):
        prev = a.clone()
        eng.train_step(a, imgs, labs)
        torch.cuda.synchronize()
        bns = [eng.spec.stem_bn] + [bn for b in eng.spec.blocks for bn in b.bns + ([b.down[1]] if b.down else [])]
        for bs in bns:
            st = eng.bn[bs.name]
            c = bs.c
            fin = [f for k, f in eng._fins.items() if k[0] == "f" and k[1] == bs.name][0]
            aff, sav = torch.empty_like(st["affine"]), torch.empty_like(st["saved"])
            # the slot sums are shifted by the step's statistic shift (engine.py bn_shift)
            K.bn_finalize(eng._red(bs, "fwd"), K.STAT_SLOTS, c, fin.count, layout.view(a, f"{bs.name}.weight"),
                          layout.view(a, f"{bs.name}.bias"), eng.eps, eng.mom, None, None, aff, sav,
                          sshift=st["sshift"])
            bf = [f for k, f in eng._fins.items() if k[0] == "b" and k[1] == bs.name][0]
            coef = torch.empty_like(st["coef"])
            dg = torch.empty(c, dtype=torch.float32, device=DEV)
            db = torch.empty(c, dtype=torch.float32, device=DEV)
            # a BN pair sharing dz (block output BN + shortcut BN) keeps 3 stat rows per slot in
            # the first BN's slot region
            two = [b for b in eng.spec.blocks if b.down and bs.name in (b.bns[-1].name, b.down[1].name)]
            ns, which = (3, 1 if bs.name == two[0].bns[-1].name else 2) if two else (2, 1)
            part = eng._red(two[0].bns[-1] if two else bs, "bwd")
            K.bn_bwd_finalize(part, K.STAT_SLOTS, ns, which, c, bf.count, layout.view(a, f"{bs.name}.weight"),
                              st["saved"], coef, dg.data_ptr(), db.data_ptr(), 1.0, False)
            torch.cuda.synchronize()
            assert torch.allclose(aff, st["affine"], rtol=1e-6, atol=1e-7), (mode, step, bs.name)
            assert torch.allclose(sav, st["saved"], rtol=1e-6, atol=1e-7), (mode, step, bs.name)
            assert torch.allclose(coef, st["coef"], rtol=1e-5, atol=1e-6), (mode, step, bs.name)
            gw = layout.grad_view(eng.grads, f"{bs.name}.weight").float()
            gb = layout.grad_view(eng.grads, f"{bs.name}.bias").float()
            assert torch.allclose(dg, gw, rtol=1e-5, atol=1e-6), (mode, step, bs.name)
            assert torch.allclose(db, gb, rtol=1e-5, atol=1e-6), (mode, step, bs.name)
            # running statistics: exactly one momentum update from this step's batch mean
            m = eng.mom
            rm_want = (1 - m) * layout.view(prev, f"{bs.name}.running_mean") + m * sav[0]
            assert torch.allclose(layout.view(a, f"{bs.name}.running_mean"), rm_want, rtol=1e-5, atol=1e-6), \
                (mode, step, bs.name)
        for b, d in zip(eng.spec.blocks, eng.blk):  # in-block applies (BN + ReLU)
            for i in range(len(b.convs) - 1):
                bs = b.bns[i]
                want = torch.empty_like(d["a"][i])
                K.bn_apply(d["y"][i], eng.bn[bs.name]["affine"], want, bs.c, relu=True)
                torch.cuda.synchronize()
                assert torch.equal(want, d["a"][i]), (mode, step, bs.name)
    eng.fin_apply, eng.fuse_fin, eng.fuse_bnbwd = before


def test_dgrad_fused_bn_backward_sums_match_reduce_kernel(setup):
    """engine.fuse_bnbwd: the BN-backward slot sums produced in the dgrad epilogue equal what the
    separate bn_bwd_reduce pass computes from the stored dgrad output."""
    model, layout, arena, eng, x, y = setup
    n = 256
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    before = eng.fuse_bnbwd
    eng.fuse_bnbwd = True
    a = arena.clone()
    eng.train_step(a, imgs, labs)
    torch.cuda.synchronize()
    checked = 0
    for b, d in zip(eng.spec.blocks, eng.blk):
        for i in range(1, len(b.convs)):  # in-block BNs fed by a dgrad epilogue
            bs = b.bns[i - 1]
            npix = d["da"][i - 1].numel() // bs.c
            ref = torch.zeros_like(eng._red(bs, "bwd"))
            K.bn_bwd_reduce(d["da"][i - 1], d["a"][i - 1], d["y"][i - 1], eng.bn[bs.name]["saved"], ref, npix, bs.c)
            torch.cuda.synchronize()
            # the region is sized for 3 stat rows; NS = 2 here
            got = _slot_sums(eng._red(bs, "bwd"), bs.c, eng.deterministic)
            want = _slot_sums(ref, bs.c, eng.deterministic)
            assert torch.allclose(got, want, rtol=1e-3, atol=1e-3 * want.abs().max().item()), bs.name
            checked += 1
    # the last block's output BN: its sums come out of the head launch (engine.head)
    bs = eng.spec.blocks[-1].bns[-1]
    npix = eng.dfinal.numel() // bs.c
    ref = torch.zeros_like(eng._red(bs, "bwd"))
    K.bn_bwd_reduce(eng.dfinal, eng.final, eng.blk[-1]["y"][-1], eng.bn[bs.name]["saved"], ref, npix, bs.c)
    torch.cuda.synchronize()
    got = _slot_sums(eng._red(bs, "bwd"), bs.c, eng.deterministic)
    want = _slot_sums(ref, bs.c, eng.deterministic)
    assert torch.allclose(got, want, rtol=1e-3, atol=1e-3 * want.abs().max().item()), bs.name
    eng.fuse_bnbwd = before
    assert checked == 8


def test_segmented_graphs_match_single_graph(setup):
    """Backward split into per-bucket graphs (overlapped sync rounds) computes the same step."""
    from psx.parallel.overlap import plan_buckets

    model, layout, arena, eng, x, y = setup
    n = 256
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    a1 = arena.clone()
    eng.capture(a1, imgs, labs, warmup=1)
    a1.copy_(arena)
    eng.step_graph()
    torch.cuda.synchronize()
    ref = eng.grads.clone()
    buckets = plan_buckets(layout, 2 << 20)
    eng.set_segments([b.keys for b in buckets])
    a2 = arena.clone()
    eng.capture(a2, imgs, labs, warmup=1)
    assert len(eng.graphs) == len(buckets) == 4
    a2.copy_(arena)
    seen = []
    eng.step_graph(on_segment=seen.append)
    torch.cuda.synchronize()
    assert seen == [0, 1, 2, 3]
    assert _cos(eng.grads.float(), ref.float()) > 0.97
    fc = layout.entries["fc.weight"].offset
    assert _cos(eng.grads[fc:].float(), ref[fc:].float()) > 0.9999
    eng.set_segments([[k for k, _ in eng.backward_units(None)]])


def test_eval_counts_correct(setup):
    model, layout, arena, eng, x, y = setup
    n = 64
    imgs = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labs = torch.randint(0, 100, (n,), dtype=torch.int32, device=DEV)
    eng.index.copy_(torch.arange(eng.B, dtype=torch.int32, device=DEV))
    eng.unpack(arena)
    eng.evaluate_batch(arena, imgs, labs)
    torch.cuda.synchronize()
    assert 0 <= eng.correct.item() <= eng.B
