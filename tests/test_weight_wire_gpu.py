"""Weight-image fetch path (parallel/codec.py WeightWire) on one MI355X.

* the flat-grid unpack kernel (csrc/kernels/optim.hip param_unpack_tiles) produces exactly the
  operands of the per-tap kernel, from the fp32 arena and from a bf16 image;
* the SGD apply's image output is the bf16 rounding of the fp32 result;
* whole runs with the fast path on and off end in bit-identical master states (loopback and
  the RCCL channel at world size 1).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.models.engine import HipResNetEngine  # noqa: E402
from psx.models.layout import ParamLayout  # noqa: E402
from psx.models.resnet import build_model  # noqa: E402
from psx.ops import kernels as K  # noqa: E402
from psx.parallel.runner import run_local  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("model_name,hw", [("resnet18", (32, 32)), ("resnet50", (224, 224))])
def test_unpack_tiles_matches_per_tap(model_name, hw):
    torch.manual_seed(0)
    model = build_model(model_name, None, seed=0)
    lay = ParamLayout.from_module(model)
    arena, _ = lay.pack(model)
    arena = (arena + 0.01 * torch.randn_like(arena)).cuda()
    eng = HipResNetEngine(model, lay, 2, in_hw=hw)
    ref = torch.zeros_like(eng.wbuf)
    K.param_unpack(arena, eng.descs, eng.ndesc, ref)
    got = torch.zeros_like(eng.wbuf)
    K.param_unpack_tiles(arena, eng.descs, eng.ndesc, eng.ntiles, got)
    torch.cuda.synchronize()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    img = arena[: lay.param_numel].to(torch.bfloat16)
    got2 = torch.zeros_like(eng.wbuf)
    K.param_unpack_tiles(img, eng.descs, eng.ndesc, eng.ntiles, got2)
    torch.cuda.synchronize()
    assert torch.equal(got2.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize("gather", [False, True])
def test_unpack_launch_scatters_fp32_remainder(gather):
    """The extra workgroups of the unpack launch: dst[idx] = small (wire) or dst[idx] = arena[idx]."""
    from psx.parallel.codec import WeightWire

    torch.manual_seed(2)
    model = build_model("resnet18", None, seed=0)
    lay = ParamLayout.from_module(model)
    arena, _ = lay.pack(model)
    arena = (arena + 0.01 * torch.randn_like(arena)).cuda()
    eng = HipResNetEngine(model, lay, 2, in_hw=(32, 32))
    w = WeightWire(lay, "cuda")
    w.publish_full(arena)
    dst = torch.full_like(arena, -7.0)
    ref = dst.clone()
    w.consume_small(ref)
    got_w = torch.zeros_like(eng.wbuf)
    src = arena if gather else w.small
    K.param_unpack_tiles(w.img, eng.descs, eng.ndesc, eng.ntiles, got_w, scatter=(src, w.small_index, dst, gather))
    ref_w = torch.zeros_like(eng.wbuf)
    K.param_unpack_tiles(w.img, eng.descs, eng.ndesc, eng.ntiles, ref_w)
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)
    assert torch.equal(got_w.view(torch.int16), ref_w.view(torch.int16))


@pytest.mark.parametrize("n,mom", [(1 << 20, False), (1000003, False), (4096, True)])
def test_sgd_apply_image_is_bf16_of_result(n, mom):
    torch.manual_seed(1)
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda").half()
    buf = torch.zeros(n, device="cuda") if mom else None
    img = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    p_ref = p.clone()
    K.sgd_apply(p_ref, g, 0.1, gscale=0.5, momentum=0.9 if mom else 0.0, buf=buf.clone() if mom else None,
                first=True)
    K.sgd_apply(p, g, 0.1, gscale=0.5, momentum=0.9 if mom else 0.0, buf=buf, first=True, img=img)
    torch.cuda.synchronize()
    assert torch.equal(p, p_ref)
    assert torch.equal(img.view(torch.int16), p.to(torch.bfloat16).view(torch.int16))


def _cfg(**kw):
    base = dict(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=0, verbose=0, lr=0.1,
                max_steps=6, dtype="bf16")
    base.update(kw)
    return PSConfig(**base).validate()


def _close(a, b, rel=2e-4):
    """Whole runs differ by the run-to-run noise of the fp32-atomic BN statistics."""
    return abs(a - b) <= rel * max(abs(a), abs(b))


@pytest.mark.parametrize("use_graph", [True, False])
def test_fetched_operands_identical(use_graph):
    """Server state after a few updates -> worker A (WeightWire) and worker B (fp32 arena fetch):
    after each step's prologue both engines hold identical bf16 operands and fp32 small entries."""
    from psx.parallel.compute import HipCompute
    from psx.parallel.runner import build_state, make_datasets, make_local_channel
    from psx.parallel.server import ParameterServer
    from psx.parallel.worker import InProcessChannel

    cfg = _cfg(mode="sync", workers=1, use_graph=use_graph)
    model, lay, arena, counters = build_state(cfg)
    srv = ParameterServer(cfg, lay, arena, counters, device="cuda", total_workers=1, log=lambda *a, **k: None)
    srv.register_worker("w", 0)
    train, _ = make_datasets(cfg, torch.device("cuda"), 100)
    ca = HipCompute(model, lay, 64, "cuda", use_graph=use_graph, dtype="bf16")
    cb = HipCompute(model, lay, 64, "cuda", use_graph=use_graph, dtype="bf16")
    cha = make_local_channel(cfg, srv, lay, "cuda")
    assert cha.weight_wire() is not None
    ca.use_wire(cha.weight_wire(), small_from=cha.small_source())
    assert cha.weight_wire() is srv.wire and cha.small_source() is srv.arena  # read in place
    chb = InProcessChannel(srv)
    idx = list(range(64))
    for step in range(3):
        cha.fetch(0, ca.local_arena)
        chb.fetch(0, cb.local_arena)
        ca.train_step(train, idx)
        cb.train_step(train, idx)
        torch.cuda.synchronize()
        assert torch.equal(ca.engine.wbuf.view(torch.int16), cb.engine.wbuf.view(torch.int16)), step
        for name, e in lay.entries.items():
            if e.region == "param" and len(e.shape) != 4:
                assert torch.equal(lay.view(ca.local_arena, name), lay.view(cb.local_arena, name)), (step, name)
        srv.apply(ca.grads, 1.0)  # the next version (its image comes out of this apply)


@pytest.mark.parametrize("workers,bn_sync", [(1, False), (2, True)])
def test_loopback_image_path_matches(workers, bn_sync, monkeypatch):
    sums = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PSX_WEIGHT_IMAGE", flag)
        res = run_local(_cfg(mode="sync", workers=workers, bn_sync=bn_sync), log=lambda *a, **k: None)
        sums[flag] = res["server"]["final_param_checksum"]
        assert res["server"]["global_steps_completed"] == 6
    assert _close(sums["1"], sums["0"]), sums


_DIST = r"""
import json, sys
sys.path.insert(0, {root!r})
import psx
from psx.parallel.runner import run_distributed
from psx.utils.config import PSConfig
cfg = PSConfig(model="resnet18", batch_size=64, epochs=1, train_samples=2048, eval_every=0, verbose=0, lr=0.1,
               max_steps=6, mode="sync", dtype="bf16").validate()
res = run_distributed(cfg, log=lambda *a, **k: None)
print("RESULT " + json.dumps(res["server"]["final_param_checksum"]))
"""


def test_rccl_channel_image_path_matches_loopback():
    """world size 1 through DistTransport (RCCL broadcast/reduce) with the image path on and off,
    against the loopback run: all three final states are identical."""
    out = {}
    for flag, port in (("1", 29641), ("0", 29642)):
        env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PSX_WEIGHT_IMAGE=flag)
        r = subprocess.run([sys.executable, "-c", _DIST.format(root=ROOT)], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
        out[flag] = json.loads(line[7:])
    loop = run_local(_cfg(mode="sync", workers=1), log=lambda *a, **k: None)["server"]["final_param_checksum"]
    assert _close(out["1"], out["0"]) and _close(out["1"], loop), (out, loop)
