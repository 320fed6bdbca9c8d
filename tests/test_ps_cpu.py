"""End-to-end parameter-server runs on CPU: loopback (1 process) and multi-process over gloo.

The multi-process tests launch real ranks (torch.distributed gloo, 127.0.0.1) through the same
runner the GPU job uses (RCCL there); the model is the CPU-sized TinyResNet.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from psx.models.layout import ParamLayout
from psx.models.resnet import TinyResNet
from psx.parallel.compute import TorchCompute
from psx.parallel.runner import run_local
from psx.parallel.server import ParameterServer
from psx.utils import metrics as M
from psx.utils.config import PSConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def tiny_cfg(**kw):
    base = dict(model="resnet_tiny", batch_size=8, epochs=1, train_samples=96, test_samples=32, eval_every=1,
                verbose=0, use_graph=False, lr=0.05)
    base.update(kw)
    return PSConfig(**base).validate()


@pytest.mark.parametrize("workers", [1, 2])
def test_accumulate_pushes_window_mean(monkeypatch, workers):
    """--sync-steps 2 --accumulate: one push per window of 2 batches, carrying the mean of the
    window's batch gradients (the reference pushes the first batch's only); single-worker loop
    and the interleaved multi-worker loopback."""
    from psx.parallel import compute as CM
    from psx.parallel import worker as WM

    batch_g, pushed = {}, {}
    orig_step, orig_push = CM.TorchCompute.train_step, WM.InProcessChannel.push

    def step(self, *a, **k):
        r = orig_step(self, *a, **k)
        batch_g.setdefault(id(self.grads.untyped_storage()), []).append(self.grads.float().clone())
        return r

    def push(self, worker_id, grads, local_step, buffers=None):
        pushed.setdefault(id(grads.untyped_storage()), []).append(grads.float().clone())
        return orig_push(self, worker_id, grads, local_step, buffers)

    monkeypatch.setattr(CM.TorchCompute, "train_step", step)
    monkeypatch.setattr(WM.InProcessChannel, "push", push)
    res = run_local(tiny_cfg(mode="sync", workers=workers, sync_steps=2, accumulate=True, eval_every=0),
                    log=lambda *a, **k: None)
    nb = 12 // workers
    assert res["server"]["global_steps_completed"] == nb // 2
    assert sorted(batch_g) == sorted(pushed) and len(batch_g) == workers
    for key, bg in batch_g.items():
        assert len(bg) == nb and len(pushed[key]) == nb // 2
        for i, p in enumerate(pushed[key]):
            ref = (bg[2 * i] + bg[2 * i + 1]) / 2
            assert torch.allclose(p, ref.half().float(), atol=1e-3, rtol=1e-2), (key, i)


def test_inprocess_sync_matches_manual_average():
    torch.manual_seed(0)
    cfg = tiny_cfg(mode="sync", workers=2)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    srv = ParameterServer(cfg, lay, arena.clone(), counters, total_workers=2, log=lambda *a: None)
    for w in range(2):
        assert srv.RegisterWorker(f"w{w}", w) == (w, 2)
    g0 = torch.randn(lay.param_numel).half()
    g1 = torch.randn(lay.param_numel).half()
    before = srv.arena.clone()
    assert srv.PushGradrients(0, g0, 0) is True  # reference RPC name (typo kept)
    assert torch.equal(srv.arena, before)  # barrier not complete yet
    assert srv.push_gradients(1, g1, 0) is True
    expect = before[: lay.param_numel] - 0.05 * (g0.float() + g1.float()) / 2
    assert torch.allclose(srv.arena[: lay.param_numel], expect, atol=1e-6)
    _, gs = srv.FetchParameters(0)
    assert gs == 1


def test_inprocess_async_staleness_weights():
    cfg = tiny_cfg(mode="async", workers=2, staleness_bound=1)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    srv = ParameterServer(cfg, lay, arena.clone(), counters, total_workers=2, log=lambda *a: None)
    srv.register_worker("a", 0)
    srv.register_worker("b", 1)
    g = torch.ones(lay.param_numel, dtype=torch.float16)
    p0 = srv.arena[0].item()
    assert srv.push_gradients(0, g, 0)  # staleness 0, weight 1
    assert srv.arena[0].item() == pytest.approx(p0 - 0.05, abs=1e-6)
    assert srv.push_gradients(1, g, 0)  # staleness 1, weight 1/1.1
    assert srv.arena[0].item() == pytest.approx(p0 - 0.05 - 0.05 / 1.1, abs=1e-6)
    assert not srv.push_gradients(0, g, 0)  # staleness 2 > bound 1 -> rejected, no update
    assert srv.arena[0].item() == pytest.approx(p0 - 0.05 - 0.05 / 1.1, abs=1e-6)


def test_torch_compute_grads_match_autograd():
    torch.manual_seed(0)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, _ = lay.pack(m)
    from psx.utils.data import DeviceDataset

    ds = DeviceDataset.synthetic(16, 32, 10, seed=0, device="cpu")
    comp = TorchCompute(TinyResNet(10), lay, 8, grad_dtype=torch.float32)
    comp.local_arena.copy_(arena)
    comp.train_step(ds, list(range(8)))
    assert comp.last_loss() > 0
    assert torch.isfinite(comp.grads).all()
    assert comp.grads.abs().sum() > 0


@pytest.mark.parametrize("mode,workers", [("sync", 1), ("sync", 3), ("async", 3)])
def test_run_local(mode, workers, capsys):
    cfg = tiny_cfg(mode=mode, workers=workers)
    res = run_local(cfg, log=lambda *a, **k: None)
    srv = res["server"]
    out = capsys.readouterr().out
    recs = M.parse_lines(out.splitlines())
    types = [r["type"] for r in recs]
    assert types.count("WORKER_FINAL_METRICS") == workers
    assert types.count("SERVER_FINAL_METRICS") == 1
    steps = -(-(96 // workers) // 8)  # ceil(shard / batch)
    assert srv["gradients_processed"] == workers * steps
    if mode == "sync":
        assert srv["global_steps_completed"] == steps
    else:
        assert srv["global_steps_completed"] == workers * steps
        assert srv["max_staleness_observed"] == workers - 1
        assert srv["staleness_histogram"][workers - 1] > 0
    w = [r for r in recs if r["type"] == "WORKER_FINAL_METRICS"][0]
    assert w["local_steps_completed"] == steps and len(w["all_accuracies_percent"]) == 1


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(nproc, args, timeout=240, max_restarts=0):
    """Run a multi-process CPU job; METRICS_JSON records are read from the per-rank jsonl files
    (--log-dir), not from the ranks' merged stdout, where concurrent writes may interleave."""
    import tempfile

    port = _free_port()
    logdir = tempfile.mkdtemp(prefix="psx_metrics_")
    if "--log-dir" not in args:
        args = list(args) + ["--log-dir", logdir]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           f"--max-restarts={max_restarts}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "scripts", "psx_train.py"),
           "--cpu"] + args
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    recs = []
    for f in sorted(os.listdir(logdir)):
        with open(os.path.join(logdir, f)) as fh:
            recs += [json.loads(ln) for ln in fh if ln.strip()]
    return (recs or M.parse_lines(r.stdout.splitlines())), r.stdout


TINY = ["--model", "resnet_tiny", "--batch-size", "8", "--epochs", "1", "--train-samples", "96",
        "--test-samples", "16", "--eval-every", "1", "--verbose", "0", "--no-graph", "--lr", "0.05"]


@pytest.mark.parametrize("topology", ["colocated", "dedicated"])
def test_dist_sync_gloo(topology):
    recs, out = _spawn(3, ["--mode", "sync", "--topology", topology] + TINY)
    W = 3 if topology == "colocated" else 2
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]
    wks = [r for r in recs if r["type"] == "WORKER_FINAL_METRICS"]
    assert len(srv) == 1 and len(wks) == W
    steps = -(-(96 // W + 96 % W) // 8)
    assert srv[0]["global_steps_completed"] == steps
    assert srv[0]["gradients_processed"] == W * steps
    assert sorted(w["worker_id"] for w in wks) == list(range(W))
    assert srv[0]["topology"] == topology and srv[0]["gpus"] == 3


@pytest.mark.parametrize("mode,workers", [("sync", 2), ("async", 2)])
def test_bn_sync_updates_server_running_stats(mode, workers):
    from psx.parallel.runner import build_state

    cfg = tiny_cfg(mode=mode, workers=workers, bn_sync=True, eval_every=0)
    _, layout, arena0, _ = build_state(cfg)
    res = run_local(cfg, log=lambda *a, **k: None)
    assert res["server"]["global_steps_completed"] > 0
    # reference parity (bn_sync off) leaves the server's running stats at their init values
    cfg2 = tiny_cfg(mode=mode, workers=workers, bn_sync=False, eval_every=0)
    from psx.parallel import runner as R

    srv_holder = {}
    orig = R.ParameterServer

    class Spy(orig):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            srv_holder["s"] = self

    R.ParameterServer = Spy
    try:
        R.run_local(cfg, log=lambda *a, **k: None)
        on = srv_holder["s"].arena[layout.param_numel:].clone()
        R.run_local(cfg2, log=lambda *a, **k: None)
        off = srv_holder["s"].arena[layout.param_numel:].clone()
    finally:
        R.ParameterServer = orig
    init = arena0[layout.param_numel:]
    assert torch.equal(off, init)
    assert not torch.equal(on, init)


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_dist_bn_sync_gloo(mode):
    recs, _ = _spawn(2, ["--mode", mode, "--bn-sync", "--topology", "dedicated" if mode == "sync" else "colocated"]
                     + TINY)
    assert len([r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]) == 1


def test_dist_async_gloo():
    recs, out = _spawn(3, ["--mode", "async", "--staleness-bound", "50"] + TINY)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"][0]
    wks = [r for r in recs if r["type"] == "WORKER_FINAL_METRICS"]
    assert len(wks) == 3
    total = sum(w["local_steps_completed"] for w in wks)
    assert srv["gradients_processed"] == total
    assert srv["global_steps_completed"] == srv["async_updates"] == total - srv["rejected_pushes"]
    assert sum(srv["staleness_histogram"]) == srv["async_updates"]


def test_fetch_codec_roundtrip_is_compute_exact():
    from psx.parallel.codec import FetchCodec

    torch.manual_seed(0)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, _ = lay.pack(m)
    arena += 0.001 * torch.randn_like(arena)
    c = FetchCodec(lay, "bf16conv")
    assert c.nbytes < 0.6 * arena.numel() * 4
    local = torch.zeros_like(arena)
    c.unpack(local, [w.clone() for w in c.pack(arena)])
    for name, e in lay.entries.items():
        if e.region == "counter":
            continue
        got, ref = lay.view(local, name), lay.view(arena, name)
        if e.region == "param" and len(e.shape) == 4:  # conv weight: the bf16 bits the engine uses
            assert torch.equal(got.to(torch.bfloat16), ref.to(torch.bfloat16)), name
        else:
            assert torch.equal(got, ref), name


def test_weight_wire_roundtrip_matches_fetch_codec():
    from psx.parallel.codec import FetchCodec, WeightWire, weight_image_enabled
    from psx.utils.config import PSConfig

    torch.manual_seed(0)
    m = TinyResNet(10)
    lay = ParamLayout.from_module(m)
    arena, _ = lay.pack(m)
    arena += 0.001 * torch.randn_like(arena)
    w = WeightWire(lay, "cpu")
    c = FetchCodec(lay, "bf16conv")
    assert w.nbytes - c.nbytes < 16  # same payload, one buffer (16-byte aligned image)
    w.publish_full(arena)
    a1, a2 = torch.zeros_like(arena), torch.zeros_like(arena)
    w.to_arena(a1)
    c.unpack(a2, [x.clone() for x in c.pack(arena)])
    assert torch.equal(a1, a2)
    # the remainder travels alone: a worker's local conv region is left untouched
    loc = torch.full_like(arena, 7.0)
    w.consume_small(loc)
    for name, e in lay.entries.items():
        if e.region == "counter":
            continue
        if e.region == "param" and len(e.shape) == 4:
            assert (lay.view(loc, name) == 7.0).all(), name
        else:
            assert torch.equal(lay.view(loc, name), lay.view(arena, name)), name
    ok = PSConfig(mode="sync", dtype="bf16").validate()
    assert ok.fetch_codec == "bf16conv" and weight_image_enabled(ok)
    assert PSConfig().validate().fetch_codec == "fp32"  # default: fp32 compute, fp32 fetch (reference)
    assert not weight_image_enabled(PSConfig(mode="sync").validate())
    for bad in (dict(mode="async"), dict(sync_steps=2), dict(codec="topk"), dict(fetch_codec="fp32"),
                dict(overlap=True)):
        assert not weight_image_enabled(PSConfig(dtype="bf16", **bad).validate()), bad
    with pytest.raises(ValueError):
        PSConfig(dtype="fp32", fetch_codec="bf16conv").validate()


@pytest.mark.parametrize("codec", ["fp32", "bf16conv"])
def test_dist_sync_fetch_codecs(codec):
    dt = ["--dtype", "bf16"] if codec == "bf16conv" else []  # bf16 conv weights = the bf16 compute path
    recs, _ = _spawn(2, ["--mode", "sync", "--fetch-codec", codec] + dt + TINY)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"][0]
    assert srv["global_steps_completed"] > 0


def test_plan_buckets_resnet18():
    from psx.models.resnet import ResNet18
    from psx.parallel.overlap import plan_buckets

    lay = ParamLayout.from_module(ResNet18(100))
    bk = plan_buckets(lay, 2 << 20)
    assert [b.keys[0] for b in bk] == ["fc", "layer4.0", "layer3.1", "layer2.1"]
    assert bk[-1].keys[-1] == "stem"
    # contiguous partition of the trainable prefix, in backward order
    assert bk[0].hi == lay.param_numel and bk[-1].lo == 0
    for a, b in zip(bk, bk[1:]):
        assert a.lo == b.hi
    assert sum(b.numel for b in bk) == lay.param_numel == 11_220_132
    one = plan_buckets(lay, 1 << 40)
    assert len(one) == 1 and one[0].numel == lay.param_numel


@pytest.mark.parametrize("extra", [[], ["--bucket-mb", "0.01"], ["--bucket-mb", "0.01", "--bn-sync"],
                                   ["--bucket-mb", "0.01", "--fetch-codec", "fp32", "--topology", "dedicated"],
                                   ["--bucket-mb", "0.01", "--codec", "fp16", "--topology", "dedicated"]])
def test_dist_sync_overlap_matches_serial(extra):
    """The bucketed/overlapped round must give exactly the serial round's parameters: both gather
    the wires to rank 0 and sum them in fp32 in worker order (per bucket range vs whole arena)."""
    outs = {}
    for ov in (True, False):
        d = os.path.join("/tmp", f"psx_ov_{os.getpid()}_{int(ov)}")
        args = (["--mode", "sync", "--codec", "none", "--ckpt-every", "1000", "--ckpt-dir", d] + TINY + extra
                + (["--overlap"] if ov else ["--no-overlap"]))
        recs, _ = _spawn(3, args)
        srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"][0]
        outs[ov] = srv
    assert outs[True]["global_steps_completed"] == outs[False]["global_steps_completed"] > 0
    assert outs[True]["final_param_checksum"] == pytest.approx(outs[False]["final_param_checksum"], rel=1e-6)


@pytest.mark.parametrize("codec", ["none", "fp16"])
def test_dist_sharded_server_matches_rank0_server(codec):
    """--topology sharded (parallel/sharded.py: reduce-scatter, per-rank range apply, all-gather
    of the bf16 image + fp32 remainder) ends in the rank-0 PS's parameters (3 ranks, gloo)."""
    outs = {}
    for topo in ("sharded", "colocated"):
        recs, _ = _spawn(3, ["--mode", "sync", "--codec", codec, "--topology", topo] + TINY)
        srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]
        assert len(srv) == 1
        outs[topo] = srv[0]
    assert outs["sharded"]["topology"] == "sharded"
    assert outs["sharded"]["global_steps_completed"] == outs["colocated"]["global_steps_completed"] > 0
    assert outs["sharded"]["gradients_processed"] == outs["colocated"]["gradients_processed"]
    # the gradient sums come from different collectives (gloo all-reduce vs reduce): their
    # rounding differs (fp32: ~1e-6 of the checksum after the run; fp16 sums: ~2e-5)
    assert outs["sharded"]["final_param_checksum"] == pytest.approx(outs["colocated"]["final_param_checksum"],
                                                                    rel=1e-5 if codec == "none" else 1e-4)


def test_shard_plan_covers_every_entry_once():
    from psx.models.resnet import ResNet18
    from psx.parallel.codec import small_index_of
    from psx.parallel.sharded import ShardPlan

    lay = ParamLayout.from_module(ResNet18(100))
    for world in (1, 2, 3, 8):
        p = ShardPlan(lay, world)
        assert p.chunk % 8 == 0 and p.padded >= lay.param_numel and p.lo[0] == 0 and p.hi[-1] == lay.param_numel
        assert all(a == b for a, b in zip(p.hi, p.lo[1:]))
        assert torch.equal(p.dst.sort().values, small_index_of(lay).sort().values)
        assert p.src.max().item() < world * p.S and len(set(p.src.tolist())) == p.src.numel()


@pytest.mark.parametrize("topology", ["colocated", "dedicated"])
def test_fault_restart_resumes_from_checkpoint(tmp_path, topology):
    """Worker 1 dies at its step 5; torchrun restarts the group, the server resumes from the
    last checkpoint (step 4) and workers skip the rounds it already contains, so the job ends
    with exactly the fault-free number of global steps."""
    ck = tmp_path / "ck"
    args = ["--mode", "sync", "--topology", topology, "--epochs", "2", "--ckpt-every", "2", "--ckpt-dir", str(ck),
            "--resume", "latest", "--fault-inject", "kill_worker:1@5", "--verbose", "1"]
    tiny = list(TINY)
    for opt in ("--epochs", "--verbose"):
        i = tiny.index(opt)
        del tiny[i:i + 2]
    recs, out = _spawn(3, args + tiny, max_restarts=1)
    assert "fault injected" in out and "[Resume] restored global step 4" in out
    W = 3 if topology == "colocated" else 2
    steps = -(-(96 // W + 96 % W) // 8)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]
    assert srv[-1]["global_steps_completed"] == 2 * steps


def test_scaling_harness_commands_and_efficiency():
    """bench/scaling.py: the per-N commands (torchrun on 127.0.0.1 for N > 1, as the driver runs
    them), the JSON-line parser and the weak-scaling efficiency."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("scaling", os.path.join(ROOT, "bench", "scaling.py"))
    S = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(S)
    c1 = S.command(1, 5, 2, ["--mode", "sync"])
    assert c1[1].endswith("bench.py") and "--gpus" in c1 and "torch.distributed.run" not in c1
    c8 = S.command(8, 5, 2, ["--mode", "sync"], port=29999)
    assert "torch.distributed.run" in c8 and "--nproc-per-node=8" in c8 and "127.0.0.1" in c8
    assert c8[c8.index("--gpus") + 1] == "8"
    out = 'noise\n{"metric": "m", "value": 100.0, "ms_per_step": 2.0, "unit": "images/s"}\ntrailer\n'
    assert S.parse_result(out)["value"] == 100.0
    eff = S.efficiency({1: {"value": 100.0}, 2: {"value": 190.0}, 8: {"value": 640.0}})
    assert eff == {1: 1.0, 2: 0.95, 8: 0.8}
    assert S.efficiency({2: {"value": 1.0}}) == {2: None}


def test_eval_workers_first_only_worker0_evaluates():
    """--eval-workers first (SURVEY.md §7.4 option): only worker 0 evaluates; default all."""
    res = run_local(tiny_cfg(mode="sync", workers=2, eval_workers="first"), log=lambda *a, **k: None)
    accs = [w["all_accuracies_percent"] for w in sorted(res["workers"], key=lambda w: w["worker_id"])]
    assert len(accs[0]) == 1 and accs[1] == []
    res = run_local(tiny_cfg(mode="sync", workers=2), log=lambda *a, **k: None)
    assert all(len(w["all_accuracies_percent"]) == 1 for w in res["workers"])


@pytest.mark.parametrize("topology", ["colocated", "dedicated"])
def test_sync_round_fp32_aggregation(topology):
    """gloo world 3: the server arena after one sync round equals the float64 average of the
    decoded fp16 pushes to fp32 rounding (the workers' wires are gathered and summed in fp32,
    not reduced in fp16)."""
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "helpers", "sync_agg_rank.py"),
           topology]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if "RESULT " in ln][0].split("RESULT ", 1)[1])
    assert res["gs"] == 1
    assert res["err"] < 1e-6, res  # fp32 rounding of the update only
    assert res["err_fp16_sum"] > 10 * res["err"], res  # what an fp16 running sum would have cost


def test_rounds_to_batches():
    from psx.parallel.worker import rounds_to_batches

    assert rounds_to_batches(0, 12, 2) == 0
    assert rounds_to_batches(3, 12, 2) == 6            # windows of 2: round r ends at batch 2r
    assert rounds_to_batches(7, 12, 2) == 12 + 2        # 6 rounds per epoch
    assert rounds_to_batches(4, 13, 3) == 12            # ceil(13/3) = 5 rounds per epoch (last window partial)
    assert rounds_to_batches(5, 13, 3) == 13            # epoch 1 fully done at its 5th round
    assert rounds_to_batches(6, 13, 3) == 13 + 3
    assert rounds_to_batches(5, 10, 1) == 5


@pytest.mark.parametrize("accumulate", [False, True])
def test_fault_restart_with_sync_steps_odd_checkpoint(tmp_path, accumulate):
    """--sync-steps 2 with a checkpoint every 3 rounds (odd): after the restart the workers skip
    exactly the batches of the checkpointed rounds, keep their window alignment, and the job
    ends with the fault-free number of rounds (no round re-run, no collective mismatch)."""
    ck = tmp_path / "ck"
    # the fault hits right after round 3: the window's first batch (reference rule, local step 5)
    # or its last (--accumulate, local step 6)
    fault = "kill_worker:1@6" if accumulate else "kill_worker:1@5"
    args = ["--mode", "sync", "--epochs", "2", "--sync-steps", "2", "--ckpt-every", "3", "--ckpt-dir", str(ck),
            "--resume", "latest", "--fault-inject", fault, "--verbose", "1"]
    if accumulate:
        args.append("--accumulate")
    tiny = list(TINY)
    for opt in ("--epochs", "--verbose"):
        i = tiny.index(opt)
        del tiny[i:i + 2]
    recs, out = _spawn(3, args + tiny, max_restarts=1)
    assert "fault injected" in out and "[Resume] restored global step 3" in out, out[-3000:]
    steps = -(-(96 // 3) // 8)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]
    assert srv[-1]["global_steps_completed"] == 2 * -(-steps // 2)


def test_hung_worker_watchdog_restart(tmp_path):
    """Liveness guard: worker 1 stalls (alive, no exit) at its step 5; the other ranks' round
    watchdogs see no sync round complete for --round-timeout seconds, exit with status 3, torchrun
    restarts the group and the job resumes from the last checkpoint to the fault-free number of
    global steps."""
    ck = tmp_path / "ck"
    args = ["--mode", "sync", "--epochs", "2", "--ckpt-every", "2", "--ckpt-dir", str(ck), "--resume", "latest",
            "--fault-inject", "hang_worker:1@5", "--round-timeout", "6", "--verbose", "1"]
    tiny = list(TINY)
    for opt in ("--epochs", "--verbose"):
        i = tiny.index(opt)
        del tiny[i:i + 2]
    recs, out = _spawn(3, args + tiny, max_restarts=1, timeout=300)
    assert "hangs at step 5" in out and "psx watchdog" in out and "[Resume] restored global step 4" in out, out[-3000:]
    steps = -(-(96 // 3) // 8)
    srv = [r for r in recs if r["type"] == "SERVER_FINAL_METRICS"]
    assert srv[-1]["global_steps_completed"] == 2 * steps


def test_overlap_auto_resolution():
    """--overlap auto (None): bucketed rounds with >= 2 ranks for dense sync rounds, never at N=1,
    with top-k payloads, --sync-steps > 1 or the sharded server; explicit flags win."""
    from psx.utils.config import PSConfig

    assert PSConfig(mode="sync").validate().resolve_overlap(8) is True
    assert PSConfig(mode="sync").validate().resolve_overlap(1) is False
    assert PSConfig(mode="async").validate().resolve_overlap(8) is False
    assert PSConfig(mode="sync", codec="topk").validate().resolve_overlap(8) is False
    assert PSConfig(mode="sync", sync_steps=2).validate().resolve_overlap(8) is False
    assert PSConfig(mode="sync", topology="sharded").validate().resolve_overlap(8) is False
    assert PSConfig(mode="sync", overlap=False).validate().resolve_overlap(8) is False
    assert PSConfig(mode="sync", overlap=True).validate().resolve_overlap(1) is True
