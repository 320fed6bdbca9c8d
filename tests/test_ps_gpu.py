"""Parameter-server runs on one MI355X through the HIP engine (loopback runner)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

from psx.parallel.runner import run_local  # noqa: E402
from psx.utils import metrics as M  # noqa: E402
from psx.utils.config import PSConfig  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cfg(**kw):
    base = dict(model="resnet18", batch_size=128, epochs=1, train_samples=4096, test_samples=1024, eval_every=1,
                verbose=0, lr=0.1)
    base.update(kw)
    return PSConfig(**base).validate()


def test_sync_single_worker_loss_decreases(capsys):
    c = cfg(mode="sync", workers=1, epochs=3, train_samples=6400, eval_every=3, bn_sync=True)
    res = run_local(c, log=lambda *a, **k: None)
    recs = M.parse_lines(capsys.readouterr().out.splitlines())
    w = [r for r in recs if r["type"] == "WORKER_FINAL_METRICS"][0]
    assert res["server"]["global_steps_completed"] == 3 * 50
    # learnable synthetic data: accuracy well above chance (1 %) after 150 steps
    assert w["final_test_accuracy_percent"] > 5.0, w
    assert w["images_per_second"] > 1000


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_two_simulated_workers(mode, capsys):
    c = cfg(mode=mode, workers=2, max_steps=8, eval_every=0)
    res = run_local(c, log=lambda *a, **k: None)
    s = res["server"]
    assert s["gradients_processed"] == 16
    if mode == "async":
        assert s["global_steps_completed"] == 16 and s["max_staleness_observed"] == 1
    else:
        assert s["global_steps_completed"] == 8


def test_bench_contract_single_gpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "2"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["steps"] == 5 and rec["value"] > 0
    assert torch.cuda.is_available()
