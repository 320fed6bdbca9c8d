"""Single-process baseline trainer (psx.baseline; reference baseline/baseline_training.py)."""
import json
import os

import pytest
import torch

from psx import baseline as BL


def test_multistep_lr_matches_torch():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.1)
    ref = torch.optim.lr_scheduler.MultiStepLR(opt, milestones=[10, 15], gamma=0.1)
    ours = BL.MultiStepLR(0.1, (10, 15), 0.1)
    for _ in range(20):
        assert ours.lr == pytest.approx(opt.param_groups[0]["lr"])
        opt.step()
        ref.step()
        ours.step()


def test_cpu_sgd_step_matches_torch_sgd():
    torch.manual_seed(0)
    tr = BL.BaselineTrainer("resnet_tiny", batch=8, device="cpu", use_graph=False, log=lambda *a: None)
    p0 = tr.params.clone()
    ref = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([ref], lr=0.1, momentum=0.9, weight_decay=5e-4)
    for _ in range(3):
        g = torch.randn_like(p0)
        tr.compute.grads[: tr.n] = g
        tr._sgd_step()
        ref.grad = g.clone()
        opt.step()
    assert torch.allclose(tr.params, ref.detach(), atol=1e-6)


def test_baseline_main_cpu(tmp_path, capsys):
    out = tmp_path / "res"
    res = BL.main(["--model", "resnet_tiny", "--epochs", "2", "--batch-size", "16", "--train-samples", "64",
                   "--test-samples", "32", "--cpu", "--out-dir", str(out), "--no-graph"])
    assert len(res["test_accuracies"]) == 2 and res["model_parameters"] > 0
    s = json.load(open(out / "baseline_summary.json"))
    assert s["epochs"] == 2 and "final_accuracy" in s
    assert (out / "baseline_results.png").exists()
    assert "METRICS_JSON" in capsys.readouterr().out
