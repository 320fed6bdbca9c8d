"""Baseline trainer on the HIP engine: fused SGD-momentum kernel vs torch.optim.SGD, and a short
ResNet-18 run whose training loss falls."""
import pytest
import torch

from psx import baseline as BL
from psx.ops import kernels as K

pytestmark = pytest.mark.gpu


def test_sgd_momentum_kernel_matches_torch():
    torch.manual_seed(0)
    n = 1_000_003
    p = torch.randn(n, device="cuda")
    buf = torch.zeros(n, device="cuda")
    ref = torch.nn.Parameter(p.clone())
    opt = torch.optim.SGD([ref], lr=0.05, momentum=0.9, weight_decay=5e-4)
    for i in range(3):
        g = torch.randn(n, device="cuda")
        K.sgd_apply(p, g, 0.05, momentum=0.9, wd=5e-4, buf=buf, first=i == 0)
        ref.grad = g.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, ref.detach(), atol=1e-5)


def test_baseline_resnet18_loss_falls():
    from psx.utils.data import DeviceDataset

    tr = BL.BaselineTrainer("resnet18", batch=128, device="cuda", log=lambda *a: None)
    train = DeviceDataset.synthetic(4096, 32, 100, seed=0, device="cuda")
    test = DeviceDataset.synthetic(1024, 32, 100, seed=0, device="cuda", offset=10_000_000)
    m = tr.fit(train, test, epochs=3)
    assert m.train_losses[-1] < m.train_losses[0]
    assert m.test_accuracies[-1] > 5.0  # well above 1% chance on the synthetic task
