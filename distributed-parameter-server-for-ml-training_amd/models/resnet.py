"""PyTorch reference models (numerics oracle, CPU path, and state_dict layout source).

``ResNet18`` is the CIFAR-style ResNet-18 the reference trains (reference:
src/parameter_server/server.py:20-76; byte-identical copies in src/workers/worker.py:20-76 and
baseline/baseline_training.py:37-95): 3x3 stride-1 stem without max-pool, four stages of two
BasicBlocks (64/128/256/512), global average pool, Linear(512 -> classes). Module names are kept
identical so ``state_dict()`` keys match the reference wire/checkpoint layout exactly
(122 entries, 11,220,132 trainable parameters for 100 classes).

``ResNet50`` is the ImageNet-shape bottleneck network required by the BASELINE.json top-k
configuration (torchvision naming: conv1/bn1/layerN.i.convK/bnK/downsample.{0,1}/fc).

These modules are the *reference* implementation used by the CPU test-suite and by the
numerics tests of the HIP engine (models/engine.py), which runs the same networks on
hand-written CDNA4 kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        # the reference names the projection shortcut "shortcut" (server.py:28-32)
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        else:
            self.shortcut = nn.Sequential()

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return F.relu(y + self.shortcut(x))


class ResNet18(nn.Module):
    """CIFAR ResNet-18 with the reference's module names."""

    def __init__(self, num_classes: int = 100):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        widths, strides = (64, 128, 256, 512), (1, 2, 2, 2)
        cin = 64
        for i, (w, s) in enumerate(zip(widths, strides)):
            blocks = [BasicBlock(cin, w, s), BasicBlock(w, w, 1)]
            cin = w
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, num_classes)

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        for i in range(4):
            x = getattr(self, f"layer{i + 1}")(x)
        x = torch.flatten(self.avg_pool(x), 1)
        return self.fc(x)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, 1, 0, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)  # torchvision v1.5 stride placement
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, 1, 0, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        y = F.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        sc = x if self.downsample is None else self.downsample(x)
        return F.relu(y + sc)


class ResNet50(nn.Module):
    """ImageNet-shape ResNet-50 (torchvision layer naming)."""

    def __init__(self, num_classes: int = 1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin = 64
        for i, (w, n, s) in enumerate(zip((64, 128, 256, 512), (3, 4, 6, 3), (1, 2, 2, 2))):
            blocks = []
            for j in range(n):
                blocks.append(Bottleneck(cin, w, s if j == 0 else 1))
                cin = w * 4
            setattr(self, f"layer{i + 1}", nn.Sequential(*blocks))
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.maxpool(F.relu(self.bn1(self.conv1(x))))
        for i in range(4):
            x = getattr(self, f"layer{i + 1}")(x)
        return self.fc(torch.flatten(self.avgpool(x), 1))


class TinyResNet(ResNet18):
    """Same module names/structure family as ResNet18 (one BasicBlock per stage, widths
    8/16/32/64) — a seconds-per-step model for the CPU test-suite only."""

    def __init__(self, num_classes: int = 10):
        nn.Module.__init__(self)
        self.conv1 = nn.Conv2d(3, 8, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(8)
        cin = 8
        for i, (w, s) in enumerate(zip((8, 16, 32, 64), (1, 2, 2, 2))):
            setattr(self, f"layer{i + 1}", nn.Sequential(BasicBlock(cin, w, s)))
            cin = w
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(64, num_classes)


MODELS = {"resnet18": ResNet18, "resnet50": ResNet50, "resnet_tiny": TinyResNet}

# input geometry per model: (channels, height, width), default classes
MODEL_INPUT = {"resnet18": ((3, 32, 32), 100), "resnet50": ((3, 224, 224), 1000), "resnet_tiny": ((3, 32, 32), 10)}


def build_model(name: str, num_classes: int | None = None, seed: int | None = 0) -> nn.Module:
    if name not in MODELS:
        raise ValueError(f"unknown model {name!r}; choose from {sorted(MODELS)}")
    if seed is not None:
        torch.manual_seed(seed)
    nc = num_classes if num_classes is not None else MODEL_INPUT[name][1]
    return MODELS[name](num_classes=nc)
