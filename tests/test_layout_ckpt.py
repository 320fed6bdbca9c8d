"""Parameter arena layout (reference state_dict parity) and checkpoint round trips — CPU."""
import torch

from psx.models.layout import ParamLayout
from psx.models.resnet import ResNet18, ResNet50, TinyResNet, build_model
from psx.utils import checkpoint as ckpt


def test_resnet18_layout_matches_reference_counts():
    m = ResNet18(100)
    lay = ParamLayout.from_module(m)
    s = lay.summary()
    # numbers measured on the reference model
    assert s["state_dict_entries"] == 122
    assert s["trainable_tensors"] == 62
    assert s["trainable_params"] == 11_220_132
    assert s["float_buffer_elems"] == 9_600
    assert s["int64_counters"] == 20
    assert s["grad_wire_bytes_fp16"] == 2 * 11_220_132
    names = list(m.state_dict().keys())
    assert list(lay.entries.keys()) == names
    assert "layer2.0.shortcut.0.weight" in names and "avg_pool" not in "".join(names)


def test_resnet50_layout():
    lay = ParamLayout.from_module(ResNet50(1000))
    assert lay.param_numel == 25_557_032


def test_pack_roundtrip_and_views():
    torch.manual_seed(0)
    m = TinyResNet(10)
    with torch.no_grad():
        m.bn1.running_mean.add_(0.5)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    sd = lay.to_state_dict(arena, counters)
    for k, v in m.state_dict().items():
        assert torch.equal(sd[k], v), k
        assert sd[k].dtype == v.dtype
    assert torch.equal(lay.view(arena, "fc.weight"), m.fc.weight)
    # trainable params form a prefix: the wire buffer is arena[:param_numel]
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.equal(arena[: lay.param_numel], flat)


def test_checkpoint_roundtrip_loads_into_reference_model(tmp_path):
    torch.manual_seed(1)
    m = build_model("resnet18", seed=3)
    lay = ParamLayout.from_module(m)
    arena, counters = lay.pack(m)
    arena[:10] += 1.0
    mom = torch.randn(lay.param_numel)
    p = ckpt.save(ckpt.path_for(str(tmp_path), 7), lay, arena, counters, 7, "sync", 4, 0.1, mom, "{}")
    assert ckpt.latest(str(tmp_path)) == p
    a2, c2, step, mom2, obj = ckpt.restore(p, lay)
    assert step == 7 and torch.equal(a2, arena) and torch.equal(mom2, mom)
    assert obj["format"] == "psx-ckpt-v1" and obj["mode"] == "sync"
    # the parameters dict is a plain reference-layout state_dict
    ref = ResNet18(100)
    ref.load_state_dict(obj["parameters"])
    assert torch.equal(ref.conv1.weight.reshape(-1)[:10], arena[:10])
