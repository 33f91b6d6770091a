"""Model zoo parity: every ``select_model`` name builds a model whose parameter list
(count and per-tensor shapes, in registration order) equals the reference model's,
so a reference flat vector (``server.py:196-200``, the interchange/checkpoint layout)
loads into it. The digests are SHA-1 prefixes of ``repr([tuple(p.shape) for p in
model.parameters()])`` of the reference definitions in
``pytorch_impl/libs/garfieldpp/models/*.py`` (num_classes 10; pimanet 1), computed
once from those files. ``shufflenetg2`` is not pinned: the reference's own
constructor fails under current torch (parity unpinned)."""
import hashlib

import pytest
import torch

from garfield_amd.models import build_model

REFERENCE = {
    "preactresnet18": (11171146, "b85b158a6e8da794"), "googlenet": (6166250, "0be5dcb0c06759cc"),
    "densenet121": (6956298, "1390ef7f2e50b4b7"), "resnext29": (9128778, "f78814927d84a7a1"),
    "mobilenet": (3217226, "69700f2a0b568ebb"), "mobilenetv2": (2296922, "5cbaf5d86e08f026"),
    "dpn92": (34236634, "55e496389ac378ff"), "senet18": (11260354, "5fb6346ca6db3314"),
    "efficientnetb0": (3599686, "0f61a839bc5ab740"), "regnetx200": (2321946, "630e31e9d444f350"),
    "resnet18": (11173962, "b33a36854ce89033"), "cifarnet": (62006, "13e7742d2b713760"),
    "convnet": (21840, "771bacf045244762"), "cnn": (5852170, "ab71b8f9f2895eaf"),
    "pimanet": (4801, "6410902c1b7c3589"),
}


@pytest.mark.parametrize("name", sorted(REFERENCE))
def test_parameter_list_matches_reference(name):
    count, digest = REFERENCE[name]
    m = build_model(name, num_classes=1 if name == "pimanet" else 10)
    shapes = [tuple(p.shape) for p in m.parameters()]
    assert sum(p.numel() for p in m.parameters()) == count
    assert hashlib.sha1(repr(shapes).encode()).hexdigest()[:16] == digest


def test_resnet50_torchvision_layout():
    """``resnet50`` is torchvision's architecture in the reference (10 classes: SURVEY §2.1)."""
    m = build_model("resnet50", num_classes=10)
    assert sum(p.numel() for p in m.parameters()) == 23528522
    assert len(list(m.parameters())) == 161


@pytest.mark.parametrize("name", ["preactresnet18", "senet18", "googlenet", "efficientnetb0"])
def test_fixed_models_run_and_backprop(name):
    m = build_model(name, num_classes=10)
    y = m(torch.randn(2, 3, 32, 32))
    y.sum().backward()
    assert y.shape == (2, 10) and m.linear.weight.grad is not None
