"""The fp32 grouped-channel executor (parallel/grouped_fp32.py) against k independent fp32
workers run one after the other on the same model (per-worker losses, per-worker parameter
gradients in the exchange rows, and the k sequential running-statistics updates)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.ops.grouped import GradSink
from garfield_amd.parallel.grouped_fp32 import GroupedChannelResNet, supports


@pytest.mark.parametrize("name,G,B,hw", [("resnet18", 3, 2, 16), ("resnet50", 2, 2, 32)])
def test_grouped_channel_resnet_matches_sequential_workers(name, G, B, hw):
    torch.manual_seed(0)
    model = build_model(name, num_classes=10).double()
    assert supports(model)
    ref = copy.deepcopy(model)
    params = list(model.parameters())
    offsets, off = {}, 0
    for p in params:
        offsets[id(p)] = off
        off += p.numel()
    d = off
    flat = torch.zeros(G * d, dtype=torch.float64)
    sink = GradSink(flat, d, 0, offsets, G)
    ex = GroupedChannelResNet(model, G, sink)
    x = torch.randn(G * B, 3, hw, hw, dtype=torch.float64)
    y = torch.randint(0, 10, (G * B,))
    losses = ex.run(x, y)

    ref.train()
    rparams = list(ref.parameters())
    for g in range(G):
        out = ref(x[g * B:(g + 1) * B])
        loss = F.cross_entropy(out, y[g * B:(g + 1) * B])
        grads = torch.autograd.grad(loss, rparams)
        assert abs(float(loss) - float(losses[g])) < 1e-8
        expect = torch.cat([gr.reshape(-1) for gr in grads])
        got = flat.view(G, d)[g]
        assert ((got - expect).norm() / expect.norm()).item() < 1e-6, g   # (B=2 at 1x1: ill-conditioned BN)
    for (n1, b1), (n2, b2) in zip(model.named_buffers(), ref.named_buffers()):
        if b1.dtype.is_floating_point:
            assert torch.allclose(b1, b2, rtol=1e-8, atol=1e-10), n1
