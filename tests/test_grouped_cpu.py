"""Worker batching on CPU: the grouped ResNet pass (k workers as one batch with
per-worker BatchNorm statistics and per-worker weight gradients) must equal k
separate standard forward/backward passes — gradients, losses and running
statistics — and the engine must train the same way with and without it."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.ops.grouped import GradSink
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches
from garfield_amd.parallel.grouped import GroupedResNet, supports
from garfield_amd.utils.flat import FlatParams


def _per_worker(model, xs, ys, k):
    model.train()
    grads, losses = [], []
    B = xs.shape[0] // k
    for g in range(k):
        model.zero_grad()
        loss = F.cross_entropy(model(xs[g * B:(g + 1) * B]), ys[g * B:(g + 1) * B])
        loss.backward()
        losses.append(loss.item())
        grads.append([p.grad.detach().clone() for p in model.parameters()])
    return grads, torch.tensor(losses, dtype=torch.float64)


@pytest.mark.parametrize("name", ["resnet18", "resnet50"])
def test_grouped_matches_separate_workers(name):
    """fp64 end to end, so the comparison is exact up to summation order (a deep
    BatchNorm net with 4-sample workers amplifies fp32 rounding to ~1e-3)."""
    torch.manual_seed(0)
    ref = build_model(name, 10).double()
    model = copy.deepcopy(ref).to(memory_format=torch.channels_last)
    k, B = 3, 4
    xs = torch.randn(k * B, 3, 32, 32, dtype=torch.float64)
    ys = torch.randint(0, 10, (k * B,))
    ref_grads, ref_losses = _per_worker(ref, xs, ys, k)

    flat = FlatParams(model, with_grad=False, dtype=torch.float64)
    X = torch.zeros(k, flat.ld, dtype=torch.float64)
    offsets = {id(p): o for p, o in zip(flat.params, flat.offsets)}
    ex = GroupedResNet(model, k, GradSink(X.view(-1), flat.ld, 0, offsets, k))
    losses = ex.run(xs.contiguous(memory_format=torch.channels_last), ys)

    assert torch.allclose(losses, ref_losses.double(), rtol=1e-10, atol=1e-12)
    for g in range(k):
        for v, r, p in zip(flat.views(X[g]), ref_grads[g], flat.params):
            assert v.shape == r.shape
            rel = ((v - r).norm() / r.norm().clamp_min(1e-30)).item()
            assert rel < 1e-9, (g, tuple(p.shape), rel)
    for m1, m2 in zip(ref.modules(), model.modules()):
        if isinstance(m1, nn.BatchNorm2d):
            assert torch.allclose(m1.running_mean, m2.running_mean, rtol=1e-10, atol=1e-12)
            assert torch.allclose(m1.running_var, m2.running_var, rtol=1e-10, atol=1e-12)


def test_supports():
    assert supports(build_model("resnet50", 10))
    assert supports(build_model("resnet18", 10))
    assert not supports(build_model("cifarnet"))
    assert not supports(build_model("mlp"))


@pytest.mark.parametrize("rule", ["average", "krum"])
def test_engine_worker_batching_matches_per_worker(rule):
    outs = []
    for wb in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar=rule, f=1, workers_per_rank=5, exchange_dtype=torch.float32, autocast_dtype=None,
                           worker_batching=wb, lr=0.05, byzantine={3: "reverse"} if rule == "krum" else {})
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(), cfg)
        assert (eng._gexec is not None) == wb
        b = synthetic_batches(5, 4, (3, 32, 32), 10, "cpu")
        losses = [float(eng.step(b)) for _ in range(2)]
        outs.append((eng.flat.reference_vector().clone(), losses, eng.last_weights))
    (p0, l0, w0), (p1, l1, w1) = outs
    assert l0 == pytest.approx(l1, rel=1e-4)
    rel = ((p0 - p1).norm() / p0.norm()).item()
    assert rel < 1e-3, rel  # fp32: the per-worker gradients agree to ~1e-3 (BN with 4-sample workers)
    if rule == "krum" and w0 is not None:
        assert torch.equal(w0, w1) and w1[3] == 0


def test_wgrad3x3_split_choice():
    """Pixel splits of the halo 3x3 weight gradient on the step's shapes (8 workers x 250 CIFAR images):
    the sweep's best S per ResNet-18 layer (profiles/r3/conv3x3/bench_conv3x3_shapes.log) and, on the
    small ResNet-50 layers, at least three 128-pixel tiles per split (profiles/r4/splits/)."""
    from garfield_amd.ops.grouped import _wgrad3x3_splits
    G = 8
    # (rows per worker, C, Cout) -> S
    cases = {(250 * 1024, 64, 64): 64, (250 * 256, 128, 128): 16, (250 * 64, 256, 256): 4,
             (250 * 16, 512, 512): 1, (250 * 64, 64, 64): 32, (250 * 16, 128, 128): 8}
    for (rows, c, co), want in cases.items():
        S = _wgrad3x3_splits(rows, (c // 64) * (co // 64) * G)
        assert S == want, (rows, c, co, S)
        assert S <= -(-rows // 128)


def test_masked_grad_materialize_applies_bits_in_memory_order():
    """MaskedGrad (the lazily masked residual gradient): bit i of byte j keeps element 8j + i of dy's
    channels_last memory order, as the BatchNorm forward writes its ReLU bits."""
    from garfield_amd.ops.grouped import MaskedGrad, rows2d

    torch.manual_seed(0)
    dy = torch.randn(2, 16, 3, 5).contiguous(memory_format=torch.channels_last)
    flat = rows2d(dy).reshape(-1)
    keep = torch.rand(flat.numel()) > 0.5
    w = (keep.view(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    out = MaskedGrad(dy, w).materialize()
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(rows2d(out).reshape(-1), torch.where(keep, flat, torch.zeros(())))


def test_largest_index_counts_activations_and_strided_columns():
    """Capacity accounting of the grouped step (meta-tensor forward): ResNet-50 ImageNet shape, the
    layer1 output (rows x 256 x 56 x 56) or layer2's stride-2 3x3 column matrix, whichever is larger."""
    from garfield_amd.parallel import grouped

    m = build_model("resnet50", 1000)
    for rows in (8, 4000):
        want = max(rows * 256 * 56 * 56, rows * 28 * 28 * 9 * 128)
        assert grouped.largest_index(m, rows, (3, 224, 224)) == want
    assert grouped.fits(m, 2000, (3, 224, 224)) and not grouped.fits(m, 4000, (3, 224, 224))


def test_oversized_grouped_step_routes_to_per_worker_path(monkeypatch):
    """A grouped step past the kernels' 32-bit indexing runs its workers one at a time (decided before
    any kernel runs, not a mid-step error): with the limit lowered below the job's size the engine
    steps like the per-worker engine (same math; its model is channels_last, so not bit for bit)."""
    from garfield_amd.parallel import grouped

    batches = synthetic_batches(5, 4, (3, 32, 32), 10, torch.device("cpu"))
    outs = []
    for wb in (True, False):
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(),
                                 EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.05, worker_batching=wb,
                                              exchange_dtype=torch.float32, autocast_dtype=None))
        if wb:
            assert eng._gexec is not None
            monkeypatch.setattr(grouped, "INDEX_LIMIT", grouped.largest_index(eng.model, 20, (3, 32, 32)) - 1)
            assert not eng._groupable(batches) and eng.grouped_inputs(4, (3, 32, 32)) is None
        for _ in range(2):
            eng.step(batches)
        outs.append(eng.flat.reference_vector().clone())
    assert ((outs[0] - outs[1]).norm() / outs[1].norm()).item() < 1e-3   # as test_engine_worker_batching_matches_per_worker
