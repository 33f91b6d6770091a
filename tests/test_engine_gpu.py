"""Single-GPU robust training engine (native HIP path) — one process, n logical workers."""
import os

import pytest
import torch
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rule,f,k", [("krum", 2, 8), ("bulyan", 1, 8), ("median", 1, 8), ("trimmed-mean", 2, 8),
                                      ("average", 0, 4), ("aksel", 2, 8), ("brute", 2, 8), ("condense", 1, 8),
                                      ("averaged-median", 2, 8), ("average-nan", 0, 4)])
def test_engine_step_all_rules(cuda, rule, f, k):
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("cifarnet"), F.cross_entropy, DistContext(device=cuda),
                             EngineConfig(gar=rule, f=max(f, 1), workers_per_rank=k))
    batches = synthetic_batches(k, 8, (3, 32, 32), 10, cuda)
    before = eng.flat_model().clone()
    loss = eng.step(batches)
    torch.cuda.synchronize()
    assert torch.isfinite(loss)
    after = eng.flat_model()
    assert torch.isfinite(after).all()
    assert not torch.equal(before, after)


def test_engine_krum_excludes_attackers_and_trains(cuda):
    torch.manual_seed(0)
    cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.05, byzantine={2: "reverse", 5: "random"},
                       weight_decay=0.0)
    eng = RobustDataParallel(build_model("cifarnet"), F.cross_entropy, DistContext(device=cuda), cfg)
    batches = synthetic_batches(8, 32, (3, 32, 32), 10, cuda)
    losses = [float(eng.step(batches)) for _ in range(15)]
    w = eng.last_weights.cpu()
    assert w[2] == 0 and w[5] == 0
    assert losses[-1] < losses[0]


def test_engine_matches_reference_sgd_on_average(cuda):
    """average GAR + fused SGD == mean gradient + torch SGD (fp32 exchange, no autocast)."""
    torch.manual_seed(0)
    m1 = build_model("cifarnet")
    m2 = build_model("cifarnet")
    m2.load_state_dict(m1.state_dict())
    k = 4
    cfg = EngineConfig(gar="average", f=1, workers_per_rank=k, lr=0.1, momentum=0.9, weight_decay=5e-4,
                       exchange_dtype=torch.float32, autocast_dtype=None)
    eng = RobustDataParallel(m1, F.cross_entropy, DistContext(device=cuda), cfg)
    m2 = m2.to(cuda)
    opt = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    batches = synthetic_batches(k, 16, (3, 32, 32), 10, cuda)
    for _ in range(2):
        eng.step(batches)
        opt.zero_grad()
        grads = []
        for x, y in batches:
            m2.zero_grad()
            F.cross_entropy(m2(x), y).backward()
            grads.append(torch.cat([p.grad.reshape(-1) for p in m2.parameters()]).clone())
        g = torch.stack(grads).mean(0)
        pos = 0
        for p in m2.parameters():
            p.grad = g[pos:pos + p.numel()].view_as(p).clone()
            pos += p.numel()
        opt.step()
    flat2 = torch.cat([p.detach().reshape(-1) for p in m2.parameters()])
    assert torch.allclose(eng.flat_model(), flat2, atol=2e-4, rtol=1e-3)


def test_engine_channels_last_matches_nchw(cuda):
    """channels_last changes only the memory order of the flat buffer, not the training math."""
    outs = []
    for cl in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar="average", f=1, workers_per_rank=5, exchange_dtype=torch.float32,
                           autocast_dtype=None, channels_last=cl)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        b = synthetic_batches(5, 4, (3, 32, 32), 10, cuda, channels_last=cl)
        for _ in range(2):
            eng.step(b)
        outs.append(eng.flat.reference_vector())
    # NCHW and NHWC convolutions use different MIOpen algorithms (accumulation order,
    # Winograd): compare the whole parameter vector in relative norm
    rel = ((outs[0] - outs[1]).norm() / outs[0].norm()).item()
    assert rel < 1e-3, rel


@pytest.mark.parametrize("rule", ["krum", "median"])
def test_engine_cuda_graph_matches_eager(cuda, rule):
    """Per-worker HIP-graph replay == eager steps (same math, fewer launches).

    MIOpen's split-K weight-gradient kernels are not bitwise deterministic, so the
    graph run is compared against the eager run-to-run noise floor."""
    outs = []
    for graph in (False, False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar=rule, f=1, workers_per_rank=5, cuda_graph=graph, byzantine={4: "reverse"}, lr=1e-3,
                           worker_batching=False)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        b = synthetic_batches(5, 8, (3, 32, 32), 10, cuda)
        init = eng.flat.reference_vector().clone()
        for _ in range(3):
            eng.step(b)
        if graph:
            assert eng._graph is not None and not eng._graph_failed
        outs.append(eng.flat.reference_vector().clone() - init)   # the accumulated update
    noise = ((outs[0] - outs[1]).norm() / outs[0].norm()).item()
    rel = ((outs[0] - outs[2]).norm() / outs[0].norm()).item()
    assert rel < max(10 * noise, 1e-3), (rel, noise)


@pytest.mark.parametrize("rule,f", [("krum", 2), ("median", 1), ("bulyan", 1), ("aksel", 2), ("brute", 2),
                                    ("average", 0), ("trimmed-mean", 2)])
def test_sharded_gpu_path_single_rank_matches(cuda, rule, f):
    """The sharded aggregation's GPU code (row-list GAR on the shard, Gram all-reduce,
    fused update of the master shard, working-weight refresh) with identity
    collectives on one rank == the redundant path."""
    outs = []
    for shard in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar=rule, f=max(f, 1), workers_per_rank=8, shard_gar=shard,
                           byzantine={} if rule == "average" else {3: "reverse"}, lr=0.01)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        assert (eng._shard is not None) == shard
        b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda)
        for _ in range(3):
            eng.step(b)
        torch.cuda.synchronize()
        outs.append((eng.flat.reference_vector().clone(), eng.last_weights))
    (p0, w0), (p1, w1) = outs
    rel = ((p1 - p0).norm() / p0.norm()).item()
    assert rel < 1e-5, rel
    if w0 is not None:
        assert torch.equal(w0.cpu(), w1.cpu())


@pytest.mark.gpu
def test_cuda_graph_never_writes_loader_tensors(cuda):
    """Per-worker HIP-graph path fed by DeviceLoaders with a short last batch: the
    engine copies into its OWN static inputs (the loader's label/input views stay
    untouched) and a batch of another shape runs eagerly instead of failing."""
    from garfield_amd.data.datasets import DeviceLoader, TensorDataset

    torch.manual_seed(0)
    k = 3
    ds = TensorDataset(torch.randn(10 * k, 3, 32, 32), torch.randint(0, 10, (10 * k,)))
    loaders = [DeviceLoader(ds, range(10 * j, 10 * (j + 1)), 4, cuda) for j in range(k)]   # 4, 4, 2
    y0 = [ld.y.clone() for ld in loaders]
    x0 = [ld.x.clone() for ld in loaders]
    cfg = EngineConfig(gar="median", f=1, workers_per_rank=k, cuda_graph=True, worker_batching=False, lr=1e-3)
    eng = RobustDataParallel(build_model("cifarnet"), F.cross_entropy, DistContext(device=cuda), cfg)
    for it in range(2 * len(loaders[0])):
        loss = eng.step([ld[it] for ld in loaders])
        assert torch.isfinite(loss).item()
    torch.cuda.synchronize()
    assert eng._graph is not None
    for ld, y, x in zip(loaders, y0, x0):
        assert torch.equal(ld.y, y) and torch.equal(ld.x, x)


@pytest.mark.gpu
@pytest.mark.parametrize("rule,f,overlap", [("krum", 2, "1"), ("median", 1, "1"), ("bulyan", 1, "1"),
                                            ("krum", 2, "0")])
def test_bucketed_exchange_overlap_loopback(cuda, rule, f, overlap, monkeypatch):
    """Sharded aggregation with layer buckets on one rank and the exchange machinery of a
    multi-rank step (GARFIELD_LOOPBACK_EXCHANGE=1: comm stream, bucket signals recorded by
    the HIP-graph backward, per-bucket events), with the next forward replayed as three
    graphs cut at the bucket boundaries: the layer3/layer4 updates run on the comm stream
    beside the next step's stem-to-layer2 stage, and each later stage waits for its bucket.
    Fresh inputs every step, so a stage that ran before its weights were updated, or an
    update that read rows the next backward had already overwritten, would change the
    result. Must equal the redundant (unsharded) path."""
    monkeypatch.setenv("GARFIELD_LOOPBACK_EXCHANGE", "1")
    monkeypatch.setenv("GARFIELD_OVERLAP", overlap)     # in-graph bucket signals, or after the backward
    outs = []
    for shard in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar=rule, f=f, workers_per_rank=8, shard_gar=shard, byzantine={5: "reverse"}, lr=0.01,
                           cuda_graph=True)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        if shard:
            assert eng._gexec is not None and len(eng._shard.buckets) == 3
            assert (eng._gexec.mark_events() is not None) == (overlap == "1")
        for it in range(4):
            b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda, seed=100 + it)
            eng.step(b)
        torch.cuda.synchronize()
        if shard:
            assert isinstance(eng._ggraph, list) and len(eng._ggraph) == 3 and eng._shard.staged
        outs.append(eng.flat.reference_vector().clone())
    rel = ((outs[1] - outs[0]).norm() / outs[0].norm()).item()
    assert rel < 1e-5, rel


@pytest.mark.gpu
def test_layerwise_krum_on_gpu_matches_per_segment_gar(cuda):
    """Layer-wise Krum on the GPU path (grouped ResNet-18 rows, HIP GAR per parameter
    segment): the update equals the per-segment HIP Krum selection of the same rows, combined
    in fp32."""
    from garfield_amd.ops import gar

    torch.manual_seed(0)
    cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, byzantine={3: "reverse"}, lr=0.1, momentum=0.0,
                       weight_decay=0.0, layerwise=True, cuda_graph=False)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
    b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda)
    before = eng.flat.data[: eng.d].clone()
    eng.step(b)
    torch.cuda.synchronize()
    expect = torch.empty(eng.d, dtype=torch.float32, device=cuda)
    for off, numel in zip(eng.flat.offsets, eng.flat.numels):
        seg = eng.G[:, off:off + numel]
        w = gar.krum_weights(seg, 2)
        expect[off:off + numel] = (w[:, None] * seg.float()).sum(0)    # combined in fp32
    got = (before - eng.flat.data[: eng.d]) / 0.1
    assert ((got - expect).norm() / expect.norm()).item() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("model,n,steps", [("resnet18", 8, 2), ("resnet50", 16, 1)])
def test_layerwise_krum_device_equals_segment_loop_bitwise(cuda, monkeypatch, model, n, steps):
    """Layer-wise Krum as device operations (segmented Gram, batched selection, segmented
    combine + SGD) against the per-segment loop (HIP Krum weights of each segment's rows, an fp32
    HIP combine per segment, then the fused update). The two Grams are summed in different
    orders, so a segment whose Krum scores TIE at the selection boundary (honest iid workers,
    n = 16) may select differently: every segment whose weights differ must be such a near-tie
    (fp64 scores of the m-th and (m+1)-th best within 1e-4 relative), and every other segment's
    parameters and momentum agree to fp32 rounding (bit for bit on the n = 8 ResNet-18 case, two
    steps)."""
    import garfield_amd.parallel.engine as E

    outs = []
    f = 2
    for dev_path in (False, True):
        monkeypatch.setattr(E, "LW_DEVICE", dev_path)
        torch.manual_seed(0)
        cfg = EngineConfig(gar="krum", f=f, workers_per_rank=n, byzantine={3: "reverse"}, lr=0.05, momentum=0.9,
                           weight_decay=5e-4, layerwise=True, cuda_graph=False)
        eng = RobustDataParallel(build_model(model), F.cross_entropy, DistContext(device=cuda), cfg)
        for it in range(steps):
            eng.step(synthetic_batches(n, 4, (3, 32, 32), 10, cuda, seed=7 + it))
        torch.cuda.synchronize()
        outs.append((eng.flat.data[: eng.d].clone(), eng.mom[: eng.d].clone(), eng.last_weights.clone(),
                     eng.G[:, : eng.d].clone()))
    (p0, m0, w0, G0), (p1, m1, w1, G1) = outs
    segs = sorted(zip(eng.flat.offsets, eng.flat.numels))
    assert w0.shape == w1.shape == (len(segs), n)
    assert float(w1[:, 3].abs().max()) == 0.0          # the reversed gradient is never selected
    assert torch.equal(G0, G1)                          # the same gradient rows reached the GAR
    m = n - f - 2
    differ = [s for s in range(len(segs)) if not torch.equal(w0[s], w1[s])]
    for s in differ:
        off, numel = segs[s]
        X = G1[:, off:off + numel].double()
        D = torch.cdist(X, X) ** 2
        D.fill_diagonal_(float("inf"))
        score = D.sort(1).values[:, : n - f - 2].sum(1).sort().values
        assert (score[m] - score[m - 1]).abs() <= 1e-4 * score[m - 1].abs(), (s, score[m - 1:m + 1])
    if steps == 1:
        assert len(differ) <= len(segs) // 10
        for s, (off, numel) in enumerate(segs):
            if s not in differ:      # same selection: equal up to fp32 rounding of 12-row sums
                for a0, a1 in ((p0, p1), (m0, m1)):
                    x0, x1 = a0[off:off + numel].double(), a1[off:off + numel].double()
                    assert ((x0 - x1).norm() / x0.norm().clamp_min(1e-30)).item() < 1e-6, s
    else:
        assert not differ
        assert torch.equal(p0, p1) and torch.equal(m0, m1)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_fp32_grouped_path_matches_per_worker_engine(cuda, graph):
    """fp32 (the reference's precision) with worker batching: the grouped NHWC executor on the
    fp32 kernels (conv_f32.hip split-bf16 MFMA, bn_nhwc.hip in fp32) against the per-worker fp32
    engine. The two run different convolution algorithms (fp32 rounding differs by ~1e-3 of a
    gradient), so: the first update within 2e-2 and the parameters within 2e-3 after 3 averaged
    steps (reference layout), HIP-graph replays included. The exact grouped math is checked in
    fp64 on the CPU (tests/test_grouped_cpu.py)."""
    outs, deltas = [], []
    for wb in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar="average", f=0, workers_per_rank=8, lr=0.05, momentum=0.9, weight_decay=5e-4,
                           autocast_dtype=None, lp_weights=False, worker_batching=wb, cuda_graph=graph,
                           exchange_dtype=torch.float32)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        assert (eng._gexec is not None) == wb
        p0 = eng.flat.reference_vector().clone()     # reference layout: both engines comparable
        for it in range(3):
            eng.step(synthetic_batches(8, 8, (3, 32, 32), 10, cuda, seed=40 + it))
            if it == 0:
                deltas.append(eng.flat.reference_vector() - p0)
        torch.cuda.synchronize()
        if wb and graph:
            assert eng._ggraph is not None        # batched library GEMMs: replay-safe
        outs.append(eng.flat.reference_vector().clone())
    rel = ((deltas[1] - deltas[0]).norm() / deltas[0].norm()).item()     # the first update
    assert rel < 2e-2, rel
    rel = ((outs[1] - outs[0]).norm() / outs[0].norm()).item()
    assert rel < 2e-3, rel


@pytest.mark.gpu
@pytest.mark.parametrize("rule,f", [("krum", 2), ("bulyan", 1), ("brute", 2), ("aksel", 2)])
def test_sharded_layerwise_matches_unsharded_on_gpu(cuda, rule, f):
    """Layer-wise rules through the sharded aggregator (one rank: per-bucket segment Grams over the
    owned ranges -- Aksel: per-segment distances to the median --, batched selection, per-bucket
    segmented combine / Bulyan tail) equal the unsharded path: same per-segment weights,
    parameters to fp32 rounding."""
    outs = []
    for shard in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar=rule, f=f, workers_per_rank=8, byzantine={3: "reverse"}, lr=0.05, momentum=0.9,
                           weight_decay=5e-4, layerwise=True, shard_gar=shard, cuda_graph=False)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
        assert (eng._shard is not None) == shard
        eng.step(synthetic_batches(8, 4, (3, 32, 32), 10, cuda, seed=3))
        torch.cuda.synchronize()
        w = eng.last_weights
        outs.append((eng.flat.reference_vector().clone(), w.clone() if w is not None else None))
    (p0, w0), (p1, w1) = outs
    if rule != "bulyan":
        assert w0.shape == w1.shape and torch.equal(w0.float(), w1.float())
    rel = ((p1 - p0).norm() / p0.norm()).item()
    assert rel < 1e-6, rel


@pytest.mark.gpu
def test_layerwise_bulyan_device_matches_per_segment_rule(cuda):
    """Layer-wise Bulyan on device (segmented Gram, the t selections of every segment in one
    batched launch, one segmented tail launch) == per segment: the HIP Bulyan selection W of the
    segment's rows, V = W · rows in fp32, the averaged median of V (beta = t - 2f)."""
    from garfield_amd.ops import gar

    torch.manual_seed(0)
    n, f = 16, 3
    cfg = EngineConfig(gar="bulyan", f=f, workers_per_rank=n, byzantine={3: "reverse", 9: "reverse"}, lr=0.1,
                       momentum=0.0, weight_decay=0.0, layerwise=True, cuda_graph=False)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
    b = synthetic_batches(n, 4, (3, 32, 32), 10, cuda)
    eng.step(b)
    torch.cuda.synchronize()
    t = n - 2 * f - 2
    expect = torch.empty(eng.d, dtype=torch.float32, device=cuda)
    for off, numel in zip(eng.flat.offsets, eng.flat.numels):
        seg = eng.G[:, off:off + numel]
        W = gar.bulyan_weights(seg, f).float()
        assert float(W[:, 3].abs().max()) == 0.0 and float(W[:, 9].abs().max()) == 0.0
        expect[off:off + numel] = gar._torch_closest_mean(W.double() @ seg.double(), t - 2 * f).float()
    got = eng._gagg[: eng.d]                      # the device path's fp32 aggregate
    # fp32 selection means (device) vs fp64 ones: a coordinate whose beta-th and (beta+1)-th closest
    # means are within rounding may average a different set -- two means on opposite sides of the
    # median at (nearly) the same distance, so the two choices differ by ~2|v - med| / beta (a few
    # coordinates in 1e5 carry most of the norm difference); every other coordinate agrees to rounding
    err = (got - expect).abs()
    bad = (err > 1e-5 * expect.abs() + 1e-6 * expect.abs().mean()).float().mean().item()
    print("layer-wise bulyan: fraction of coordinates off by more than rounding", bad,
          "max err", err.max().item(), "rel norm", (err.norm() / expect.norm()).item())
    assert bad < 1e-3
    assert (err.norm() / expect.norm()).item() < 5e-3


@pytest.mark.gpu
def test_byzps_one_gpu_grouped_matches_plain_engine(cuda):
    """Byzantine-server mode on one GPU (the rank is a server replica hosting its workers,
    MAR median over one model = identity): the grouped HIP-graph worker path runs and the
    parameters equal the plain engine's after 3 steps."""
    from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig

    outs = []
    for byzps in (False, True):
        torch.manual_seed(0)
        kw = dict(gar="krum", f=2, workers_per_rank=8, byzantine={6: "reverse"}, lr=0.01, cuda_graph=True)
        model = build_model("resnet18")
        if byzps:
            eng = ByzantinePSDataParallel(model, F.cross_entropy, DistContext(device=cuda),
                                          ByzPSConfig(num_ps=1, fps=0, mar="median", ps_workers=True, **kw))
            assert eng._gexec is not None
        else:
            eng = RobustDataParallel(model, F.cross_entropy, DistContext(device=cuda), EngineConfig(**kw))
        b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda)
        for _ in range(3):
            eng.step(b)
        torch.cuda.synchronize()
        if byzps:
            assert eng._ggraph is not None
        outs.append(eng.flat.reference_vector().clone())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("rule,f", [("krum", 4), ("bulyan", 4), ("median", 8), ("trimmed-mean", 8), ("average", 1)])
def test_engine_more_than_128_workers(cuda, rule, f):
    """n = 256 logical workers (e.g. 8 GPUs x 32 workers): the [n, d] set runs on the
    gar_large.hip path; the update equals the rule applied to the same rows (+ SGD)."""
    from garfield_amd.ops import gar

    torch.manual_seed(0)
    k = 256
    cfg = EngineConfig(gar=rule, f=f, workers_per_rank=k, lr=0.1, momentum=0.0, weight_decay=0.0,
                       byzantine={3: "reverse", 77: "reverse"}, cuda_graph=False)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(device=cuda), cfg)
    batches = synthetic_batches(k, 2, (1, 28, 28), 10, cuda)
    before = eng.flat.data[: eng.d].clone()
    eng.step(batches)
    torch.cuda.synchronize()
    kw = {"f": f} if rule not in ("median", "average") else {}
    want = gar.aggregate(rule, eng.G, **kw).float()
    got = (before - eng.flat.data[: eng.d]) / 0.1
    assert torch.allclose(got, want, rtol=2e-2, atol=1e-4), (got - want).abs().max()
    if rule == "krum":
        w = eng.last_weights.cpu()
        assert w[3] == 0 and w[77] == 0 and abs(float(w.sum()) - 1) < 1e-5


def test_grouped_resume_after_capture_is_exact(cuda, tmp_path):
    """Restoring a checkpoint into an engine whose grouped step is already captured as a
    HIP graph: the replayed continuation equals the uninterrupted run bit for bit."""
    from garfield_amd.utils.checkpoint import load_engine, save_engine

    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda),
                             EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.02, cuda_graph=True))
    batches = synthetic_batches(5, 8, (3, 32, 32), 10, cuda)
    for _ in range(3):
        eng.step(batches)
    assert eng._ggraph is not None
    ck = str(tmp_path / "ck.pt")
    save_engine(ck, eng)
    for _ in range(2):
        eng.step(batches)
    straight = eng.flat_model().clone()
    load_engine(ck, eng)
    assert eng._ggraph is None and eng.step_count == 3
    for _ in range(2):
        eng.step(batches)
    assert eng._ggraph is not None
    assert torch.equal(eng.flat_model(), straight)


@pytest.mark.gpu
@pytest.mark.parametrize("P,T,d,dtype", [(3, 2, 100003, torch.bfloat16), (0, 1, 4096, torch.bfloat16),
                                         (7, 1, 5000, torch.float32), (1, 3, 777, torch.float16)])
def test_fused_collude_kernel_matches_attack_functions(cuda, native, P, T, d, dtype):
    """gar_combine.hip k_collude (lie / empire in place on the exchanged rows, estimates read once)
    against runtime/attacks.py's lie_attack / empire_attack on the same rows (fp32 statistics, one
    rounding to the exchange dtype)."""
    from garfield_amd.runtime.attacks import EMPIRE_EPS, LIE_Z, empire_attack, lie_attack

    g = torch.Generator(device="cpu").manual_seed(P * 31 + T)
    for empire in (False, True):
        ld = (d + 7) // 8 * 8   # rows 16-byte aligned, as the exchange buffer's padded rows are
        X = torch.zeros(P + T, ld, dtype=dtype, device=cuda)[:, :d]
        X.copy_((torch.randn(P + T, d, generator=g) * 0.01 + 0.003).to(dtype))
        ests = [X[i].float() for i in range(P)]
        want = []
        for t in range(T):
            gt = X[P + t].float()
            E = torch.stack([gt, *ests])
            want.append((empire_attack if empire else lie_attack)(gt, E).to(dtype))
        native.gpu_collude([X[i] for i in range(P + T)], P, empire, EMPIRE_EPS if empire else LIE_Z)
        for t in range(T):
            got, w = X[P + t].float(), want[t].float()
            err = ((got - w).abs() / (w.abs() + 1e-3)).max().item()
            assert err < 1e-2, (empire, t, err)


def test_resume_in_new_process_replays_kernel_choices(cuda, tmp_path):
    """The grouped step times some kernel choices in its first eager step (gemm_nt tiles, stride-2
    dgrad form, small-image wgrad form: ops/tuning.py), and the candidates round bf16 differently.
    A checkpoint carries the table: a NEW process whose tables were pre-seeded with other choices
    restores the checkpoint and continues bit for bit like the writer."""
    import json
    import subprocess
    import sys

    from garfield_amd.ops import tuning
    from garfield_amd.utils.checkpoint import save_engine

    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet50"), F.cross_entropy, DistContext(device=cuda),
                             EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.02, cuda_graph=True))
    batches = synthetic_batches(5, 8, (3, 32, 32), 10, cuda)
    for _ in range(2):
        eng.step(batches)
    ck = str(tmp_path / "ck.pt")
    save_engine(ck, eng)
    for _ in range(2):
        eng.step(batches)
    torch.cuda.synchronize()
    want = eng.flat_model().cpu()
    table = tuning.export()
    assert table["gemm"] and table["scwg"], "the measured paths must have run (ResNet-50 CIFAR)"
    tp = tmp_path / "table.json"
    tp.write_text(json.dumps(table))
    out = str(tmp_path / "child.pt")
    child = os.path.join(os.path.dirname(__file__), "_resume_child.py")
    r = subprocess.run([sys.executable, child, ck, str(tp), out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = torch.load(out, weights_only=True)
    assert got["table"] == table
    assert torch.equal(got["flat"], want)


def test_capture_after_dropping_engine_in_reference_cycle(cuda):
    """Regression (round 5 suite abort): a dead engine held only by a reference cycle, with its HIP
    graphs, must not be collected in the middle of the next engine's graph capture (_capture_guard).
    The collector runs at nearly every allocation here; the new engine captures and steps normally."""
    import gc

    def make():
        torch.manual_seed(0)
        return RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda),
                                  EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.02, cuda_graph=True))

    batches = synthetic_batches(5, 8, (3, 32, 32), 10, cuda)
    old = make()
    for _ in range(3):
        old.step(batches)
    assert old._ggraph is not None
    old.cycle = {"engine": old}     # only the cyclic collector can free it now
    del old
    thresholds = gc.get_threshold()
    gc.set_threshold(1, 1, 1)
    try:
        new = make()
        for _ in range(3):
            new.step(batches)
        torch.cuda.synchronize()
    finally:
        gc.set_threshold(*thresholds)
    assert new._ggraph is not None
    assert torch.isfinite(new.flat_model()).all()


def test_capacity_routing_at_the_boundary(cuda, monkeypatch):
    """Capacity routing decided before capture: with the indexing limit at exactly the job's largest tensor
    the step is grouped (one HIP graph); one element lower it runs the workers one at a time, and both
    train (finite, changed parameters). The limit is lowered instead of allocating 2^31-element tensors."""
    from garfield_amd.parallel import grouped

    batches = synthetic_batches(5, 8, (3, 32, 32), 10, cuda)
    for delta, want_grouped in ((0, True), (-1, False)):
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda),
                                 EngineConfig(gar="krum", f=1, workers_per_rank=5, lr=0.02, cuda_graph=True))
        limit = grouped.largest_index(eng.model, 5 * 8, (3, 32, 32)) + delta
        monkeypatch.setattr(grouped, "INDEX_LIMIT", limit)
        before = eng.flat_model().clone()
        for _ in range(3):
            loss = eng.step(batches)
        torch.cuda.synchronize()
        assert (eng._ggraph is not None) == want_grouped
        assert (eng._graph is not None) == (not want_grouped)   # the per-worker graphs
        assert torch.isfinite(loss).item() and not torch.equal(before, eng.flat_model())
