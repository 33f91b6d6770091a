"""Robust DP engine on CPU: single process and 2-rank gloo (multi-process) runs."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("rule,f", [("krum", 2), ("median", 1), ("bulyan", 1), ("trimmed-mean", 2),
                                    ("average", 1), ("brute", 2), ("aksel", 2)])
def test_single_process_rules(rule, f):
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(),
                             EngineConfig(gar=rule, f=f, workers_per_rank=8,
                                          byzantine={} if rule == "average" else {1: "reverse"}))
    b = synthetic_batches(8, 16, (1, 28, 28), 10, "cpu")
    l0 = float(eng.step(b))
    for _ in range(5):
        l1 = float(eng.step(b))
    assert torch.isfinite(eng.flat_model()).all()
    assert l1 < l0 + 1e-3


def _worker(rank, world, port, outdir, rule):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(rank)  # different init per rank: the engine must broadcast rank 0's
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                             EngineConfig(gar=rule, f=1, workers_per_rank=4, byzantine={3: "reverse"}))
    b = synthetic_batches(4, 8, (1, 28, 28), 10, "cpu", seed=rank)
    for _ in range(3):
        eng.step(b)
    torch.save({"flat": eng.flat_model().clone(), "w": eng.last_weights}, os.path.join(outdir, f"r{rank}.pt"))
    shutdown(ctx)


@pytest.mark.parametrize("rule", ["krum", "median"])
def test_two_rank_gloo_replicas_identical(rule):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, free_port(), d, rule), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
        assert torch.equal(r0["flat"], r1["flat"])


def _sharded_worker(rank, world, port, outdir, rule, shard):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                             EngineConfig(gar=rule, f=1, workers_per_rank=4, byzantine={3: "reverse"},
                                          shard_gar=shard, lr=0.05))
    assert (eng._shard is not None) == shard
    b = synthetic_batches(4, 8, (1, 28, 28), 10, "cpu", seed=rank)
    for _ in range(3):
        eng.step(b)
    torch.save({"flat": eng.flat_model().clone(), "mom": eng.momentum_vector()[: eng.d].clone()},
               os.path.join(outdir, f"{int(shard)}r{rank}.pt"))
    shutdown(ctx)


@pytest.mark.parametrize("rule", ["krum", "median", "bulyan", "aksel", "average", "trimmed-mean", "brute"])
def test_two_rank_sharded_aggregation_matches_allgather(rule):
    """all_to_all + sharded GAR + all-gather == all-gather + redundant GAR (and replicas agree)."""
    with tempfile.TemporaryDirectory() as d:
        for shard in (False, True):
            mp.spawn(_sharded_worker, args=(2, free_port(), d, rule, shard), nprocs=2, join=True)
        r = {k: torch.load(os.path.join(d, f"{k}.pt"), weights_only=True) for k in ("0r0", "0r1", "1r0", "1r1")}
        assert torch.equal(r["1r0"]["flat"], r["1r1"]["flat"])           # sharded replicas identical
        assert torch.equal(r["0r0"]["flat"], r["0r1"]["flat"])           # redundant replicas identical
        ref_flat = r["0r0"]["flat"]
        rel = ((r["1r0"]["flat"] - ref_flat).norm() / ref_flat.norm()).item()
        assert rel < 1e-5, rel
        m0, m1 = r["0r0"]["mom"], r["1r0"]["mom"]
        assert ((m1 - m0).norm() / m0.norm()).item() < 1e-5


@pytest.mark.parametrize("rule,f", [("krum", 2), ("median", 1), ("bulyan", 1), ("aksel", 2)])
def test_single_rank_sharded_path_matches(rule, f):
    """shard_gar=True on one rank runs the sharded code path with identity collectives."""
    outs = []
    for shard in (False, True):
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(),
                                 EngineConfig(gar=rule, f=f, workers_per_rank=8, shard_gar=shard,
                                              byzantine={1: "reverse"}))
        assert (eng._shard is not None) == shard
        b = synthetic_batches(8, 16, (1, 28, 28), 10, "cpu")
        for _ in range(3):
            eng.step(b)
        outs.append(eng.flat_model().clone())
    rel = ((outs[1] - outs[0]).norm() / outs[0].norm()).item()
    assert rel < 1e-6, rel


def _grouped_sharded_worker(rank, world, port, outdir, shard):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, ctx,
                             EngineConfig(gar="krum", f=1, workers_per_rank=3, byzantine={1: "reverse"},
                                          shard_gar=shard, worker_batching=True, autocast_dtype=None,
                                          exchange_dtype=torch.float32, lr=0.01))
    assert eng._gexec is not None and (eng._shard is not None) == shard
    b = synthetic_batches(3, 4, (3, 32, 32), 10, "cpu", seed=rank)
    for _ in range(2):
        eng.step(b)
    torch.save({"flat": eng.flat_model().clone()}, os.path.join(outdir, f"{int(shard)}r{rank}.pt"))
    shutdown(ctx)


def test_two_rank_grouped_workers_with_sharded_aggregation():
    """The flagship multi-GPU configuration on CPU: worker batching + sharded aggregation."""
    with tempfile.TemporaryDirectory() as d:
        for shard in (False, True):
            mp.spawn(_grouped_sharded_worker, args=(2, free_port(), d, shard), nprocs=2, join=True)
        r = {k: torch.load(os.path.join(d, f"{k}.pt"), weights_only=True)["flat"]
             for k in ("0r0", "0r1", "1r0", "1r1")}
        assert torch.equal(r["1r0"], r["1r1"]) and torch.equal(r["0r0"], r["0r1"])
        rel = ((r["1r0"] - r["0r0"]).norm() / r["0r0"].norm()).item()
        assert rel < 1e-5, rel


@pytest.mark.parametrize("rule,f", [("krum", 2), ("bulyan", 1)])
def test_layerwise_gar_matches_per_tensor_oracle(rule, f):
    """Garfield_CC's per-layer mode (reference trainer.py:90-140): the GAR runs on each
    parameter tensor's gradients separately; one SGD step (no momentum / decay) must
    equal the fp64 oracle applied tensor by tensor -- and differ from the flat rule."""
    from garfield_amd.ops import reference as ref

    torch.manual_seed(0)
    k = 8
    cfg = dict(gar=rule, f=f, workers_per_rank=k, byzantine={1: "reverse"}, lr=0.1, momentum=0.0,
               weight_decay=0.0, exchange_dtype=torch.float32)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(), EngineConfig(layerwise=True, **cfg))
    b = synthetic_batches(k, 16, (1, 28, 28), 10, "cpu")
    before = eng.flat.data[: eng.d].clone()
    eng.step(b)
    G = eng.G.double()
    expect = torch.empty(eng.d, dtype=torch.float64)
    for off, numel in zip(eng.flat.offsets, eng.flat.numels):
        seg = G[:, off:off + numel]
        expect[off:off + numel] = ref.krum(seg, f) if rule == "krum" else ref.bulyan(seg, f)
    got = (before - eng.flat.data[: eng.d]).double() / 0.1
    assert ((got - expect).norm() / expect.norm()).item() < 1e-5
    flat = ref.krum(G, f) if rule == "krum" else ref.bulyan(G, f)
    assert ((flat - expect).norm() / expect.norm()).item() > 1e-6   # a different rule than the flat one


@pytest.mark.parametrize("collusion", ["fw", "all"])
def test_colluding_attacks_use_exchanged_rows(collusion):
    """lie / empire run on the exchanged rows: the attacker's own honest gradient plus
    fw - 1 honest peers (reference byzWorker.py:108-143) or every honest row."""
    from garfield_amd.runtime.attacks import empire_attack, lie_attack

    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(),
                             EngineConfig(gar="average", f=2, workers_per_rank=8, byzantine={1: "lie", 5: "empire"},
                                          collusion=collusion))
    b = synthetic_batches(8, 16, (1, 28, 28), 10, "cpu")
    eng.compute_local(b)
    G0 = eng.G.clone()   # every row still honest: the colluders act after the exchange
    honest = [0, 2, 3, 4, 6, 7]
    peers = honest[:1] if collusion == "fw" else honest
    eng.aggregate_and_update()
    for s, fn in ((1, lie_attack), (5, empire_attack)):
        want = fn(G0[s], torch.stack([G0[s].float(), *[G0[p].float() for p in peers]]))
        assert torch.allclose(eng.G[s], want, rtol=1e-6, atol=1e-7)
    assert torch.equal(eng.G[honest], G0[honest])


def _collusion_worker(rank, world, port, outdir, shard):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                             EngineConfig(gar="median", f=2, workers_per_rank=4, byzantine={1: "lie", 6: "empire"},
                                          shard_gar=shard, lr=0.05, collusion="all"))
    b = synthetic_batches(4, 8, (1, 28, 28), 10, "cpu", seed=rank)
    for _ in range(3):
        eng.step(b)
    torch.save({"flat": eng.flat_model().clone()}, os.path.join(outdir, f"{int(shard)}r{rank}.pt"))
    shutdown(ctx)


def test_two_rank_collusion_sharded_matches_allgather():
    """Colluders on a coordinate shard (owner side) == colluders on gathered rows."""
    with tempfile.TemporaryDirectory() as d:
        for shard in (False, True):
            mp.spawn(_collusion_worker, args=(2, free_port(), d, shard), nprocs=2, join=True)
        a = torch.load(os.path.join(d, "0r0.pt"), weights_only=True)["flat"]
        for name in ("0r1.pt", "1r0.pt", "1r1.pt"):
            other = torch.load(os.path.join(d, name), weights_only=True)["flat"]
            assert torch.allclose(a, other, rtol=1e-5, atol=1e-6), name


def _lw_sharded_worker(rank, world, port, outdir, shard):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from garfield_amd.parallel.comm import init_distributed, shutdown

    ctx = init_distributed(backend="gloo", device="cpu")
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                             EngineConfig(gar="krum", f=1, workers_per_rank=4, byzantine={3: "reverse"},
                                          shard_gar=shard, layerwise=True, lr=0.05))
    assert (eng._shard is not None) == shard
    b = synthetic_batches(4, 8, (1, 28, 28), 10, "cpu", seed=rank)
    for _ in range(3):
        eng.step(b)
    w = eng.last_weights
    torch.save({"flat": eng.flat_model().clone(), "mom": eng.momentum_vector()[: eng.d].clone(),
                "w": w.clone() if w is not None else None}, os.path.join(outdir, f"{int(shard)}r{rank}.pt"))
    shutdown(ctx)


def test_two_rank_sharded_layerwise_krum_matches_redundant():
    """Layer-wise Krum with the sharded exchange (per-segment partial distances summed over
    ranks, per-segment selections, owned coordinates combined by segment) == the redundant
    layer-wise path; replicas identical."""
    with tempfile.TemporaryDirectory() as d:
        for shard in (False, True):
            mp.spawn(_lw_sharded_worker, args=(2, free_port(), d, shard), nprocs=2, join=True)
        r = {k: torch.load(os.path.join(d, f"{k}.pt"), weights_only=True) for k in ("0r0", "0r1", "1r0", "1r1")}
        assert torch.equal(r["1r0"]["flat"], r["1r1"]["flat"]) and torch.equal(r["0r0"]["flat"], r["0r1"]["flat"])
        w0, w1 = r["0r0"]["w"], r["1r0"]["w"]
        assert w1.shape == w0.shape and w1.shape[0] >= 2                  # one selection per parameter tensor
        assert torch.equal(w1, w0.to(w1.dtype))                            # the same per-segment selections
        assert float(w1[:, 3].abs().max()) == 0.0                          # the reversed slot is never selected
        ref_flat = r["0r0"]["flat"]
        rel = ((r["1r0"]["flat"] - ref_flat).norm() / ref_flat.norm()).item()
        assert rel < 1e-5, rel
        m0, m1 = r["0r0"]["mom"], r["1r0"]["mom"]
        assert ((m1 - m0).norm() / m0.norm()).item() < 1e-5


@pytest.mark.parametrize("rule,n,f,ok", [
    ("krum", 64, 2, True), ("krum", 256, 2, False),
    ("bulyan", 64, 3, True), ("bulyan", 72, 1, False), ("bulyan", 128, 31, True), ("bulyan", 128, 30, False),
    ("brute", 64, 1, True), ("brute", 72, 1, False),
    ("aksel", 128, 2, True), ("aksel", 256, 2, False),
])
def test_sharded_layerwise_routing_respects_device_limits(rule, n, f, ok):
    """Multi-rank layer-wise runs take the sharded device path only inside its kernels' limits
    (segmented Gram n <= 128, Bulyan tail t <= 64, Brute n <= 64); beyond them the engine keeps
    the unsharded per-segment loop instead of failing after the exchange."""
    from garfield_amd.parallel.sharded import layerwise_device_ok

    assert layerwise_device_ok(rule, n, f) == ok
