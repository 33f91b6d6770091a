"""Multi-rank rehearsals of the default multi-GPU path (sharded, bucketed aggregation)
on gloo/CPU at 4 and 8 ranks: every rank runs what ``bench.py --gpus N`` runs on N
MI355X (one process per device), with CPU tensors.

* 8 ranks x 2 workers (n = 16): sharded == redundant (all-gather) aggregation,
  BITWISE, for every distance-based and coordinate-wise rule, with a colluding
  ``lie`` attacker and a ``reverse`` one; every replica's checksum equal;
* 8 ranks x 8 grouped ResNet workers (n = 64): shard_pad(8), the three layer
  buckets and the n = 64 Krum selection of the flagship configuration;
* the exchange leaves in ONE ``all_to_all_single`` per bucket;
* the same runs through ``GlooDirect`` (``parallel/rccl.py``): the direct-RCCL branch of the
  exchange that 8 GPUs take, with its call contract checked (one group of point-to-point
  transfers per bucket straight from the exchange rows, sizes matched against the peers'
  receives, the own shard never sent; in-place all-gather of this rank's block), bitwise
  equal to the torch.distributed branch.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches

RULES = [("krum", 2), ("bulyan", 2), ("median", 2), ("trimmed-mean", 2), ("brute", 2), ("aksel", 2)]
BYZ = {3: "lie", 12: "reverse"}
LW_RULES = [("bulyan", 2), ("krum", 2), ("brute", 2), ("aksel", 2), ("median", 2)]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from garfield_amd.parallel.comm import init_distributed

    return init_distributed(backend="gloo", device="cpu")


def _direct(mode):
    """mode 2: the sharded exchange through GlooDirect, DirectRCCL's call contract (the branch
    8 GPUs take), with the CPU shadow so the weight all-gathers and the compact all-reduce run."""
    from garfield_amd.parallel import rccl

    if mode != 2:
        rccl.set_direct_backend(None)
        return None
    made = []

    def factory(world, rank):
        made.append(rccl.GlooDirect(world, rank))
        return made[-1]

    rccl.set_direct_backend(factory)
    return made


def _rules_worker(rank, world, port, outdir, mode, layerwise=False):
    from garfield_amd.parallel.comm import shutdown

    ctx = _init(rank, world, port)
    made = _direct(mode)
    out = {}
    for rule, f in (LW_RULES if layerwise else RULES):
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("mlp"), F.nll_loss, ctx,
                                 EngineConfig(gar=rule, f=f, workers_per_rank=2, byzantine=BYZ, shard_gar=mode > 0,
                                              lr=0.05, collusion="all", shadow_cpu=mode == 2, layerwise=layerwise))
        assert (eng._shard is not None) == (mode > 0)
        if mode == 2:
            assert eng._shard._rccl is made[-1] and eng._shadow is not None
        b = synthetic_batches(2, 8, (1, 28, 28), 10, "cpu", seed=rank)
        for _ in range(2):
            eng.step(b)
        w = eng.last_weights
        out[rule] = {"flat": eng.flat_model().clone(), "sum": eng.replica_checksum(),
                     "calls": dict(made[-1].calls) if mode == 2 else {},
                     "w": w.clone().float() if w is not None else torch.zeros(0)}
    torch.save(out, os.path.join(outdir, f"{mode}r{rank}.pt"))
    shutdown(ctx)


def test_eight_rank_sharded_equals_redundant_bitwise():
    """Redundant (0), sharded over torch.distributed (1) and sharded through the direct-RCCL
    contract (2): bitwise equal for every rule, on every rank."""
    world = 8
    with tempfile.TemporaryDirectory() as d:
        for mode in (0, 1, 2):
            mp.spawn(_rules_worker, args=(world, free_port(), d, mode), nprocs=world, join=True)
        res = {(s, r): torch.load(os.path.join(d, f"{s}r{r}.pt"), weights_only=True)
               for s in (0, 1, 2) for r in range(world)}
        for rule, _ in RULES:
            ref = res[(0, 0)][rule]
            for s in (0, 1, 2):
                for r in range(world):
                    got = res[(s, r)][rule]
                    assert got["sum"] == ref["sum"], (rule, s, r)
                    assert torch.equal(got["flat"], ref["flat"]), (rule, s, r)
            calls = res[(2, 0)][rule]["calls"]
            assert calls["exchange"] == 2 and calls["all_gather_inplace"] == 2, (rule, calls)
            assert "all_reduce" not in calls, (rule, calls)   # every MLP parameter is a shadow view


def test_eight_rank_sharded_layerwise_equals_redundant_bitwise():
    """Garfield_CC's per-layer aggregation (--layerwise) sharded over 8 ranks (per-segment partial
    distances summed over ranks, per-segment selections, each rank's owned coordinates
    aggregated with their segment's selection), through the direct-RCCL contract (2), == the
    redundant per-segment loop (0), BITWISE, for Bulyan, Krum, Brute, Aksel (and a coordinate
    rule, where per-layer == flat); the reversed attacker never selected by Krum."""
    world = 8
    with tempfile.TemporaryDirectory() as d:
        for mode in (0, 2):
            mp.spawn(_rules_worker, args=(world, free_port(), d, mode, True), nprocs=world, join=True)
        res = {(s, r): torch.load(os.path.join(d, f"{s}r{r}.pt"), weights_only=True)
               for s in (0, 2) for r in range(world)}
        for rule, _ in LW_RULES:
            ref = res[(0, 0)][rule]
            for s in (0, 2):
                for r in range(world):
                    got = res[(s, r)][rule]
                    assert got["sum"] == ref["sum"], (rule, s, r)
                    assert torch.equal(got["flat"], ref["flat"]), (rule, s, r)
        wk = res[(2, 0)]["krum"]["w"]
        assert wk.dim() == 2 and wk.shape[0] >= 2 and float(wk[:, 12].abs().max()) == 0.0


def _grouped_worker(rank, world, port, outdir, mode, k):
    from garfield_amd.parallel.comm import shutdown

    ctx = _init(rank, world, port)
    made = _direct(mode)
    shard = mode > 0
    torch.manual_seed(0)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, ctx,
                             EngineConfig(gar="krum", f=2, workers_per_rank=k, byzantine={5: "reverse", 9: "lie"},
                                          shard_gar=shard, worker_batching=True, autocast_dtype=None,
                                          exchange_dtype=torch.float32, lr=0.01, shadow_cpu=mode == 2))
    assert eng._gexec is not None and (eng._shard is not None) == shard
    if shard:
        assert len(eng._shard.buckets) == 3 and eng.ld % (64 * world) == 0
    calls = []
    if mode == 1:
        import torch.distributed as dist

        orig = dist.all_to_all_single

        def counting(*a, **kw):
            calls.append(1)
            return orig(*a, **kw)

        dist.all_to_all_single = counting
    b = synthetic_batches(k, 2, (3, 16, 16), 10, "cpu", seed=rank)
    steps = 2
    per_step = []
    for _ in range(steps):
        before = dict(made[-1].calls) if mode == 2 else {}
        eng.step(b)
        if mode == 2:
            per_step.append({kk: v - before.get(kk, 0) for kk, v in made[-1].calls.items()})
    torch.save({"flat": eng.flat_model().clone(), "sum": eng.replica_checksum(), "a2a": len(calls),
                "w": eng.last_weights, "n": eng.n, "per_step": per_step},
               os.path.join(outdir, f"{mode}r{rank}.pt"))
    shutdown(ctx)


@pytest.mark.parametrize("world,k", [(4, 4), (8, 8)])
def test_grouped_sharded_flagship_path(world, k):
    """ResNet worker batching + sharded bucketed Krum at 4 x 4 (n = 16) and 8 x 8 (n = 64)
    ranks x workers: replicas identical, sharded == redundant, 3 all_to_all per step; the
    direct-RCCL contract (mode 2) bitwise equal to the torch.distributed branch, with the exact
    collective pattern of a GPU step: 3 point-to-point exchange groups + 1 Gram all-gather + 3 in-place weight
    all-gathers + 1 all-reduce per bucket of its BatchNorm affine parameters."""
    with tempfile.TemporaryDirectory() as d:
        for mode in (0, 1, 2):
            mp.spawn(_grouped_worker, args=(world, free_port(), d, mode, k), nprocs=world, join=True)
        res = {(s, r): torch.load(os.path.join(d, f"{s}r{r}.pt"), weights_only=True)
               for s in (0, 1, 2) for r in range(world)}
        ref = res[(0, 0)]
        assert ref["n"] == world * k
        for s in (0, 1, 2):
            for r in range(world):
                got = res[(s, r)]
                assert got["sum"] == res[(s, 0)]["sum"], (s, r)
                assert torch.equal(got["flat"], res[(s, 0)]["flat"]), (s, r)
        assert all(res[(1, r)]["a2a"] == 3 * 2 for r in range(world))   # one all_to_all per bucket and step
        assert all(torch.equal(res[(1, r)]["w"], res[(1, 0)]["w"]) for r in range(world))   # one Krum selection
        rel = ((res[(1, 0)]["flat"] - ref["flat"]).norm() / ref["flat"].norm()).item()
        assert rel < 1e-5, rel
        assert torch.equal(res[(2, 0)]["flat"], res[(1, 0)]["flat"])     # direct contract == dist branch
        for r in range(world):
            for calls in res[(2, r)]["per_step"]:
                assert calls == {"exchange": 3, "all_gather": 1, "all_gather_inplace": 3, "all_reduce": 3}, calls


def _byzps_worker(rank, world, port, outdir, num_ps):
    import torch.distributed as dist

    from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig
    from garfield_amd.parallel.comm import shutdown

    ctx = _init(rank, world, port)
    torch.manual_seed(0)
    eng = ByzantinePSDataParallel(build_model("mlp"), F.nll_loss, ctx,
                                  ByzPSConfig(gar="median", f=1, workers_per_rank=2, num_ps=num_ps, fps=1 if num_ps > 2
                                              else 0, mar="median", byzantine={5: "reverse"}, lr=0.05))
    moved = []
    names = ("broadcast", "all_gather_into_tensor", "all_gather", "all_reduce", "all_to_all_single")
    orig = {k: getattr(dist, k) for k in names}

    def counting(name):
        def f(t, *a, **kw):
            moved.append(t.numel() * t.element_size() if isinstance(t, torch.Tensor) else
                         sum(x.numel() * x.element_size() for x in t))
            return orig[name](t, *a, **kw)
        return f

    inner = eng._exchange_models

    def patched():
        for k in names:
            setattr(dist, k, counting(k))
        try:
            inner()
        finally:
            for k in names:
                setattr(dist, k, orig[k])

    eng._exchange_models = patched
    b = synthetic_batches(2, 8, (1, 28, 28), 10, "cpu", seed=rank)
    for _ in range(2):
        eng.step(b)
    torch.save({"bytes": sum(moved) / 2, "d": eng.d, "ld": eng.ld, "flat": eng.flat_model().clone()},
               os.path.join(outdir, f"r{rank}.pt"))
    shutdown(ctx)


@pytest.mark.parametrize("num_ps", [1, 3])
def test_byzantine_server_model_exchange_moves_only_server_rows(num_ps):
    """The model exchange of the Byzantine-server mode moves <= num_ps x d x 4 bytes per rank
    and step (the server rows only, never M[world, ld]); honest replicas stay identical."""
    world = 5
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_byzps_worker, args=(world, free_port(), d, num_ps), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in res:
        assert 0 < r["bytes"] <= num_ps * r["ld"] * 4, (r["bytes"], num_ps * r["ld"] * 4)
    honest = res[1:] if num_ps > 2 else res   # rank 0 is the Byzantine server when fps = 1
    assert all(torch.equal(r["flat"], honest[-1]["flat"]) for r in honest)


def _byzps_cfg5_worker(rank, world, port, outdir, ps_attack):
    from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig
    from garfield_amd.parallel.comm import shutdown

    ctx = _init(rank, world, port)
    torch.manual_seed(0)
    eng = ByzantinePSDataParallel(build_model("mlp"), F.nll_loss, ctx,
                                  ByzPSConfig(gar="trimmed-mean", f=1, workers_per_rank=1, num_ps=3, fps=1,
                                              mar="median", ps_attack=ps_attack, lr=0.05))
    assert eng.n_w == 5 and eng.is_ps == (rank < 3)
    for it in range(3):
        eng.step(synthetic_batches(1, 8, (1, 28, 28), 10, "cpu", seed=10 * it + rank))
    torch.save({"flat": eng.flat_model().clone()}, os.path.join(outdir, f"{ps_attack or 'none'}_{rank}.pt"))
    shutdown(ctx)


def test_byzantine_server_config5_attacked_server_is_rejected():
    """BASELINE config 5's pattern: 3 server replicas + 5 worker ranks, f_ps = 1, f_w = 1, Trimmed-Mean
    over the workers, coordinate-wise median as the model aggregation. Server rank 0 is Byzantine and
    replaces its model by -100 x its update (``ps_attack=reverse``) every step: every rank -- the
    attacker included, which adopts the aggregate too -- ends bit-identical to the attack-free run (the
    median of three models, two of them the honest servers' identical ones, is the honest model)."""
    world = 8
    with tempfile.TemporaryDirectory() as d:
        for attack in ("", "reverse"):
            mp.spawn(_byzps_cfg5_worker, args=(world, free_port(), d, attack), nprocs=world, join=True)
        clean = [torch.load(os.path.join(d, f"none_{r}.pt"), weights_only=True)["flat"] for r in range(world)]
        hit = [torch.load(os.path.join(d, f"reverse_{r}.pt"), weights_only=True)["flat"] for r in range(world)]
    assert all(torch.equal(c, clean[0]) for c in clean)
    assert all(torch.equal(h, clean[0]) for h in hit)


def _world1_worker(port, outdir):
    """One rank, gloo: the sharded step with its collectives (GARFIELD_COLL_WORLD1=1) vs without."""
    import torch.distributed as dist

    from garfield_amd.parallel.comm import DistContext

    outs = []
    for coll in ("0", "1"):
        os.environ["GARFIELD_COLL_WORLD1"] = coll
        if coll == "1":
            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("convnet"), F.nll_loss, DistContext(backend="gloo" if coll == "1" else "none"),
                                 EngineConfig(gar="krum", f=1, workers_per_rank=5, shard_gar=True, lr=0.05))
        assert eng._shard._coll == (coll == "1")
        for it in range(3):
            eng.step(synthetic_batches(5, 4, (1, 28, 28), 10, torch.device("cpu"), seed=it))
        eng.sync_master()
        outs.append((eng.flat.reference_vector().clone(), eng.momentum_vector().clone()))
    dist.destroy_process_group()
    torch.save(outs, os.path.join(outdir, "w1.pt"))


def test_world1_collectives_equal_shortcuts():
    """GARFIELD_COLL_WORLD1=1 on a one-rank gloo group: the multi-rank sharded call sequence
    (packed all_to_all per bucket, partial-Gram all-gather, weight all-gathers, sync_master,
    momentum_vector) equals the world-1 shortcuts bit for bit (the GPU twin runs on a one-rank
    RCCL communicator: tests/test_rccl_gpu.py)."""
    with tempfile.TemporaryDirectory() as d:
        p = mp.get_context("spawn").Process(target=_world1_worker, args=(free_port(), d))
        p.start()
        p.join(300)
        assert p.exitcode == 0
        (a, ma), (b, mb) = torch.load(os.path.join(d, "w1.pt"), weights_only=True)
        assert torch.equal(a, b) and torch.equal(ma, mb)
