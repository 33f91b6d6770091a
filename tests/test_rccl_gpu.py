"""The direct RCCL calls (``parallel/rccl.py``, ``csrc/rccl_direct.cpp``) against torch's own
librccl and communicator, on a one-rank NCCL process group: the symbols bind, every call
enqueues on the caller's stream and moves the right bytes. Multi-rank transfers run at
round end on 8 GPUs; their call contract is rehearsed on gloo in ``test_scale_cpu.py``."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def one_rank_nccl():
    if dist.is_initialized():
        pytest.skip("a process group is already initialised")
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def test_direct_rccl_calls_on_one_rank(one_rank_nccl, monkeypatch):
    from garfield_amd.parallel.rccl import DirectRCCL

    monkeypatch.setenv("GARFIELD_DIRECT_RCCL", "1")
    dev = one_rank_nccl
    d = DirectRCCL.create()
    assert d is not None, "the direct RCCL path must bind on a GPU box"
    s = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    a = torch.randn(4096, device=dev, generator=g).to(torch.bfloat16)
    b = torch.empty_like(a)
    red = torch.randn(777, device=dev, generator=g)
    red0 = red.clone()
    # point-to-point group: two rows' shards to "rank 0" (itself), matched in issue order
    rows = torch.randn(2, 3000, device=dev, generator=g).to(torch.bfloat16)
    recv = torch.empty(2, 1000, dtype=torch.bfloat16, device=dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        d.all_to_all(a, b, s)
        d.all_reduce_sum(red, s)
        d.exchange([rows[0, 1000:2000], rows[1, 2000:3000]], [0, 0], [recv[0], recv[1]], [0, 0], s)
    s.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(red, red0)
    assert torch.equal(recv[0], rows[0, 1000:2000]) and torch.equal(recv[1], rows[1, 2000:3000])
    # in-place all-gather of this rank's own block
    blk = torch.randn(1000, device=dev, generator=g)
    out = torch.empty(1000, device=dev)
    out.copy_(blk)
    with torch.cuda.stream(s):
        d.all_gather(out, out, s)
    s.synchronize()
    assert torch.equal(out, blk)


class _Calls:
    """Counts the torch.distributed collectives the engines issue (wrapping the module functions)."""

    NAMES = ("all_to_all_single", "all_gather_into_tensor", "all_reduce", "broadcast", "broadcast_object_list")

    def __init__(self, monkeypatch):
        self.n = dict.fromkeys(self.NAMES, 0)
        for name in self.NAMES:
            fn = getattr(dist, name)

            def wrap(*a, _fn=fn, _name=name, **kw):
                self.n[_name] += 1
                return _fn(*a, **kw)
            monkeypatch.setattr(dist, name, wrap)


def _resnet_engine(dev, cls=None, cfg=None, **kw):
    import torch.nn.functional as F

    from garfield_amd.models import build_model
    from garfield_amd.parallel.comm import DistContext
    from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel

    torch.manual_seed(0)
    cfg = cfg or EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, cuda_graph=True, **kw)
    return (cls or RobustDataParallel)(build_model("resnet18"), F.cross_entropy,
                                       DistContext(device=dev, backend="nccl"), cfg)


def _run(eng, dev, steps=10):
    from garfield_amd.parallel.engine import synthetic_batches

    for it in range(steps):
        eng.step(synthetic_batches(8, 8, (3, 32, 32), 10, dev, seed=300 + it))
    eng.synchronize()
    torch.cuda.synchronize()


@pytest.mark.parametrize("path", ["torch.distributed", "direct"])
def test_sharded_step_on_one_rank_rccl_equals_loopback(one_rank_nccl, monkeypatch, path):
    """The default multi-rank sharded step (``torch.distributed``: per bucket a ``[dst, worker,
    shard]`` pack and one ``all_to_all_single`` issued from the comm stream after the device-side
    hand-off, the partial-Gram all-gather, the in-place ``all_gather_into_tensor`` of the bf16
    working weights, the BatchNorm-affine all-reduce, ``sync_master`` and ``momentum_vector``;
    the grouped step captured with ``capture_error_mode="thread_local"`` beside RCCL's watchdog, as the
    staged three-graph forward: every torch.distributed work is waited on by the comm stream)
    and the opt-in direct RCCL path (point-to-point from the exchange rows, staged three-graph
    forward), both as REAL RCCL calls on a one-rank communicator (``GARFIELD_COLL_WORLD1=1``).
    Ten HIP-graph steps with fresh inputs must be bitwise equal to the same step without any
    collective (the world-1 loopback run of the same machinery)."""
    dev = one_rank_nccl
    outs = []
    for coll in ("0", "1"):
        monkeypatch.setenv("GARFIELD_COLL_WORLD1", coll)
        monkeypatch.setenv("GARFIELD_LOOPBACK_EXCHANGE", "1" if coll == "0" else "0")
        monkeypatch.setenv("GARFIELD_OVERLAP", "1")
        monkeypatch.setenv("GARFIELD_DIRECT_RCCL", "1" if (coll == "1" and path == "direct") else "0")
        calls = _Calls(monkeypatch) if coll == "1" else None
        eng = _resnet_engine(dev, shard_gar=True)
        sh = eng._shard
        assert sh._coll == (coll == "1")
        assert (sh._rccl is not None) == (coll == "1" and path == "direct")
        _run(eng, dev)
        if coll == "1" and path == "torch.distributed":
            nb = len(sh.buckets)
            assert nb == 3
            assert calls.n["all_to_all_single"] == 10 * nb            # one packed exchange per bucket and step
            assert calls.n["all_gather_into_tensor"] >= 10 * (nb + 1)  # weights per bucket + the partial Grams
            assert calls.n["all_reduce"] >= 10                         # BatchNorm affine (fp32 read directly)
            assert calls.n["broadcast_object_list"] == 1               # the kernel-choice agreement (ops/tuning)
        # every path stream-ordered on the comm stream: the next forward staged at the bucket boundaries
        assert isinstance(eng._ggraph, list) and len(eng._ggraph) == 3 and sh.staged
        eng.sync_master()
        outs.append((eng.flat.reference_vector().clone(), eng.momentum_vector().clone()))
        del eng, sh
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def test_unsharded_slot_allgather_on_one_rank_rccl(one_rank_nccl, monkeypatch):
    """The unsharded engine's in-place slot all-gathers (``comm.all_gather_rows``: NCCL's in-place
    ``all_gather_into_tensor``, input = this rank's row of the output) on a real one-rank RCCL
    communicator: bitwise equal to the run without collectives."""
    dev = one_rank_nccl
    outs = []
    for coll in ("0", "1"):
        monkeypatch.setenv("GARFIELD_COLL_WORLD1", coll)
        calls = _Calls(monkeypatch)
        eng = _resnet_engine(dev, shard_gar=False)
        assert eng._shard is None
        _run(eng, dev, steps=5)
        assert calls.n["all_gather_into_tensor"] == (5 * 8 if coll == "1" else 0)
        outs.append(eng.flat.reference_vector().clone())
    assert torch.equal(outs[0], outs[1])


def test_byzps_on_one_rank_rccl(one_rank_nccl, monkeypatch):
    """Byzantine-server mode (one server replica hosting its 8 workers, MAR over one model) with its
    slot all-gathers and model broadcast on a real one-rank RCCL communicator: equal to the run
    without collectives."""
    from dataclasses import asdict

    from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig
    from garfield_amd.parallel.engine import EngineConfig

    dev = one_rank_nccl
    outs = []
    for coll in ("0", "1"):
        monkeypatch.setenv("GARFIELD_COLL_WORLD1", coll)
        calls = _Calls(monkeypatch)
        base = EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, cuda_graph=True, byzantine={6: "reverse"})
        cfg = ByzPSConfig(**asdict(base), num_ps=1, fps=0, mar="median", ps_workers=True)
        eng = _resnet_engine(dev, cls=ByzantinePSDataParallel, cfg=cfg)
        _run(eng, dev, steps=4)
        assert calls.n["broadcast"] == (1 + 4 if coll == "1" else 0)   # initial weights + one model per step
        assert calls.n["all_gather_into_tensor"] == (4 * 8 if coll == "1" else 0)
        outs.append(eng.flat.reference_vector().clone())
    assert torch.equal(outs[0], outs[1])


def test_quorum_engine_on_one_rank_rccl(one_rank_nccl, monkeypatch):
    """The asynchronous-quorum engine's per-root broadcast groups and decision group (``new_group``
    subgroups of a real RCCL communicator, one rank: quorum 1 = this rank): the update equals the
    synchronous engine's on the same rows."""
    from dataclasses import asdict

    from garfield_amd.parallel.engine import EngineConfig
    from garfield_amd.parallel.quorum import QuorumConfig, QuorumDataParallel

    dev = one_rank_nccl
    outs = []
    for quorum in (False, True):
        monkeypatch.setenv("GARFIELD_COLL_WORLD1", "1" if quorum else "0")
        base = EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, cuda_graph=True, shard_gar=False)
        if quorum:
            eng = _resnet_engine(dev, cls=QuorumDataParallel, cfg=QuorumConfig(**asdict(base)))
        else:
            eng = _resnet_engine(dev, cfg=base)
        _run(eng, dev, steps=4)
        if quorum:
            eng.finish()
            assert eng.last_quorum == [0] and eng.skipped == 0
        outs.append(eng.flat.reference_vector().clone())
    assert torch.equal(outs[0], outs[1])
