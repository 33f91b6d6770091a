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


def test_sharded_step_on_direct_rccl_one_rank_equals_loopback(one_rank_nccl, monkeypatch):
    """The full sharded grouped step with its collectives issued through the direct RCCL path on
    a one-rank communicator (GARFIELD_DIRECT_RCCL_WORLD1=1): the partial-Gram all-gather, the
    in-place bf16 weight all-gathers and the BatchNorm-affine all-reduce run as real RCCL calls on
    the comm stream, beside the next step's staged three-graph forward, with the in-graph bucket
    signals on. Ten steps with fresh inputs must be bitwise equal to the same step without the
    collectives (the world-1 loopback run of the same machinery)."""
    import torch.nn.functional as F

    from garfield_amd.models import build_model
    from garfield_amd.parallel.comm import DistContext
    from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches

    dev = one_rank_nccl
    monkeypatch.setenv("GARFIELD_LOOPBACK_EXCHANGE", "1")
    monkeypatch.setenv("GARFIELD_OVERLAP", "1")
    outs = []
    for direct in ("0", "1"):
        monkeypatch.setenv("GARFIELD_DIRECT_RCCL", direct)
        monkeypatch.setenv("GARFIELD_DIRECT_RCCL_WORLD1", direct)
        torch.manual_seed(0)
        cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, shard_gar=True, lr=0.01, cuda_graph=True)
        eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=dev), cfg)
        assert (eng._shard._rccl is not None) == (direct == "1")
        for it in range(10):
            eng.step(synthetic_batches(8, 8, (3, 32, 32), 10, dev, seed=300 + it))
        eng.synchronize()
        torch.cuda.synchronize()
        assert isinstance(eng._ggraph, list) and len(eng._ggraph) == 3 and eng._shard.staged
        outs.append((eng.flat.reference_vector().clone(), eng.momentum_vector().clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
