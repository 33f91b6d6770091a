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


def test_direct_rccl_calls_on_one_rank(one_rank_nccl):
    from garfield_amd.parallel.rccl import DirectRCCL

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
