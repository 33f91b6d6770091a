"""GPU probe (one rank, RCCL): the direct collectives of parallel/rccl.py on torch's
communicator, and what each way of running a collective beside a graph replay costs
the graph (device time per replay of a 400-kernel graph on the main stream):

* torch collective issued from a side stream (ProcessGroupNCCL's own stream waits on it);
* the same collective enqueued directly on the side stream (DirectRCCL);
both behind a device-side counter hand-off from the main stream (parallel/signals.py).

    python scripts/probe_rccl_direct.py
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from garfield_amd.parallel.rccl import DirectRCCL  # noqa: E402
from garfield_amd.parallel.signals import DeviceSignal  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    t = torch.ones(8, device=dev)
    dist.all_reduce(t)
    rc = DirectRCCL.create()
    res = {"direct_available": rc is not None}
    side = torch.cuda.Stream()
    # correctness on one rank
    send = torch.randn(1 << 20, device=dev).to(torch.bfloat16)
    recv = torch.empty_like(send)
    with torch.cuda.stream(side):
        rc.all_to_all(send, recv, side)
        g = torch.empty_like(send)
        rc.all_gather(send, g, side)
        r = send.float().clone()
        rc.all_reduce_sum(r, side)
    torch.cuda.synchronize()
    res["all_to_all_ok"] = bool(torch.equal(recv, send))
    res["all_gather_ok"] = bool(torch.equal(g, send))
    res["all_reduce_ok"] = bool(torch.equal(r, send.float()))
    # cost beside a graph replay
    cap = torch.cuda.Stream()
    a = torch.randn(1 << 20, device=dev)
    b = torch.empty_like(a)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cap):
        for i in range(400):
            (b if i % 2 else a).copy_(a if i % 2 else b)
    cur = torch.cuda.current_stream()
    big = torch.randn(32 << 20, device=dev).to(torch.bfloat16)
    big_out = torch.empty_like(big)
    sig = DeviceSignal(dev)
    done = torch.cuda.Event()

    def timed(name, fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(cur)
        for _ in range(iters):
            fn()
        t1.record(cur)
        torch.cuda.synchronize()
        res[name] = round(t0.elapsed_time(t1) / iters, 4)

    def plain():
        graph.replay()

    def handoff_torch():
        graph.replay()
        sig.record(cur)
        sig.wait_on(side)
        with torch.cuda.stream(side):
            w = dist.all_to_all_single(big_out, big, async_op=True)
        w.wait()

    def handoff_direct():
        graph.replay()
        sig.record(cur)
        sig.wait_on(side)
        rc.all_to_all(big, big_out, side)
        done.record(side)
        cur.wait_event(done)

    for name, fn in (("plain", plain), ("handoff_torch_a2a", handoff_torch), ("handoff_direct_a2a", handoff_direct),
                     ("plain_again", plain)):
        timed(name, fn)
    res["misses"] = sig.misses()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
