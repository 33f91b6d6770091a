"""Collective bandwidth benchmark of the exchange layer (``bench_comm``).

The reference has no collective benchmark; its closest harness is ``rpc_bench.py``.
This measures the primitives the engine uses on the real process group: RCCL over
xGMI on GPUs, gloo on CPU.

* ``all_gather`` — ``all_gather_into_tensor`` of a ``[d]`` row into ``[world, d]``.
  This is the robust-DP gradient exchange.
* ``broadcast`` — flat-model broadcast (PS → all).
* ``all_reduce`` — the plain-DP baseline (what averaging would cost).
* ``all_to_all`` — for completeness (``all_to_all_single``).

Launch: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 -m garfield_amd.apps.comm_bench``.
Rank 0 prints one JSON line per (op, size). Following nccl-tests, ``algbw`` = bytes per rank
÷ time, and ``busbw`` = algbw × the op's bus factor: (n−1)/n for all_gather / all_to_all,
2(n−1)/n for all_reduce, and 1 for broadcast.
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist

from garfield_amd.parallel.comm import init_distributed, shutdown

DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def _bus_factor(op: str, n: int) -> float:
    if n <= 1:
        return 1.0
    return {"all_gather": (n - 1) / n, "all_to_all": (n - 1) / n, "all_reduce": 2 * (n - 1) / n,
            "broadcast": 1.0}[op]


def bench_op(ctx, op: str, numel: int, dtype, iters: int, warmup: int) -> dict:
    dev, n = ctx.device, ctx.world_size
    x = torch.randn(numel, device=dev).to(dtype)
    if op == "all_gather":
        out = torch.empty(n * numel, device=dev, dtype=dtype)
        fn = lambda: dist.all_gather_into_tensor(out, x)  # noqa: E731
    elif op == "broadcast":
        fn = lambda: dist.broadcast(x, src=0)  # noqa: E731
    elif op == "all_reduce":
        fn = lambda: dist.all_reduce(x)  # noqa: E731
    elif op == "all_to_all":
        m = (numel // n) * n
        xs, out = x[:m].contiguous(), torch.empty(m, device=dev, dtype=dtype)
        fn = lambda: dist.all_to_all_single(out, xs)  # noqa: E731
    else:
        raise ValueError(op)
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    for _ in range(warmup):
        fn()
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    nbytes = numel * x.element_size() * (n if op == "all_gather" else 1)
    algbw = nbytes / dt / 1e9
    return {"op": op, "world": n, "numel": numel, "dtype": str(dtype).replace("torch.", ""), "bytes": nbytes,
            "ms": dt * 1e3, "algbw_GBps": algbw, "busbw_GBps": algbw * _bus_factor(op, n),
            "backend": dist.get_backend()}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--ops", nargs="+", default=["all_gather", "broadcast", "all_reduce", "all_to_all"])
    ap.add_argument("--sizes", nargs="+", type=int, default=[1 << 20, 1 << 22, 23528522, 1 << 26],
                    help="elements per rank (23528522 = ResNet-50/10-class parameters)")
    ap.add_argument("--dtype", choices=list(DTYPES), default="bf16")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    ctx = init_distributed(device=a.device)
    if not dist.is_initialized():   # single process: a 1-rank group still exercises the backend
        backend = "nccl" if ctx.device.type == "cuda" else "gloo"
        dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1)
        ctx.initialized_here = True
    rows = []
    try:
        for op in a.ops:
            for s in a.sizes:
                r = bench_op(ctx, op, s, DTYPES[a.dtype], a.iters, a.warmup)
                rows.append(r)
                if ctx.rank == 0:
                    print(json.dumps(r), flush=True)
    finally:
        shutdown(ctx)
    return rows


if __name__ == "__main__":
    main()
