"""GAR micro-benchmark: latency and achieved bandwidth of every rule.

Reference: ``pytorch_impl/applications/benchmarks/gar_bench.py:41-89`` (one
wall-clock call per GAR on ``torch.rand(d)`` CUDA tensors, sweeping n, d and f,
bulyan skipped for n > 23). Here each rule is timed with HIP events over several
back-to-back calls on an ``[n, d]`` gradient buffer (the engine's exchange
layout), optionally also from a list of separate tensors, and the effective
bandwidth (gradient bytes read / time) is reported next to the ~6.3 TB/s HBM3E
streaming ceiling of one MI355X.

Usage::

    python -m garfield_amd.apps.gar_bench --n 8 16 32 64 --d 23528522 --dtype bf16
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from garfield_amd.ops import gar

RULES = ["average", "krum", "bulyan", "median", "trimmed-mean", "averaged-median", "aksel", "brute", "condense",
         "average-nan"]


def default_f(rule: str, n: int) -> int | None:
    if rule in ("average", "average-nan", "median"):
        return None
    if rule == "bulyan":
        f = (n - 3) // 4
    elif rule == "krum":
        f = (n - 3) // 2
    elif rule == "condense":
        f = (n - 2) // 2
    else:
        f = (n - 1) // 2
    f = min(f, 2) if rule != "bulyan" else min(f, 3)
    return f if f >= 1 else None


def bench_rule(rule, G, f, iters, warmup):
    kw = {} if f is None else {"f": f}
    if rule == "averaged-median":
        kw = {"f": f or 0}
    for _ in range(warmup):
        gar.aggregate(rule, G, **kw)
    dev = G.device if isinstance(G, torch.Tensor) else G[0].device
    if dev.type == "cuda":
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            gar.aggregate(rule, G, **kw)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters
    t0 = time.perf_counter()
    for _ in range(iters):
        gar.aggregate(rule, G, **kw)
    return 1000 * (time.perf_counter() - t0) / iters


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--n", type=int, nargs="+", default=[8, 16, 32, 64])
    p.add_argument("--d", type=int, nargs="+", default=[11173962, 23528522])
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp16"])
    p.add_argument("--rules", nargs="+", default=RULES)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    p.add_argument("--list-input", action="store_true", help="pass a list of n tensors instead of [n, d]")
    a = p.parse_args(argv)
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[a.dtype]
    for d in a.d:
        for n in a.n:
            ld = ((d + 63) // 64) * 64
            G = torch.randn(n, ld, device=a.device, dtype=dt)[:, :d]
            inp = [G[i].clone() for i in range(n)] if a.list_input else G
            for rule in a.rules:
                f = default_f(rule, n)
                if rule in ("krum", "bulyan", "brute", "aksel", "trimmed-mean", "condense") and f is None:
                    continue
                if rule == "brute" and n > 20:
                    continue
                ms = bench_rule(rule, inp, f, a.iters, a.warmup)
                nbytes = n * d * G.element_size()
                print(json.dumps({"rule": rule, "n": n, "d": d, "f": f, "dtype": a.dtype, "ms": round(ms, 4),
                                  "GBps_read": round(nbytes / ms / 1e6, 1)}), flush=True)
            del G, inp
            if a.device == "cuda":
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
