"""RPC transfer benchmark (reference ``pytorch_impl/applications/benchmarks/rpc_bench.py:96-116``).

Each of ``--n`` nodes hosts a Worker and a Server. Each server's model is replaced
by ``torch.rand(d)``, and ``get_fake_models()`` (an all-to-all pull) is timed.
The output is one JSON line per iteration on every rank:
``{"d":…, "n":…, "transfer_s":…, "total_s":…, "GBps":…}``. Launch one process per
node (``--rank``), or use ``--spawn`` to start all ``n`` locally on 127.0.0.1.
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from garfield_amd.apps.common import init_rpc


def run(rank: int, n: int, d: int, num_iter: int, master: str, port: int, device: str | None, out=None) -> list[dict]:
    import torch.distributed.rpc as rpc

    from garfield_amd.runtime.server import Server
    from garfield_amd.runtime.worker import Worker

    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    init_rpc(f"node:{rank}", rank, n, master, port)
    Worker(rank, n, n, 32, "cnn", "mnist", "nll", device=dev)
    ps = Server(rank, n, n, n, 0, 0, "node:", "node:", 32, "cnn", "mnist", "sgd", device=dev, lr=0.1)
    ps.fake_model = torch.rand(d, device=dev)
    # barrier: every peer has installed its fake model (the reference sleeps 5 s, :104)
    deadline = time.time() + 120
    while not all(m.numel() == d for m in ps.get_fake_models()):
        if time.time() > deadline:
            raise TimeoutError("peers did not install their fake models")
        time.sleep(0.05)
    rows = []
    for _ in range(num_iter):
        ts = time.perf_counter()
        ta = time.perf_counter()
        models = ps.get_fake_models()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        tf = time.perf_counter()
        assert len(models) == n and all(m.numel() == d for m in models)
        row = {"d": d, "n": n, "rank": rank, "transfer_s": tf - ta, "total_s": time.perf_counter() - ts,
               "GBps": 4.0 * d * n / max(tf - ta, 1e-9) / 1e9}
        rows.append(row)
        print(json.dumps(row), flush=True)
    rpc.shutdown()
    if out is not None:
        out.put(rows)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--master", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=27800)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--d", type=int, default=100000)
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--num_iter", type=int, default=10)
    ap.add_argument("--device", default=None)
    ap.add_argument("--spawn", action="store_true", help="start all n nodes locally")
    a = ap.parse_args(argv)
    if not a.spawn:
        return run(a.rank, a.n, a.d, a.num_iter, a.master, a.port, a.device)
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=run, args=(r, a.n, a.d, a.num_iter, a.master, a.port, a.device, q))
             for r in range(a.n)]
    for p in procs:
        p.start()
    rows = []
    while len(rows) < len(procs):
        try:
            rows.append(q.get(timeout=1.0))
        except Exception:  # queue.Empty
            bad = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if bad:
                for p in procs:
                    p.kill()
                raise SystemExit(f"a node failed (exit codes {bad})")
    for p in procs:
        p.join()
    return [r for rs in rows for r in rs]


if __name__ == "__main__":
    main()
