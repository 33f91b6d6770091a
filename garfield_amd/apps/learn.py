"""LEARN: decentralised Byzantine-resilient learning (every node is worker + server).

Reference: ``pytorch_impl/applications/LEARN/trainer.py:208-258``. Node ``node:i``
hosts a ``Worker`` and a ``Server``; each iteration it pulls ``n - f`` gradients,
aggregates them (GAR, f), optionally runs the ``ceil(log2(i+1))``-round average
agreement on aggregated gradients (``--non_iid``), updates, then pulls ``n - f``
models, aggregates and writes them. The reference's ``sleep(20)`` start barrier is
replaced by the blocking peer-registration handshake of ``Server.get_rrefs``.
"""
from __future__ import annotations

import argparse
import math
import sys
import time

from garfield_amd import aggregators
from garfield_amd.apps.common import StepTimer, add_common, init_rpc, print_setup, seed_all
from garfield_amd.runtime.byz_worker import ByzWorker
from garfield_amd.runtime.server import Server
from garfield_amd.runtime.worker import Worker
from garfield_amd.utils.logging import info


def parse(argv=None):
    p = argparse.ArgumentParser(description="LEARN (Garfield-MI355X)", formatter_class=argparse.RawTextHelpFormatter)
    add_common(p, ps=False)
    p.add_argument("--num_nodes", type=int, default=3)
    p.add_argument("--f", type=int, default=0, help="Number of declared Byzantine nodes.")
    p.add_argument("--non_iid", type=int, default=0, help="1: run the log2(t) average-agreement rounds.")
    p.add_argument("--collective", type=int, default=0,
                   help="1: torch.distributed collectives (RCCL over xGMI on GPUs, gloo on CPU) instead of RPC; "
                        "every pull is one all-gather (parallel/learn.py)")
    p.add_argument("--backend", default=None, help="collective backend (default: nccl=RCCL on GPU, gloo on CPU)")
    p.set_defaults(port=29700)
    return p.parse_args(argv)


def avg_agree(ps, gar, aggr_grad, rounds: int, num_wait: int, f: int):
    """Average agreement: ``rounds`` rounds of exchanging + aggregating aggregated gradients."""
    for _ in range(rounds):
        ps.latest_aggr_grad = aggr_grad
        aggr_grad = gar(gradients=ps.get_aggr_grads(num_wait), f=f)
    return aggr_grad


def main(argv=None, results: dict | None = None, progress=None):
    """Run one LEARN node; ``progress(done, total)`` is called after every iteration
    (the web demo's progress queue, reference ``LEARN/demo.py:225-235``)."""
    a = parse(argv)
    n, f = a.num_nodes, a.f
    if a.rank == 0:
        print_setup(a.rank, nodes=n, f=f, gar=a.gar, dataset=a.dataset, model=a.model, batch=a.batch,
                    optimizer=a.optimizer, opt_args=a.opt_args, non_iid=a.non_iid)
    seed_all(1234)
    if a.collective:
        return _main_collective(a, results, progress)
    init_rpc(f"node:{a.rank}", a.rank, n, a.master, a.port, a.rpc_timeout)
    gar = aggregators.get(a.gar)
    if a.attack and a.rank < f:
        ByzWorker(a.rank, n, n, a.batch, a.model, a.dataset, a.loss, a.attack, f, a.train_size, device=a.device)
    else:
        Worker(a.rank, n, n, a.batch, a.model, a.dataset, a.loss, a.train_size, device=a.device)
    ps = Server(a.rank, n, n, n, f, f, "node:", "node:", a.batch, a.model, a.dataset, a.optimizer, a.train_size,
                device=a.device, rpc_timeout=a.rpc_timeout, **a.opt_args)
    start = time.time()
    acc = None
    for i in range(a.num_iter):
        with StepTimer(a.bench) as t:
            aggr = gar(gradients=ps.get_gradients(i, n - f), f=f)
            if a.non_iid:
                aggr = avg_agree(ps, gar, aggr, math.ceil(math.log2(i + 1)), n - f, f)
            ps.latest_aggr_grad = aggr
            ps.update_model(aggr)
            ps.write_model(gar(gradients=ps.get_models(n - f), f=f))
        if a.bench:
            info(f"Training step {i} takes {t.seconds:.4f} s, consumed bandwidth {t.gbit:.4f} Gbits")
        if (a.acc_freq and i % a.acc_freq == 0) or i == a.num_iter - 1:
            acc = ps.compute_binary_accuracy() if a.dataset == "pima" else ps.compute_accuracy()
            info(f"Node {a.rank} iteration: {i} Accuracy: {acc:.2f} Time: {time.time() - start:.2f}")
        if progress is not None:
            progress(i + 1, a.num_iter)
    if results is not None:
        results["accuracy"] = acc
    info(f"Node {a.rank} model checksum {float(ps.flat.reference_vector().double().sum()):.12e}")
    import torch.distributed.rpc as rpc

    rpc.shutdown()



def _main_collective(a, results, progress):
    """LEARN with every pull as an all-gather (one node per rank; ``torchrun`` or --rank/--master)."""
    import os

    import torch

    from garfield_amd.parallel.comm import init_distributed, shutdown
    from garfield_amd.parallel.learn import CollectiveLearnNode

    if "WORLD_SIZE" not in os.environ:
        os.environ.update(RANK=str(a.rank), WORLD_SIZE=str(a.num_nodes), LOCAL_RANK=os.environ.get(
            "LOCAL_RANK", str(a.rank % max(torch.cuda.device_count(), 1))), MASTER_ADDR=a.master,
            MASTER_PORT=str(a.port))
    ctx = init_distributed(backend=a.backend, device=a.device)
    node = CollectiveLearnNode(ctx, a.model, a.dataset, a.batch, a.loss, a.optimizer, a.opt_args, a.gar, a.f,
                               a.attack, bool(a.non_iid), train_size=a.train_size)
    start = time.time()
    acc = None
    for i in range(a.num_iter):
        with StepTimer(a.bench) as t:
            loss = node.step(i)
        if a.bench:
            info(f"Training step {i} takes {t.seconds:.4f} s")
        if a.log:
            info(f"Node {ctx.rank} iteration {i} loss {loss:.4f}")
        if (a.acc_freq and i % a.acc_freq == 0) or i == a.num_iter - 1:
            acc = node.accuracy(binary=a.dataset == "pima")
            info(f"Node {ctx.rank} iteration: {i} Accuracy: {acc:.2f} Time: {time.time() - start:.2f}")
        if progress is not None:
            progress(i + 1, a.num_iter)
    if results is not None:
        results["accuracy"] = acc
    info(f"Node {ctx.rank} model checksum {float(node.model_vector().double().sum()):.12e}")
    shutdown(ctx)
    return acc


if __name__ == "__main__":
    main(sys.argv[1:])
