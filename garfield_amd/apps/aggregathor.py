"""AggregaThor: one parameter server, n workers, robust GAR on the gradients.

Reference: ``pytorch_impl/applications/Aggregathor/trainer.py`` (same flags, same
rank convention: ranks < num_ps are servers ``ps:i``, the others workers
``worker:i``). Per iteration the server pulls ``n - fw`` gradients over RPC
(fastest-first), aggregates them with ``--gar`` (HIP kernels on the server GPU)
and applies its optimizer; accuracy is evaluated every ``--acc_freq`` iterations.

Run one process per node, e.g. on one host::

    python -m garfield_amd.apps.aggregathor --rank 0 --num_workers 2 --model mlp --num_iter 50 &
    python -m garfield_amd.apps.aggregathor --rank 1 --num_workers 2 --model mlp --num_iter 50 &
    python -m garfield_amd.apps.aggregathor --rank 2 --num_workers 2 --model mlp --num_iter 50

For the one-process-per-GPU collective form (RCCL), see ``garfield_cc``.
"""
from __future__ import annotations

import argparse
import sys
import time

import torch

from garfield_amd import aggregators
from garfield_amd.apps.common import StepTimer, add_common, init_rpc, print_setup, seed_all
from garfield_amd.runtime import tools
from garfield_amd.runtime.byz_worker import ByzWorker
from garfield_amd.runtime.server import Server
from garfield_amd.runtime.worker import Worker
from garfield_amd.utils.logging import info

CIFAR_NUM_SAMPLES = 50000


def parse(argv=None):
    p = argparse.ArgumentParser(description="AggregaThor (Garfield-MI355X)",
                                formatter_class=argparse.RawTextHelpFormatter)
    return add_common(p).parse_args(argv)


def run_server(a, world_size, results: dict | None = None):
    gar = aggregators.get(a.gar)
    ps = Server(a.rank, world_size, a.num_workers, 1, a.fw, a.fps, "worker:", "ps:", a.batch, a.model, a.dataset,
                a.optimizer, a.train_size, device=a.device, rpc_timeout=a.rpc_timeout, **a.opt_args)
    lr = float(a.opt_args.get("lr", 0.1))
    iter_per_epoch = max(CIFAR_NUM_SAMPLES // (a.num_workers * a.batch), 1)
    start = time.time()
    acc = None
    for i in range(a.num_iter):
        if i % (iter_per_epoch * 30) == 0 and i != 0:
            lr *= 0.2
            tools.adjust_learning_rate(ps.optimizer, lr)
        with StepTimer(a.bench) as t:
            grads = ps.get_gradients(i, a.num_workers - a.fw)
            aggr = gar(gradients=grads, f=a.fw)
            ps.update_model(aggr)
        if a.bench:
            info(f"Training step {i} takes {t.seconds:.4f} s, consumed bandwidth {t.gbit:.4f} Gbits")
        if (a.acc_freq and i % a.acc_freq == 0) or i == a.num_iter - 1:
            acc = ps.compute_binary_accuracy() if a.dataset == "pima" else ps.compute_accuracy()
            info(f"Iteration: {i} Accuracy: {acc:.2f} Time: {time.time() - start:.2f}")
    if results is not None:
        results["accuracy"] = acc
        results["model"] = ps.flat.reference_vector().cpu()
    return ps


def main(argv=None, results: dict | None = None):
    a = parse(argv)
    world_size = a.num_workers + a.num_ps
    if a.rank == 0:
        print_setup(a.rank, workers=a.num_workers, servers=a.num_ps, fw=a.fw, fps=a.fps, gar=a.gar,
                    dataset=a.dataset, model=a.model, batch=a.batch, loss=a.loss, optimizer=a.optimizer,
                    opt_args=a.opt_args, bench=a.bench, log=a.log)
    seed_all(1234)
    if a.bench:
        torch.backends.cudnn.benchmark = True
    if a.rank < a.num_ps:
        init_rpc(f"ps:{a.rank}", a.rank, world_size, a.master, a.port, a.rpc_timeout)
        run_server(a, world_size, results)
    else:
        init_rpc(f"worker:{a.rank - a.num_ps}", a.rank, world_size, a.master, a.port, a.rpc_timeout)
        wid = a.rank - a.num_ps
        if a.attack and wid < a.fw:
            ByzWorker(a.rank, world_size, a.num_workers, a.batch, a.model, a.dataset, a.loss, a.attack, a.fw,
                      a.train_size, device=a.device)
        else:
            Worker(a.rank, world_size, a.num_workers, a.batch, a.model, a.dataset, a.loss, a.train_size,
                   device=a.device)
    import torch.distributed.rpc as rpc

    rpc.shutdown()


if __name__ == "__main__":
    main(sys.argv[1:])
