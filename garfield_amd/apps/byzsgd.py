"""ByzSGD: replicated parameter servers, some of which may be Byzantine.

Reference: ``pytorch_impl/applications/ByzSGD/trainer.py`` (ranks < num_ps are
servers ``ps:i``). Every server, each iteration: pull ``n - fw`` gradients, apply
``--gar`` (f = fw), step its optimizer, then pull ``num_ps - fps`` models from the
servers, aggregate them with ``--mar`` (f = fps) and write the result.

Deviation: the reference constructs each ``Server`` with ``num_ps=1`` (bug B5) and
so never exchanges models; here every server talks to all ``num_ps`` replicas.
``--attack`` makes servers ``rank < fps`` Byzantine (``ByzServer``) and workers
``id < fw`` Byzantine (``ByzWorker``).
"""
from __future__ import annotations

import argparse
import sys
import time

import torch

from garfield_amd import aggregators
from garfield_amd.apps.common import StepTimer, add_common, init_rpc, print_setup, seed_all
from garfield_amd.runtime.byz_server import ByzServer
from garfield_amd.runtime.byz_worker import ByzWorker
from garfield_amd.runtime.server import Server
from garfield_amd.runtime.worker import Worker
from garfield_amd.utils.logging import info


def parse(argv=None):
    p = argparse.ArgumentParser(description="ByzSGD (Garfield-MI355X)", formatter_class=argparse.RawTextHelpFormatter)
    add_common(p)
    p.add_argument("--mar", type=str, default="",
                   help="Model aggregation rule (default: --gar when fps > 0, else average)")
    p.set_defaults(num_ps=2)
    return p.parse_args(argv)


def run_server(a, world_size, results: dict | None = None):
    gar = aggregators.get(a.gar)
    mar = aggregators.get(a.mar or (a.gar if a.fps > 0 else "average"))
    args = (a.rank, world_size, a.num_workers, a.num_ps, a.fw, a.fps, "worker:", "ps:", a.batch, a.model, a.dataset,
            a.optimizer)
    if a.attack and a.rank < a.fps:
        ps = ByzServer(*args, a.attack, train_size=a.train_size, device=a.device, rpc_timeout=a.rpc_timeout,
                       **a.opt_args)
    else:
        ps = Server(*args, a.train_size, device=a.device, rpc_timeout=a.rpc_timeout, **a.opt_args)
    start = time.time()
    acc = None
    for i in range(a.num_iter):
        with StepTimer(a.bench) as t:
            grads = ps.get_gradients(i, a.num_workers - a.fw)
            ps.update_model(gar(gradients=grads, f=a.fw))
            models = ps.get_models(a.num_ps - a.fps)
            ps.write_model(mar(gradients=models, f=a.fps))
        if a.bench:
            info(f"Training step {i} takes {t.seconds:.4f} s, consumed bandwidth {t.gbit:.4f} Gbits")
        if (a.acc_freq and i % a.acc_freq == 0) or i == a.num_iter - 1:
            acc = ps.compute_binary_accuracy() if a.dataset == "pima" else ps.compute_accuracy()
            info(f"Iteration: {i} Accuracy: {acc:.2f} Time: {time.time() - start:.2f}")
    if results is not None:
        results["accuracy"] = acc
    return ps


def main(argv=None, results: dict | None = None):
    a = parse(argv)
    world_size = a.num_workers + a.num_ps
    if a.rank == 0:
        print_setup(a.rank, workers=a.num_workers, servers=a.num_ps, fw=a.fw, fps=a.fps, gar=a.gar,
                    mar=a.mar or "(auto)", dataset=a.dataset, model=a.model, batch=a.batch, optimizer=a.optimizer,
                    opt_args=a.opt_args)
    seed_all(1234)
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
