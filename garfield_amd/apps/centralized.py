"""Centralized baseline: one process, one worker, one server, no RPC.

Reference: ``pytorch_impl/applications/Centralized/trainer.py:150-186``, which
builds ``Server(0, 1, 1, 1, ...)`` with ``world_size > 0`` and therefore calls
``rpc.remote`` without ``init_rpc`` (bug B6). Here the server is built with
``world_size=0`` and the worker is called directly.
"""
from __future__ import annotations

import argparse
import sys
import time

from garfield_amd import aggregators
from garfield_amd.apps.common import StepTimer, add_common, print_setup, seed_all
from garfield_amd.runtime.server import Server
from garfield_amd.runtime.worker import Worker
from garfield_amd.utils.logging import info


def parse(argv=None):
    p = argparse.ArgumentParser(description="Centralized training (Garfield-MI355X)")
    add_common(p, ps=False)
    return p.parse_args(argv)


def main(argv=None, results: dict | None = None):
    a = parse(argv)
    print_setup(0, dataset=a.dataset, model=a.model, batch=a.batch, loss=a.loss, optimizer=a.optimizer,
                opt_args=a.opt_args)
    seed_all(1234)
    wrk = Worker(1, 2, 1, a.batch, a.model, a.dataset, a.loss, a.train_size, device=a.device)
    ps = Server(0, 0, 1, 0, 0, 0, "worker:", "ps:", a.batch, a.model, a.dataset, a.optimizer, a.train_size,
                device=a.device, **a.opt_args)
    gar = aggregators.get("average")
    start = time.time()
    acc = None
    for i in range(a.num_iter):
        with StepTimer(a.bench) as t:
            grad, loss = wrk.compute_local_gradient(i, ps.flat.reference_vector())
            ps.update_model(gar(gradients=[grad], f=0))
        if a.log:
            info(f"Iteration {i} loss {float(loss):.4f}")
        if a.bench:
            info(f"Training step {i} takes {t.seconds:.4f} s")
        if (a.acc_freq and i % a.acc_freq == 0) or i == a.num_iter - 1:
            acc = ps.compute_binary_accuracy() if a.dataset == "pima" else ps.compute_accuracy()
            info(f"Iteration: {i} Accuracy: {acc:.2f} Time: {time.time() - start:.2f}")
    if results is not None:
        results["accuracy"] = acc
    return acc


if __name__ == "__main__":
    main(sys.argv[1:])
