"""Decentralised LEARN on collectives: every rank is a node (worker + server) with its
OWN model replica; the n-to-n pulls of the RPC form become all-gathers.

Reference iteration (``pytorch_impl/applications/LEARN/trainer.py:244-258``, with the
average agreement of ``:208-222``):

1. every node computes a gradient on its own batch, pulls the gradients of the
   others (``get_gradients(i, n - f)``) and aggregates them with the GAR (f);
2. non-IID data: ``ceil(log2(i + 1))`` rounds of exchanging the aggregated gradients
   (``get_aggr_grads``) and aggregating them again;
3. the node applies the result with its own optimizer (``update_model``);
4. it pulls every node's model (``get_models(n - f)``), aggregates them and writes
   the result (``write_model``).

Here each pull is ONE ``all_gather_into_tensor`` of a reference-layout flat vector
per node into an ``[n, d]`` device buffer that is directly the GAR input (HIP kernels
on the GPU, the C++ thread pool on the CPU). Semantics kept from the reference:
Byzantine nodes are the ranks ``< f`` when ``attack`` is set, and only their
GRADIENTS are attacked (``ByzWorker``; their servers are honest ``Server``s); each
node keeps its own optimizer state. The RPC form's "fastest n - f" quorum has no
synchronous counterpart: all n rows are gathered every time, which is the RPC
form's result when every node answers (test: ``tests/test_learn_cc_cpu.py``).
"""
from __future__ import annotations

import math

import torch

from garfield_amd import aggregators
from garfield_amd.parallel.comm import DistContext, all_gather_rows
from garfield_amd.runtime.byz_worker import ByzWorker
from garfield_amd.runtime.server import Server
from garfield_amd.runtime.worker import Worker
from garfield_amd.utils.flat import padded


class CollectiveLearnNode:
    """One LEARN node per rank (see the module docstring)."""

    def __init__(self, ctx: DistContext, model: str, dataset: str, batch: int, loss: str, optimizer: str,
                 opt_args: dict | None = None, gar: str = "average", f: int = 0, attack: str = "",
                 non_iid: bool = False, mar: str | None = None, train_size: int | None = None):
        self.ctx = ctx
        self.n, self.rank, self.f = ctx.world_size, ctx.rank, f
        self.non_iid = bool(non_iid)
        dev = ctx.device
        n, r = self.n, self.rank
        if attack and r < f:
            self.worker = ByzWorker(r, n, n, batch, model, dataset, loss, attack, f, train_size, device=dev,
                                    register=False)
        else:
            self.worker = Worker(r, n, n, batch, model, dataset, loss, train_size, device=dev, register=False)
        # world_size 0: a standalone server (no RPC peers); it owns this node's model + optimizer
        self.ps = Server(r, 0, n, 0, f, f, "node:", "node:", batch, model, dataset, optimizer, train_size,
                         device=dev, register=False, **(opt_args or {}))
        self.d = self.ps.flat.d
        ld = padded(self.d)
        self._bufs = {name: torch.zeros((n, ld), dtype=torch.float32, device=dev) for name in ("grad", "aggr", "model")}
        self.gar = aggregators.get(gar)
        self.mar = aggregators.get(mar or gar)
        self.step_count = 0

    def exchange(self, name: str, vec: torch.Tensor) -> list:
        """All-gather ``vec`` (this node's reference-layout vector) from every node: the
        collective form of a pull from all n nodes. Returns the n rows in rank order."""
        buf = self._bufs[name]
        buf[self.rank, : self.d].copy_(vec)
        if self.n > 1:
            all_gather_rows(buf, self.rank)
        return [buf[i, : self.d] for i in range(self.n)]

    def _aggregate(self, rule, rows: list) -> torch.Tensor:
        return rule(gradients=torch.stack(rows) if rows[0].device.type == "cpu" else rows, f=self.f).float()

    def step(self, i: int | None = None) -> float:
        i = self.step_count if i is None else i
        model_vec = self.ps.flat.reference_vector()
        grad, loss = self.worker.compute_local_gradient(i, model_vec)
        aggr = self._aggregate(self.gar, self.exchange("grad", grad.float()))
        if self.non_iid:
            for _ in range(math.ceil(math.log2(i + 1))):
                aggr = self._aggregate(self.gar, self.exchange("aggr", aggr))
        self.ps.latest_aggr_grad = aggr
        self.ps.update_model(aggr)
        models = self.exchange("model", self.ps.flat.reference_vector())
        self.ps.write_model(self._aggregate(self.mar, models))
        self.step_count = i + 1
        return float(loss)

    def model_vector(self) -> torch.Tensor:
        return self.ps.flat.reference_vector()

    def accuracy(self, binary: bool = False) -> float:
        return self.ps.compute_binary_accuracy() if binary else self.ps.compute_accuracy()
