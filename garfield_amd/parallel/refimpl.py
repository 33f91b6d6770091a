"""The reference's training step, run as-is on PyTorch-ROCm: the self-measured baseline.

BASELINE.md ("What we will measure on MI355X", item (a)) defines the baseline this
framework must beat, since the reference publishes no numbers: the reference
algorithms executed on the same GPU. This module reproduces the AggregaThor PS step
(``pytorch_impl/applications/Aggregathor/trainer.py:231-243``) for ``k`` logical
workers in one process:

1. for each worker: ``zero_grad`` → forward/backward → ``torch.cat([p.grad.view(-1)])``
   (``garfieldpp/worker.py:86-95``, minus the RPC/CPU hop, which would only slow it);
2. Multi-Krum exactly as ``pytorch_impl/libs/aggregators/krum.py:31-82``: one
   ``sub().norm().item()`` per pair (a host sync each), host-side sorting of the
   scores, and ``sum(grads[:m]) / m``;
3. the aggregate is written into ``p.grad`` and ``torch.optim.SGD`` steps
   (``garfieldpp/server.py:245-258``).

The same bf16 autocast as the engine is used, so the comparison isolates the
framework (exchange layout, HIP GARs, fused update, graphs), not the precision.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.nn as nn


def reference_krum(gradients: list, f: int, m: int | None = None) -> torch.Tensor:
    n = len(gradients)
    m = n - f - 2 if m is None else m
    distances = []
    for x in range(n - 1):
        for y in range(x + 1, n):
            dist = gradients[x].sub(gradients[y]).norm().item()
            distances.append(dist if math.isfinite(dist) else math.inf)

    def d(i, j):
        a, b = min(i, j), max(i, j)
        return distances[(2 * n - a - 3) * a // 2 + b - 1]

    scores = []
    for i in range(n):
        dists = sorted(d(i, j) for j in range(n) if j != i)
        scores.append((sum(dists[: n - f - 1]), i))
    scores.sort(key=lambda s: s[0])
    return sum(gradients[i] for _, i in scores[:m]).div_(m)


class ReferenceStyleDP:
    def __init__(self, model: nn.Module, loss_fn, device, workers: int, f: int, lr: float, momentum: float = 0.9,
                 weight_decay: float = 5e-4, autocast_dtype=torch.bfloat16, gar: str = "krum"):
        self.model = model.to(device)
        self.loss_fn = loss_fn
        self.device = torch.device(device)
        self.k, self.f, self.gar = workers, f, gar
        self.params = [p for p in self.model.parameters() if p.requires_grad]
        self.opt = torch.optim.SGD(self.params, lr=lr, momentum=momentum, weight_decay=weight_decay)
        self.autocast_dtype = autocast_dtype

    def step(self, batches) -> torch.Tensor:
        amp = (torch.autocast("cuda", dtype=self.autocast_dtype)
               if self.autocast_dtype is not None and self.device.type == "cuda" else contextlib.nullcontext())
        grads, losses = [], []
        self.model.train()
        for x, y in batches[: self.k]:
            self.opt.zero_grad()
            with amp:
                loss = self.loss_fn(self.model(x), y)
            loss.backward()
            grads.append(torch.cat([p.grad.view(-1) for p in self.params]))
            losses.append(loss.detach())
        agg = reference_krum(grads, self.f) if self.gar == "krum" else sum(grads).div_(len(grads))
        pos = 0
        for p in self.params:
            n = p.numel()
            p.grad.copy_(agg[pos:pos + n].view_as(p))
            pos += n
        self.opt.step()
        return torch.stack(losses).float().mean()
