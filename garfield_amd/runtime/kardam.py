"""Kardam-style Lipschitz filter of the legacy "smart" protocol.

Reference: ``tensorflow_impl/applications/Garfield_legacy/byzWorker.py:399-426``.
After each update a worker estimates the empirical Lipschitz coefficient of the
model it received, ``L_t = ||g_t - g_{t-1}|| / ||θ_t - θ_{t-1}||``, keeps a window of
the last 100 values (trimmed to the newest 50 when full, "crucial in
performance"), and compares ``L_t`` with the ``100 (n - f) / n`` percentile of the
window, where n / f are the number of PS replicas and declared Byzantine ones; it
also bounds the model drift by ``lr ||g|| ((3T + 2)(n_w - f_w) / (4 f_w) + 2 ((t-1) mod T))``
when Byzantine workers are declared. The reference only prints both tests; here
``observe`` returns them, and ``accept`` is the Lipschitz test's verdict (callers
decide whether to act on it).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class LipschitzStats:
    lipschitz: float
    threshold: float
    accept: bool
    drift: float | None = None
    drift_bound: float | None = None


class LipschitzFilter:
    def __init__(self, num_ps: int, num_byz_ps: int, window: int = 100, keep: int = 50):
        if num_ps < 1 or not (0 <= num_byz_ps < num_ps):
            raise ValueError("need num_ps >= 1 and 0 <= num_byz_ps < num_ps")
        self.q = 100.0 * (num_ps - num_byz_ps) / num_ps
        self.window, self.keep = window, keep
        self.history: list[float] = []
        self._grad = None
        self._model = None
        self.rejected = 0
        self.observed = 0

    def observe(self, grad: torch.Tensor, model: torch.Tensor, drift_args: dict | None = None) -> LipschitzStats | None:
        """Record the gradient computed at ``model``; returns None on the first call."""
        grad = grad.detach().reshape(-1).double()
        model = model.detach().reshape(-1).double()
        stats = None
        if self._grad is not None:
            den = float((model - self._model).norm())
            lip = float((grad - self._grad).norm()) / den if den > 0 else float("inf")
            self.history.append(lip)
            thr = float(np.percentile(np.asarray(self.history), self.q))
            if len(self.history) >= self.window:
                self.history = self.history[-self.keep:]
            stats = LipschitzStats(lip, thr, lip <= thr)
            if drift_args and drift_args.get("num_byz_workers", 0) > 0:
                a = drift_args
                T, it = a["T"], a["iteration"]
                f, n = a["num_byz_workers"], a["num_workers"]
                stats.drift = den
                stats.drift_bound = a["lr"] * float(grad.norm()) * (((3 * T + 2) * (n - f)) / (4 * f)
                                                                    + 2 * ((it - 1) % T))
            self.observed += 1
            self.rejected += int(not stats.accept)
        self._grad, self._model = grad, model
        return stats
