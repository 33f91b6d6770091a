"""TF-transport aggregator dispatcher (reference
``tensorflow_impl/rsrcs/aggregator_tf/aggregator.py:10-30`` and the numpy GARs next to
it: ``average.py``, ``median.py``, ``krum.py`` (m = n − f − 2), ``brute.py``,
``aksel.py``, ``condense.py``, ``bulyan.py``).

Here every name runs the framework's GARs (gfx950 HIP kernels for device tensors, the
C++ thread-pool implementation for host tensors); ``native`` is accepted for API
parity and is always on. Inputs may be numpy arrays or tensors; the result has the
type of the first input. Extra names: ``TrimmedMean``, ``AverageNan``,
``AveragedMedian``.
"""
from __future__ import annotations

import numpy as np
import torch

from garfield_amd import aggregators

_RULES = {"Average": "average", "Median": "median", "Krum": "krum", "Brute": "brute", "Aksel": "aksel",
          "Condense": "condense", "Bulyan": "bulyan", "TrimmedMean": "trimmed-mean",
          "AverageNan": "average-nan", "AveragedMedian": "averaged-median"}


class Aggregator_tf:
    def __init__(self, agg: str = "Average", nb_worker: int = 0, nb_byz_worker: int = 0, native: bool = False,
                 device=None):
        if agg not in _RULES:
            raise AssertionError(f"Aggregation not implemented: {agg!r}; available: {sorted(_RULES)}")
        self.name = agg
        self.rule = aggregators.gars[_RULES[agg]]
        self.nb_worker = nb_worker
        self.f = nb_byz_worker
        self.native = native
        self.device = device

    def _kwargs(self, n: int) -> dict:
        kw = {"f": self.f}
        if self.name == "Krum":
            kw["m"] = max(n - self.f - 2, 1)
        return kw

    def aggregate(self, gradients):
        if len(gradients) == 0:
            raise AssertionError("Empty list of gradient to aggregate")
        as_numpy = isinstance(gradients[0], np.ndarray)
        rows = [torch.from_numpy(np.asarray(g, dtype=np.float32)) if isinstance(g, np.ndarray) else g
                for g in gradients]
        if self.device is not None:
            rows = [r.to(self.device, non_blocking=True) for r in rows]
        if len(rows) == 1 and self.name in ("Average", "Median"):
            out = rows[0].clone()
        else:
            out = self.rule(gradients=rows, **self._kwargs(len(rows)))
        return out.cpu().numpy() if as_numpy else out


Aggregator = Aggregator_tf
