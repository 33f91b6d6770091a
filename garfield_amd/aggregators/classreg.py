"""Class-based GAR registry: the TF graph-mode interface.

Reference: ``tensorflow_impl/rsrcs/aggregators/__init__.py:38-74`` (``_GAR`` base,
``ClassRegister`` ``register``/``itemize``/``instantiate``), the rules registered next to
it (``krum.py:165-168``: ``krum-py``, ``krum-tf``, ``krum``; ``bulyan.py:90-92``:
``bulyan-py``, ``bulyan``; ``median.py:63``; ``average.py:60``; ``average-nan.py:68``;
``averaged-median.py:67``; ``condense.py:52``) and ``tools/misc.py:83-140``
(``ClassRegister``). The legacy PS builds its rule with
``aggregators.instantiate(rule, nbworkers, nbbyzwrks, args)`` (``byzPS.py:303-309``).

The reference has up to three implementations per rule (a ``py_func`` over a ctypes
library, a pure-TF graph, a custom op). They compute the same function, so here every
name is one class over the framework's functional rules (gfx950 HIP kernels on device
tensors, the C++ thread pool on host tensors); the variant names are kept so scripts
that pick ``krum-tf`` or ``bulyan-py`` still resolve. ``args`` is the reference's list of
``"<key>:<value>"`` strings (``tools.parse_keyval``); the keys read are the ones the
reference reads (``condense``: ``ps``) plus ``m`` for Multi-Krum.

Deviation: the TF ``condense`` median is ``min(top_k(g, (n+1)//2))``, the upper median
for even n; the PyTorch rule (used here) takes the lower median (``docs/GAR_SEMANTICS.md``).
"""
from __future__ import annotations

import torch

from garfield_amd.aggregators import gars
from garfield_amd.utils.logging import UserException
from garfield_amd.utils.misc import parse_keyval


class ClassRegister:
    """Name -> class register (reference ``tools/misc.py:83-130``)."""

    def __init__(self, singular: str, optplural: str | None = None):
        self._denoms = (singular, optplural if optplural is not None else singular + "(s)")
        self._register: dict = {}

    def itemize(self):
        return self._register.keys()

    def register(self, name: str, cls) -> None:
        assert name not in self._register, f"Name {name!r} already in use while registering {cls.__name__!r}"
        self._register[name] = cls

    def instantiate(self, name: str, *args, **kwargs):
        if name not in self._register:
            cands = ", ".join(repr(k) for k in sorted(self._register))
            raise UserException(f"Unknown {self._denoms[0]} name {name!r}, expected one of: {cands}")
        return self._register[name](*args, **kwargs)


class _GAR:
    """Base class: ``__init__(nbworkers, nbbyzwrks, args)``, ``aggregate(gradients)``.

    ``gradients`` is a list of same-shape tensors (any shape: they are flattened and the
    result takes the first one's shape) or an already stacked ``[n, d]`` tensor."""

    rule_name = ""
    defaults: dict = {}

    def __init__(self, nbworkers: int, nbbyzwrks: int, args=None):
        self.nbworkers = int(nbworkers)
        self.nbbyzwrks = int(nbbyzwrks)
        self.args = parse_keyval([] if args is None else list(args), defaults=dict(self.defaults))
        self.rule = gars[self.rule_name]

    def kwargs(self) -> dict:
        return {}

    def aggregate(self, gradients):
        if isinstance(gradients, torch.Tensor):
            shape, stacked = gradients.shape[1:], gradients.reshape(gradients.shape[0], -1)
        else:
            assert len(gradients) > 0, "Empty list of gradient to aggregate"
            shape = gradients[0].shape
            stacked = torch.stack([torch.as_tensor(g).reshape(-1) for g in gradients])
        out = self.rule(gradients=stacked, f=self.nbbyzwrks, **self.kwargs())
        return out.reshape(shape)


class AverageGAR(_GAR):
    rule_name = "average"


class AverageNaNGAR(_GAR):
    rule_name = "average-nan"


class MedianGAR(_GAR):
    rule_name = "median"


class AveragedMedianGAR(_GAR):
    """beta = n - f closest to the median (``averaged-median.py:54``)."""
    rule_name = "averaged-median"

    def kwargs(self):
        return {"beta": self.nbworkers - self.nbbyzwrks}


class KrumGAR(_GAR):
    """Multi-Krum, m = n - f - 2 selected (``krum.py:93,109``) unless ``m:<int>`` is given."""
    rule_name = "krum"
    defaults = {"m": 0}

    def kwargs(self):
        m = self.args["m"] or self.nbworkers - self.nbbyzwrks - 2
        return {"m": m}


class BulyanGAR(_GAR):
    rule_name = "bulyan"


class CondenseGAR(_GAR):
    """``ps`` = probability of taking the median coordinate (``condense.py:37-40``)."""
    rule_name = "condense"
    defaults = {"ps": 0.9, "seed": -1}

    def __init__(self, nbworkers, nbbyzwrks, args=None):
        super().__init__(nbworkers, nbbyzwrks, args)
        if not 0 < self.args["ps"] <= 1:
            raise UserException(f"Invalid selection probability, got {self.args['ps']}")

    def kwargs(self):
        kw = {"p": self.args["ps"]}
        if self.args["seed"] >= 0:
            kw["seed"] = self.args["seed"]
        return kw


class TrimmedMeanGAR(_GAR):
    rule_name = "trimmed-mean"


_register = ClassRegister("GAR")
itemize = _register.itemize
register = _register.register
instantiate = _register.instantiate

for _name, _cls in (("average", AverageGAR), ("average-nan", AverageNaNGAR), ("median", MedianGAR),
                    ("averaged-median", AveragedMedianGAR), ("krum", KrumGAR), ("krum-py", KrumGAR),
                    ("krum-tf", KrumGAR), ("bulyan", BulyanGAR), ("bulyan-py", BulyanGAR),
                    ("condense", CondenseGAR), ("trimmed-mean", TrimmedMeanGAR)):
    register(_name, _cls)
