"""GAR registry with the reference's calling contract.

Reference: ``pytorch_impl/libs/aggregators/__init__.py:15-97``.

* Every rule is called with keyword arguments only: ``gradients`` (non-empty list
  of 1-D tensors, or an ``[n, d]`` tensor), ``f`` and optional ``m`` / ``mode`` /
  ``p`` / ``beta`` / ``seed``; unknown keyword arguments are ignored.
* A rule never returns a tensor aliasing one of its inputs.
* ``make_gar`` attaches ``check``, ``checked``, ``unchecked``, ``upper_bound`` and
  ``influence``; the default callable is ``checked`` unless Python runs with ``-O``.
* ``gars`` maps names to rules; every rule is also registered as
  ``"native-<name>"`` (the reference registers the native C++/CUDA variants under
  that prefix, e.g. ``krum.py:159-166``). Here every name runs the native
  implementation (gfx950 HIP on GPU tensors, C++ thread pool on CPU tensors).
* New rules (absent from the PyTorch reference): ``trimmed-mean``, and the TF-only
  ``average-nan`` and ``averaged-median``.
"""
from __future__ import annotations

import importlib

from garfield_amd.utils.logging import UserException, warning

gars: dict = {}


def make_gar(unchecked, check, upper_bound=None, influence=None, name: str = "?"):
    def checked(**kwargs):
        message = check(**kwargs)
        if message is not None:
            raise UserException(f"Aggregation rule {name!r} cannot be used with the given parameters: {message}")
        return unchecked(**kwargs)

    func = checked if __debug__ else unchecked

    def rule(**kwargs):
        return func(**kwargs)

    rule.__name__ = name.replace("-", "_")
    rule.__doc__ = unchecked.__doc__
    rule.check = check
    rule.checked = checked
    rule.unchecked = unchecked
    rule.upper_bound = upper_bound
    rule.influence = influence
    rule.gar_name = name
    return rule


def register(name, unchecked, check, upper_bound=None, influence=None):
    if name in gars:
        warning(f"Unable to register {name!r} GAR: name already in use")
        return
    gars[name] = make_gar(unchecked, check, upper_bound=upper_bound, influence=influence, name=name)


_MODULES = ("average", "median", "krum", "bulyan", "brute", "aksel", "condense", "trimmed_mean",
            "average_nan", "averaged_median")
for _m in _MODULES:
    importlib.import_module(f"garfield_amd.aggregators.{_m}")

for _name in list(gars):
    _g = gars[_name]
    register("native-" + _name, _g.unchecked, _g.check, _g.upper_bound, _g.influence)

for _name, _rule in gars.items():
    globals()[_name.replace("-", "_")] = _rule


def get(name: str):
    try:
        return gars[name]
    except KeyError:
        raise UserException(f"Unknown aggregation rule {name!r}; available: {sorted(gars)}") from None

# TF graph-mode class interface (``aggregators.instantiate(name, nbworkers, nbbyzwrks, args)``)
from garfield_amd.aggregators.classreg import instantiate, itemize  # noqa: E402,F401
