"""Reference import name ``native`` (pybind modules ``native.krum``, ``native.bulyan``,
``native.median``, ``native.brute`` with ``aggregate(list, f[, m])``; reference
``pytorch_impl/libs/native/__init__.py:139-141``), backed by the HIP / C++ kernels."""
from types import SimpleNamespace as _NS

from garfield_amd.ops import gar as _gar

krum = _NS(aggregate=lambda inputs, f, m: _gar.krum(list(inputs), f, m))
bulyan = _NS(aggregate=lambda inputs, f, m: _gar.bulyan(list(inputs), f, m))
median = _NS(aggregate=lambda inputs: _gar.median(list(inputs)))
brute = _NS(aggregate=lambda inputs, f: _gar.brute(list(inputs), f))
trimmed_mean = _NS(aggregate=lambda inputs, f: _gar.trimmed_mean(list(inputs), f))
