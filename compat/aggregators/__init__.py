"""Reference import name ``aggregators`` -> garfield_amd.aggregators."""
import sys as _sys

import garfield_amd.aggregators as _impl
from garfield_amd.aggregators import gars, make_gar, register  # noqa: F401

for _name, _rule in gars.items():
    globals()[_name.replace("-", "_")] = _rule
_sys.modules[__name__].__dict__.update({k: v for k, v in vars(_impl).items() if not k.startswith("__")})
