"""Miscellaneous helpers (reference ``pytorch_impl/libs/tools/misc.py``,
``tools/__init__.py:280-305``, ``tools/cluster.py:27-73``)."""
from __future__ import annotations

import importlib
import os
import pathlib
import time
from itertools import combinations

from garfield_amd.utils.logging import UserException, info, warning


def pairwise(data):
    """All unordered pairs (i < j) of the elements of ``data`` (reference misc.py:518)."""
    return combinations(data, 2)


def parse_keyval(list_keyval, defaults: dict | None = None) -> dict:
    """Parse ``["key:value", ...]`` into a dict; values are cast to the type of the
    matching default when there is one, else int/float/bool when they parse as such
    (reference misc.py:197-238)."""
    defaults = dict(defaults or {})
    out = {}
    for entry in list_keyval or []:
        if ":" not in entry:
            raise UserException(f"Expected 'key:value', got {entry!r}")
        key, val = entry.split(":", 1)
        if key in out:
            raise UserException(f"Key {key!r} given twice")
        if key in defaults and defaults[key] is not None:
            typ = type(defaults[key])
            if typ is bool:
                out[key] = val.lower() in ("1", "true", "yes", "y", "on")
            else:
                try:
                    out[key] = typ(val)
                except ValueError as e:
                    raise UserException(f"Key {key!r}: cannot convert {val!r} to {typ.__name__}") from e
        else:
            out[key] = _auto(val)
    for k, v in defaults.items():
        out.setdefault(k, v)
    return out


def _auto(val: str):
    for cast in (int, float):
        try:
            return cast(val)
        except ValueError:
            pass
    if val.lower() in ("true", "false"):
        return val.lower() == "true"
    return val


class TimedContext:
    """``with TimedContext() as t: ...`` then ``t.elapsed`` (seconds); optional print
    (reference misc.py:307-345). Synchronises the GPU when ``sync`` is set."""

    def __init__(self, name: str | None = None, sync: bool = False, verbose: bool = False):
        self.name, self.sync, self.verbose = name, sync, verbose
        self.elapsed = None

    def _sync(self):
        if self.sync:
            import torch

            if torch.cuda.is_available():
                torch.cuda.synchronize()

    def __enter__(self):
        self._sync()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self._sync()
        self.elapsed = time.perf_counter() - self.t0
        if self.verbose:
            info(f"{self.name or 'block'}: {self.elapsed * 1000:.3f} ms")
        return False


def import_directory(dirpath, scope: dict, package: str, post: str = "", ignore_prefix=("_", ".")) -> list:
    """Import every module of a package directory into ``scope`` (reference
    tools/__init__.py:280-305). Returns the imported module names."""
    names = []
    for path in sorted(pathlib.Path(dirpath).iterdir()):
        name = path.stem if path.suffix == ".py" else path.name
        if name.startswith(ignore_prefix) or not (path.suffix == ".py" or (path / "__init__.py").exists()):
            continue
        try:
            scope[name + post] = importlib.import_module(f"{package}.{name}")
            names.append(name)
        except Exception as e:  # report and continue, like the reference loader
            warning(f"Loading failed for module {name!r}: {e}")
    return names


def cluster_parse(spec: str | None = None, env_key: str = "OAR_FILE_NODES") -> list[str]:
    """Host list from a comma-separated spec, a nodes file (one host per line, the
    OAR/Grid5000 ``$OAR_FILE_NODES`` format), or the environment (reference
    tools/cluster.py:27-73). Duplicates collapse, order is kept."""
    if spec is None:
        spec = os.environ.get(env_key, "")
    if not spec:
        return ["127.0.0.1"]
    p = pathlib.Path(spec)
    if p.exists():
        hosts = [ln.strip() for ln in p.read_text().splitlines() if ln.strip() and not ln.startswith("#")]
    else:
        hosts = [h.strip() for h in spec.split(",") if h.strip()]
    seen, out = set(), []
    for h in hosts:
        if h not in seen:
            seen.add(h)
            out.append(h)
    return out
