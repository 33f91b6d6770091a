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


def print_args(name: str, selected, list_keyval, head: str = "[ARGS] ") -> None:
    """Print a selected instance and its ``key:value`` arguments
    (reference ``tensorflow_impl/rsrcs/tools/misc.py:172-184``)."""
    print(head + "Selected " + name + ": " + (selected if selected else "<none>"))
    for key, val in parse_keyval(list_keyval).items():
        print(head + "· " + key + ": " + str(val))


class ExpandPath:
    """Temporarily append paths to ``sys.path`` (reference ``misc.py:189-219``)."""

    def __init__(self, *paths):
        self._exp = [str(p) for p in paths]
        self._old = None

    def __enter__(self):
        import sys

        self._old = sys.path
        sys.path = sys.path + self._exp
        return self

    def __exit__(self, *exc):
        import sys

        sys.path = self._old
        return False


def make_interface(_create, _destroy, **methods):
    """Pointer-implementation class over a native handle (reference ``misc.py:224-283``):
    ``_create(*args) -> handle``, ``_destroy(handle)``, each method ``f(handle, ...)``."""
    nname = "_native"
    if nname in methods:
        raise ValueError(f"Method name {nname!r} is reserved")

    class Interface:
        def __init__(self, *args):
            setattr(self, nname, _create(*args))

        def __del__(self):
            if nname in self.__dict__:
                _destroy(self.__dict__[nname])

        def __getattr__(self, name):
            if nname not in self.__dict__:
                raise AttributeError("Unable to access instance as its creation failed")
            method = methods[name]
            native = self.__dict__[nname]
            return lambda *args: method(native, *args)

        def __call__(self):
            return self.__dict__[nname]

    return Interface


def device_from_tuple(job: str, task: int, dev_type: str = "cpu", dev_index: int = 0) -> str:
    """Device name for a cluster (job, task) pair (reference ``rsrcs/tools/tf.py:63-73``);
    here one process per device, so the (type, index) part is a torch device string."""
    return f"/job:{job}/replica:0/task:{task}/device:{dev_type.upper()}:{dev_index}"
