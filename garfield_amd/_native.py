"""Loader of the native extension ``garfield_amd._C``.

Reference counterpart: ``pytorch_impl/libs/native/__init__.py`` (JIT-builds every
``py_*``/``so_*`` directory on import). Here the extension is built ahead of time
in-tree (``python -m garfield_amd.csrc.build`` or ``__graft_entry__.build()``) and
imported; ``GARFIELD_AUTOBUILD=1`` builds it on first use.

Policy: on a machine with a GPU the native extension is MANDATORY — a missing or
broken ``_C`` raises instead of silently running a PyTorch fallback. On a CPU-only
machine the pure-PyTorch reference implementations may stand in (with a warning).
"""
from __future__ import annotations

import importlib
import os
import warnings

_C = None
_ERR: Exception | None = None


def _try_import():
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        import torch  # noqa: F401  (libc10 / libtorch symbols must be loaded first)
        _C = importlib.import_module("garfield_amd._C")
        _ERR = None
        _check_manifest()
    except Exception as e:  # pragma: no cover - depends on the build state
        _ERR = e
        if os.environ.get("GARFIELD_AUTOBUILD", "0") == "1":
            from garfield_amd.csrc import build as _b

            _b.build()
            _C = importlib.import_module("garfield_amd._C")
            _ERR = None
    return _C


def _check_manifest() -> None:
    """Warn when the loaded extension was built from other sources than the ones in the tree
    (``_C.build.json``, written by every build)."""
    try:
        import json

        from garfield_amd.csrc import build as _b

        man = _b.manifest_path()
        if man.exists() and json.loads(man.read_text()).get("sources_sha256") != _b.sources_digest():
            warnings.warn("garfield_amd: the native extension was built from different sources than the tree's "
                          "garfield_amd/csrc (rebuild: python -m garfield_amd.csrc.build)", RuntimeWarning, stacklevel=3)
    except Exception:   # the check is advisory
        pass


def available() -> bool:
    return _try_import() is not None


def native():
    """Return the extension module or raise a descriptive error."""
    m = _try_import()
    if m is None:
        raise RuntimeError(
            "garfield_amd native extension (_C) is not available: "
            f"{_ERR!r}. Build it with `python -m garfield_amd.csrc.build`."
        )
    return m


def require_for(device) -> object | None:
    """Native module for ``device``; None only for CPU tensors without an extension."""
    m = _try_import()
    if m is not None:
        return m
    if getattr(device, "type", str(device)) != "cpu":
        raise RuntimeError(
            "garfield_amd: GPU aggregation requires the native HIP extension, which failed to load: "
            f"{_ERR!r}. Run `python -m garfield_amd.csrc.build` (no silent PyTorch fallback on GPU)."
        )
    warnings.warn("garfield_amd: native extension missing, using the PyTorch reference path on CPU",
                  RuntimeWarning, stacklevel=3)
    return None
