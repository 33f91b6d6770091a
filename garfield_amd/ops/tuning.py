"""Measured kernel choices of the grouped step, made reproducible.

The grouped executor picks some kernels by timing them on the real operands during the first
(eager) step (``ops/grouped.py``): the tile configuration of every ``gemm_nt`` problem
(``_GEMM_CFG``), the stride-2 data gradient's parity-class kernel vs dcol GEMM + col2im
(``_S2_CHOICE``) and the small-image weight gradient's dense vs implicit form
(``_SC_WG_CHOICE``). The candidates round bf16 differently, so a choice that depends on a
wall-clock measurement would make two runs, two ranks, or a run resumed in a new process
compute different gradients. This module pins them:

* ``agree()``: after the first step, every rank adopts rank 0's table (one
  ``broadcast_object_list``), so all ranks capture the same kernels (the engines call it once);
* ``export()`` / ``load()``: the table travels in every engine checkpoint
  (``utils/checkpoint.py``) and is restored before the resumed step, so a resumed run replays
  the kernels of the run that wrote it;
* ``GARFIELD_TUNING_FILE=path``: the table is read from that JSON file at import (and can be
  written with ``save``), e.g. a table measured once per cluster;
* ``GARFIELD_TUNING=fixed``: no timing at all; problems not in the table take the static
  per-shape pick (``gemm_nt_pick``, the parity-class stride-2 kernel, the dense small-image
  weight gradient), identical on every machine.
"""
from __future__ import annotations

import json
import os

_TABLES: dict = {}   # kind -> the live dict of ops/grouped.py


def register(kind: str, table: dict) -> dict:
    """Register one of ``ops/grouped.py``'s choice dicts under ``kind`` (returns it)."""
    _TABLES[kind] = table
    pending = _PENDING.pop(kind, None)
    if pending:
        table.update(pending)
    return table


_PENDING: dict = {}   # entries loaded before their table registered (file read at import)


def measuring() -> bool:
    """Whether unknown problems may be timed (False under ``GARFIELD_TUNING=fixed``)."""
    return os.environ.get("GARFIELD_TUNING", "measure") != "fixed"


def _tup(x):
    return tuple(_tup(v) for v in x) if isinstance(x, (list, tuple)) else x


def _lst(x):
    return [_lst(v) for v in x] if isinstance(x, (list, tuple)) else x


def _val(v):
    if isinstance(v, bool):
        return v
    if isinstance(v, (list, tuple)):
        return tuple(_val(x) for x in v)
    return int(v)


def export() -> dict:
    """The whole table as plain lists / ints / bools (JSON and ``weights_only`` safe)."""
    return {kind: [[_lst(k), _lst(v)] for k, v in sorted(t.items(), key=repr)] for kind, t in _TABLES.items()}


def load(table: dict | None, replace: bool = False) -> None:
    """Adopt ``table`` (``export()``'s form); ``replace`` drops entries it does not hold."""
    if not table:
        return
    for kind, items in table.items():
        entries = {_tup(k): _val(v) for k, v in items}
        t = _TABLES.get(kind)
        if t is None:
            _PENDING.setdefault(kind, {}).update(entries)
            continue
        if replace:
            t.clear()
        t.update(entries)


def agree(group=None) -> None:
    """Collective: every rank adopts rank 0's table (call at the same point on every rank)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return
    box = [export()]
    dist.broadcast_object_list(box, src=0, group=group)
    load(box[0], replace=True)


def save(path: str) -> str:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".part"
    with open(tmp, "w") as fh:
        json.dump(export(), fh)
    os.replace(tmp, path)
    return path


def _load_file() -> None:
    path = os.environ.get("GARFIELD_TUNING_FILE")
    if path and os.path.exists(path):
        with open(path) as fh:
            load(json.load(fh))


_load_file()
