"""Checkpoint / resume.

The reference never saves a PyTorch checkpoint (no ``torch.save``);
its de facto interchange format is the flat fp32 vector of ``model.parameters()``
in registration order (``server.py:196-200,289-297``). A checkpoint here holds:

* ``flat``: that reference-layout parameter vector (what ``Server.write_model`` /
  ``get_model`` exchange), so a checkpoint can seed any node of any app;
* ``buffers``: the model's named buffers (BatchNorm statistics);
* ``momentum``: the engine's momentum in the same reference layout as ``flat``
  (so a channels_last / grouped GPU checkpoint resumes correctly on an NCHW
  engine, and vice versa), when present;
* ``step`` and free-form ``meta``;
* ``tuning`` (engine checkpoints): the measured kernel choices of the grouped step
  (``ops/tuning.py``), restored on load so the resumed run replays the same kernels.

Files are written atomically (temp file + rename) with ``torch.save`` and read back
with ``torch.load(weights_only=True)`` — plain tensors and primitives only.
"""
from __future__ import annotations

import os
import tempfile

import torch
import torch.nn as nn

from garfield_amd.utils.flat import flatten, write_flat_parameters


def model_state(model: nn.Module, flat: torch.Tensor | None = None) -> dict:
    """``flat`` overrides the parameter vector (an engine's fp32 master weights when the
    module itself holds low-precision working copies)."""
    vec = flat if flat is not None else flatten(p.detach() for p in model.parameters())
    return {"flat": vec.detach().float().cpu(),
            "buffers": {n: b.detach().cpu().clone() for n, b in model.named_buffers()}}


def save(path: str, model: nn.Module, step: int = 0, momentum: torch.Tensor | None = None,
         meta: dict | None = None, flat: torch.Tensor | None = None, tuning: dict | None = None) -> str:
    state = model_state(model, flat)
    state["step"] = int(step)
    if tuning:
        state["tuning"] = tuning
    if momentum is not None:
        state["momentum"] = momentum.detach().cpu()
        state["momentum_layout"] = "reference"   # checkpoints without the key hold the same layout
    state["meta"] = dict(meta or {})
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix="tmp-ckpt-", suffix=".part")
    os.close(fd)
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load(path: str, model: nn.Module | None = None, map_location="cpu") -> dict:
    state = torch.load(path, map_location=map_location, weights_only=True)
    if model is not None:
        restore(model, state)
    return state


def restore(model: nn.Module, state: dict) -> None:
    dev = next(model.parameters()).device
    write_flat_parameters(model, state["flat"].to(dev))
    saved = state.get("buffers", {})
    with torch.no_grad():
        for n, b in model.named_buffers():
            s = saved.get(n)
            if s is not None and b.shape == s.shape:
                b.copy_(s.to(b.device))


def save_engine(path: str, engine, meta: dict | None = None, write: bool = True) -> str:
    """Checkpoint of a ``RobustDataParallel`` engine (fp32 master parameters in the
    reference layout, buffers, momentum, step). Collective in sharded multi-rank runs
    (master and momentum are gathered): call it on every rank, with ``write`` True on
    one of them."""
    if hasattr(engine, "sync_master"):
        engine.sync_master()
    mom = engine.momentum_vector() if hasattr(engine, "momentum_vector") else engine.mom
    mom_ref = engine.flat.to_reference(mom)
    if not write:
        return path
    from garfield_amd.ops import tuning

    return save(path, engine.model, engine.step_count, mom_ref, meta, flat=engine.flat.reference_vector(),
                tuning=tuning.export())


def load_engine(path: str, engine) -> dict:
    state = load(path)
    if state.get("tuning"):   # the writer's kernel choices (ops/tuning.py), before any re-capture
        from garfield_amd.ops import tuning

        tuning.load(state["tuning"])
    shard = getattr(engine, "_shard", None)
    if shard is not None and hasattr(shard, "quiesce"):
        shard.quiesce()   # a previous step's updates may still run on the exchange stream
    engine.flat.load_reference_vector(state["flat"].to(engine.flat.data.device))
    saved = state.get("buffers", {})
    with torch.no_grad():
        for n, b in engine.model.named_buffers():
            s = saved.get(n)
            if s is not None and b.shape == s.shape:
                b.copy_(s.to(b.device))
    if hasattr(engine, "sync_shadow"):
        engine.sync_shadow()
    if "momentum" in state:
        m = state["momentum"].to(engine.mom.device)
        full = torch.zeros(engine.flat.ld, dtype=engine.mom.dtype, device=engine.mom.device)
        # every save_engine writes the reference layout; checkpoints from before the
        # "momentum_layout" key existed hold it too, so a missing key means "reference".
        # Only an explicit "memory" value marks a raw memory-order vector.
        if state.get("momentum_layout", "reference") == "reference":
            engine.flat.from_reference(m, full)    # reference layout -> this engine's memory order
        else:
            full[: min(m.numel(), full.numel())] = m.reshape(-1)[: full.numel()].to(full.dtype)
        shard = getattr(engine, "_shard", None)
        if shard is not None and hasattr(shard, "load_momentum"):
            shard.load_momentum(full)
        elif shard is not None:   # sharded optimizer state: this rank's slice
            engine.mom.copy_(full[shard.sl])
        else:
            engine.mom.copy_(full[: engine.mom.numel()])
    engine.step_count = int(state.get("step", 0))
    # re-capture against the restored state: the per-worker graphs and the grouped graph
    # (whose replays read the master / working weights and the BatchNorm buffers in place,
    # so they would survive, but a restored engine must not depend on that)
    engine._graph = None
    if hasattr(engine, "_ggraph"):
        engine._ggraph = None
        engine._gsrc = None
    return state


class Checkpoints:
    """Numbered checkpoints in one directory, keeping the newest ``max_to_keep``
    (the role of the reference's TF1 ``Checkpoints`` Saver wrapper,
    ``tensorflow_impl/rsrcs/tools/tf.py:78-173``, which the trainers never call).

    ``save(target, step)`` accepts a ``RobustDataParallel``-like engine (master
    weights, momentum, step) or a plain module; ``restore(target)`` loads the newest
    (or the given step). Only rank 0 should save in a data-parallel job: replicas are
    identical."""

    PREFIX, SUFFIX = "ckpt-", ".pt"

    def __init__(self, directory: str, max_to_keep: int = 5):
        self.directory = directory
        self.max_to_keep = max(int(max_to_keep), 1)
        os.makedirs(directory, exist_ok=True)

    def path(self, step: int) -> str:
        return os.path.join(self.directory, f"{self.PREFIX}{int(step):010d}{self.SUFFIX}")

    def steps(self) -> list[int]:
        out = []
        for name in os.listdir(self.directory):
            if name.startswith(self.PREFIX) and name.endswith(self.SUFFIX):
                try:
                    out.append(int(name[len(self.PREFIX):-len(self.SUFFIX)]))
                except ValueError:
                    pass
        return sorted(out)

    def latest(self) -> int | None:
        s = self.steps()
        return s[-1] if s else None

    def save(self, target, step: int | None = None, meta: dict | None = None, write: bool = True) -> str:
        """``write=False``: take part in the collectives of a sharded engine's
        checkpoint without writing (every rank but one in a data-parallel job)."""
        if hasattr(target, "flat") and hasattr(target, "step_count"):
            step = target.step_count if step is None else step
            p = save_engine(self.path(step), target, meta, write=write)
        else:
            p = save(self.path(step or 0), target, step or 0, None, meta) if write else self.path(step or 0)
        if write:
            for old in self.steps()[:-self.max_to_keep]:
                os.remove(self.path(old))
        return p

    def restore(self, target, step: int | None = None) -> dict:
        step = self.latest() if step is None else step
        if step is None:
            raise FileNotFoundError(f"no checkpoint in {self.directory}")
        if hasattr(target, "flat") and hasattr(target, "step_count"):
            return load_engine(self.path(step), target)
        return load(self.path(step), target)
