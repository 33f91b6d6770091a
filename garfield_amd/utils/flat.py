"""Flat-parameter layout: the reference's interchange and checkpoint format.

The reference moves models and gradients as the concatenation of
``p.view(-1)`` over ``model.parameters()`` in registration order
(``garfieldpp/server.py:196-200,289-297``, ``worker.py:93-94``; buffers such as
BatchNorm statistics excluded), and ``tools/pytorch.py:27-92`` provides
``flatten`` / ``relink`` / ``grads_of``.

``FlatParams`` goes one step further for the MI355X engine: every parameter's
``.data`` (and optionally ``.grad``) is re-pointed to a view of ONE contiguous fp32
buffer, so the fused GAR + SGD kernel updates the whole model in a single pass
and the flat vector needs no gather/scatter. The buffer length is padded to a
multiple of 64 elements (16-byte aligned rows for every dtype).
"""
from __future__ import annotations

import weakref
from typing import Iterable

import torch
import torch.nn as nn

PAD = 64


def padded(d: int, pad: int = PAD) -> int:
    return ((d + pad - 1) // pad) * pad


def flatten(tensors: Iterable[torch.Tensor]) -> torch.Tensor:
    """Concatenate the (flattened) tensors into one new 1-D tensor."""
    return torch.cat([t.reshape(-1) for t in tensors])


def relink(tensors: Iterable[torch.Tensor], common: torch.Tensor) -> torch.Tensor:
    """Make every tensor's storage a view of ``common`` (reference tools/pytorch.py:46-70)."""
    pos = 0
    for t in tensors:
        n = t.numel()
        t.data = common[pos:pos + n].view_as(t)
        pos += n
    return common


def grads_of(tensors: Iterable[torch.Tensor]):
    """Yield each tensor's gradient (zeros if it has none)."""
    for t in tensors:
        g = t.grad
        yield torch.zeros_like(t) if g is None else g


def flat_parameters(model: nn.Module) -> torch.Tensor:
    """Reference-layout flat copy of the model parameters (``Server.get_model``)."""
    return flatten(p.detach() for p in model.parameters())


def flat_gradients(model: nn.Module) -> torch.Tensor:
    """Reference-layout flat copy of the model gradients (``Worker.compute_gradients``)."""
    return flatten(grads_of(model.parameters()))


def write_flat_parameters(model: nn.Module, flat: torch.Tensor) -> None:
    """Copy a reference-layout flat vector into the parameters (``Server.write_model``)."""
    pos = 0
    with torch.no_grad():
        for p in model.parameters():
            n = p.numel()
            p.copy_(flat[pos:pos + n].view_as(p))
            pos += n


def is_dense(t: torch.Tensor) -> bool:
    """True when t's elements tile its storage span exactly (any dimension order)."""
    expected = 1
    for i in sorted(range(t.dim()), key=lambda i: t.stride(i)):
        if t.size(i) == 1:
            continue
        if t.stride(i) != expected:
            return False
        expected *= t.size(i)
    return True


def memory_order_flat(t: torch.Tensor) -> torch.Tensor:
    """1-D view/copy of a dense tensor in MEMORY order (== logical order when contiguous)."""
    if t.is_contiguous():
        return t.reshape(-1)
    perm = sorted(range(t.dim()), key=lambda i: -t.stride(i))
    return t.permute(perm).reshape(-1)


class FlatParams:
    """All parameters of ``model`` as views of one padded fp32 buffer (+ optional grad buffer).

    Views keep each parameter's strides (``as_strided`` over the flat storage), so
    a ``channels_last`` model stays ``channels_last``; the flat buffer is then in
    memory order. ``reference_vector()`` always returns the reference layout
    (logical ``p.view(-1)`` order) for checkpoints and the RPC API."""

    def __init__(self, model: nn.Module, device=None, dtype=torch.float32, with_grad: bool = True, pad: int = PAD):
        self.model = model
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.numels = [p.numel() for p in self.params]
        self.d = sum(self.numels)
        self.ld = padded(self.d, pad)
        device = device or self.params[0].device
        self.data = torch.zeros(self.ld, dtype=dtype, device=device)
        self.offsets = []
        pos = 0
        for p, n in zip(self.params, self.numels):
            if not is_dense(p):
                raise ValueError("FlatParams needs dense parameters")
            self.offsets.append(pos)
            pos += n
        self.sizes = [tuple(p.size()) for p in self.params]
        self.strides = [tuple(p.stride()) for p in self.params]
        with torch.no_grad():
            for p, v in zip(self.params, self.views(self.data)):
                v.copy_(p.detach())
        for p, v in zip(self.params, self.views(self.data)):
            p.data = v
        self.grad = None
        if with_grad:
            self.grad = torch.zeros(self.ld, dtype=dtype, device=device)
            self.attach_grads(self.grad)
        # called before the readers below: an engine whose updates may still be in flight on a
        # side stream (a staged sharded step) installs its ``synchronize`` here, as a
        # ``weakref.WeakMethod`` (a bound method would tie the engine, its HIP graphs and pools
        # into a reference cycle with these parameters, freed only by the cyclic collector)
        self.before_read = None

    def _sync(self) -> None:
        fn = self.before_read
        if fn is not None and isinstance(fn, weakref.WeakMethod):
            fn = fn()
        if fn is not None:
            fn()

    def views(self, flat: torch.Tensor):
        """Per-parameter views (parameter strides) of a flat buffer laid out like ``data``;
        ``flat`` may itself be a view (e.g. one row of a 2-D buffer)."""
        base = flat.storage_offset()
        for size, stride, off in zip(self.sizes, self.strides, self.offsets):
            yield torch.as_strided(flat, size, stride, base + off)

    def attach_grads(self, flat: torch.Tensor) -> None:
        """Point every ``p.grad`` at its slice of ``flat`` (backward accumulates in place)."""
        for p, v in zip(self.params, self.views(flat)):
            p.grad = v

    def vector(self) -> torch.Tensor:
        self._sync()
        return self.data[: self.d]

    def grad_vector(self) -> torch.Tensor:
        return self.grad[: self.d]

    def reference_vector(self) -> torch.Tensor:
        """Reference interchange layout: cat of p.view(-1) (logical order)."""
        self._sync()
        return flatten(p.detach() for p in self.params)

    def load_reference_vector(self, flat: torch.Tensor) -> None:
        self._sync()
        with torch.no_grad():
            pos = 0
            for p, n in zip(self.params, self.numels):
                p.copy_(flat[pos:pos + n].view(p.shape))
                pos += n

    def to_reference(self, buf: torch.Tensor) -> torch.Tensor:
        """A buffer laid out like ``data`` (memory order, e.g. the momentum) in the
        reference layout (logical ``p.view(-1)`` order per parameter)."""
        self._sync()
        return flatten(v.detach() for v in self.views(buf))

    def from_reference(self, flat: torch.Tensor, buf: torch.Tensor) -> torch.Tensor:
        """Scatter a reference-layout vector into ``buf`` (laid out like ``data``)."""
        with torch.no_grad():
            pos = 0
            for v, n in zip(self.views(buf), self.numels):
                v.copy_(flat[pos:pos + n].view(v.shape))
                pos += n
        return buf

    def grads_flat(self, out: torch.Tensor, params=None) -> torch.Tensor:
        """Write the current per-parameter gradients (memory order) into ``out[:d]``;
        ``params``: the tensors whose ``.grad`` to read, one per parameter (e.g. an engine's
        working copies), default the parameters themselves."""
        pos = 0
        for p, n in zip(self.params if params is None else params, self.numels):
            g = p.grad
            if g is None:
                out[pos:pos + n].zero_()
            else:
                out[pos:pos + n].copy_(memory_order_flat(g))
            pos += n
        return out


# --------------------------------------------------------------------------- #
# TF-tree helpers, over torch tensors / numpy arrays

def flatten_pairs(pairs, flatmap: dict | None = None):
    """Flatten ``[(gradient, variable), ...]`` skipping ``None`` gradients (reference
    ``Garfield_legacy/helper.py:65-88``). Without ``flatmap`` returns ``(flat, flatmap)``
    with ``flatmap[variable] = position``; with it, places each gradient at its
    recorded position and returns the flat tensor only. Variables are keyed by identity."""
    if flatmap is None:
        flatmap, res = {}, []
        for g, v in pairs:
            if g is None:
                continue
            flatmap[id(v)] = len(res)
            res.append(g.reshape(-1))
        return torch.cat(res), flatmap
    res = [None] * len(flatmap)
    for g, v in pairs:
        if g is not None:
            res[flatmap[id(v)]] = g.reshape(-1)
    return torch.cat(res)


def mapflat(flatmap: dict, variables: Iterable) -> list:
    """Variables ordered by their position in the flat gradient (``helper.py:90-100``);
    ``variables`` resolves the identity keys ``flatten_pairs`` records."""
    by_id = {id(v): v for v in variables}
    res = [None] * len(flatmap)
    for key, pos in flatmap.items():
        res[pos] = by_id[key]
    return res


def inflate(flat: torch.Tensor, ordered: Iterable) -> list:
    """``[(view, variable), ...]``: slices of ``flat`` shaped like each variable, in order
    (``helper.py:102-120``). The slices are views, no copy."""
    res, pos = [], 0
    for v in ordered:
        n = v.numel()
        res.append((flat[pos:pos + n].view(v.shape), v))
        pos += n
    return res


def flatten_weights(tensors: Iterable):
    """numpy concatenation of the raveled weights (reference ``TF/libs/tools.py:112-121``)."""
    import numpy as np

    return np.concatenate([np.asarray(t.detach().cpu() if isinstance(t, torch.Tensor) else t).reshape(-1)
                           for t in tensors])


def reshape_weights(model, flat) -> list:
    """Split ``flat`` into numpy arrays shaped like ``model``'s trainable parameters
    (reference ``TF/libs/tools.py:123-144``)."""
    import numpy as np

    flat = np.asarray(flat)
    out, i = [], 0
    params = model.parameters() if isinstance(model, nn.Module) else model
    for p in params:
        if isinstance(p, torch.Tensor) and not p.requires_grad:
            continue
        n = int(np.prod(p.shape))
        out.append(np.array(flat[i:i + n]).reshape(tuple(p.shape)))
        i += n
    return out
