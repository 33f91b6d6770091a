"""Byzantine gradient / model attacks as pure tensor functions.

Reference: ``garfieldpp/byzWorker.py:62-143`` (random, reverse, drop, lie, empire),
``byzServer.py:74-108`` (random, reverse, drop) and the TF ``libs/attacker.py:38-127``.
Differences, on purpose:

* ``drop`` really zeroes the coordinates (the reference calls the out-of-place
  ``masked_fill`` and discards the result, bug B3);
* ``lie`` / ``empire`` take the colluders' gradient estimates as an argument
  instead of recomputing the honest gradient (bug B12 computed it twice);
* extra ``nan`` / ``inf`` / ``zero`` attacks exercise the non-finite paths.

All attacks return a new tensor of the input's dtype / device.
"""
from __future__ import annotations

import torch

LIE_Z = 1.035        # z_max for n=20, f=8 (byzWorker.py:122)
EMPIRE_EPS = 10.0    # byzWorker.py:140
DROP_P = 0.3         # byzWorker.py:103
REVERSE_SCALE = -100.0


def random_attack(grad: torch.Tensor, generator=None, **_) -> torch.Tensor:
    return torch.rand(grad.shape, generator=generator, device=grad.device, dtype=torch.float32).to(grad.dtype)


def reverse_attack(grad: torch.Tensor, **_) -> torch.Tensor:
    return grad * REVERSE_SCALE


def drop_attack(grad: torch.Tensor, generator=None, p: float = DROP_P, **_) -> torch.Tensor:
    mask = torch.rand(grad.shape, generator=generator, device=grad.device) > 1 - p
    return grad.masked_fill(mask, 0)


def _estimates(grad: torch.Tensor, estimates) -> torch.Tensor:
    if estimates is None:
        return grad.float().unsqueeze(0)
    if isinstance(estimates, (list, tuple)):
        estimates = torch.stack([e.reshape(-1) for e in estimates])
    return estimates.float()


def lie_attack(grad: torch.Tensor, estimates=None, z: float = LIE_Z, **_) -> torch.Tensor:
    """A Little Is Enough (Baruch et al. 2019): mu + z * sigma of the colluders' estimates."""
    E = _estimates(grad, estimates)
    mu = E.mean(0)
    sigma = E.std(0, unbiased=True) if E.shape[0] > 1 else torch.zeros_like(mu)
    return (mu + z * sigma).to(grad.dtype)


def empire_attack(grad: torch.Tensor, estimates=None, eps: float = EMPIRE_EPS, **_) -> torch.Tensor:
    """Fall of Empires (Xie et al. 2019): -eps * mean of the colluders' estimates."""
    E = _estimates(grad, estimates)
    return (-eps * E.mean(0)).to(grad.dtype)


def nan_attack(grad: torch.Tensor, **_) -> torch.Tensor:
    return torch.full_like(grad, float("nan"))


def inf_attack(grad: torch.Tensor, **_) -> torch.Tensor:
    return torch.full_like(grad, float("inf"))


def zero_attack(grad: torch.Tensor, **_) -> torch.Tensor:
    return torch.zeros_like(grad)


WORKER_ATTACKS = {
    "random": random_attack,
    "reverse": reverse_attack,
    "drop": drop_attack,
    "lie": lie_attack,
    "empire": empire_attack,
    "nan": nan_attack,
    "inf": inf_attack,
    "zero": zero_attack,
}

SERVER_ATTACKS = {"random": random_attack, "reverse": reverse_attack, "drop": drop_attack,
                  "nan": nan_attack, "zero": zero_attack}

# attacks that need the colluding workers' gradient estimates
NEEDS_ESTIMATES = {"lie", "empire"}


def apply_attack(name: str, grad: torch.Tensor, estimates=None, generator=None) -> torch.Tensor:
    try:
        fn = WORKER_ATTACKS[name]
    except KeyError:
        raise ValueError(f"unknown attack {name!r}; available: {sorted(WORKER_ATTACKS)}") from None
    return fn(grad, estimates=estimates, generator=generator)
