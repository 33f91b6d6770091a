"""TF-transport attacker (reference ``tensorflow_impl/libs/attacker.py:33-127``).

Names as in the reference: ``Random``, ``Reverse``, ``PartialDrop``,
``LittleIsEnough`` (alias ``LittleIsNotEnough``, the name the reference's ByzWorker
checks — bug B9), ``FallEmpires``. The maths is shared with the PyTorch runtime
(``garfield_amd.runtime.attacks``); ``PartialDrop`` takes its probability from the
constructor (the reference requires an argument it never passes, B9), and the
collusion attacks use the colluders' gradient estimates passed in ``byz_gradients``.
"""
from __future__ import annotations

import torch

from garfield_amd.runtime import attacks as A

TF_ATTACKS = {"Random": "random", "Reverse": "reverse", "PartialDrop": "drop", "LittleIsEnough": "lie",
              "LittleIsNotEnough": "lie", "FallEmpires": "empire"}


class Attacker:
    def __init__(self, attack: str, probability: float = A.DROP_P, coeff: float = 100.0, seed: int = 0):
        if attack not in TF_ATTACKS:
            raise ValueError(f"unknown attack {attack!r}; available: {sorted(TF_ATTACKS)}")
        self.name = attack
        self.kind = TF_ATTACKS[attack]
        self.probability = probability
        self.coeff = coeff
        self.gen = None
        self.seed = seed

    @property
    def needs_estimates(self) -> bool:
        return self.kind in A.NEEDS_ESTIMATES

    def _generator(self, device):
        if self.gen is None or self.gen.device != torch.device(device):
            self.gen = torch.Generator(device=device)
            self.gen.manual_seed(self.seed)
        return self.gen

    def attack(self, gradient: torch.Tensor, byz_gradients=None) -> torch.Tensor:
        if self.kind == "reverse":
            return gradient * (-self.coeff)
        if self.kind == "drop":
            return A.drop_attack(gradient, generator=self._generator(gradient.device), p=self.probability)
        if self.kind == "random":
            return A.random_attack(gradient, generator=self._generator(gradient.device))
        est = list(byz_gradients or []) + [gradient]
        return A.WORKER_ATTACKS[self.kind](gradient, estimates=est)
