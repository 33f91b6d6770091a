"""Byzantine worker (reference ``garfieldpp/byzWorker.py:40-143``).

``ByzWorker(rank, world_size, num_workers, batch_size, model, dataset, loss, attack,
fw=1, train_size=None)``; attacks ``random | reverse | drop | lie | empire`` (plus
``nan | inf | zero``). ``lie`` / ``empire`` simulate ``fw`` colluders by computing
the honest gradient on batches ``iter+1 .. iter+fw-1`` as estimates (reference
``byzWorker.py:116,136``), once each (bug B12 computed the first one twice); ``drop``
actually zeroes 30 % of the coordinates (bug B3: the reference's ``masked_fill``
result was discarded).
"""
from __future__ import annotations

import torch

from garfield_amd.runtime.attacks import NEEDS_ESTIMATES, WORKER_ATTACKS, apply_attack
from garfield_amd.runtime.worker import Worker


class ByzWorker(Worker):
    def __init__(self, rank, world_size, num_workers, batch_size, model, dataset, loss, attack, fw=1,
                 train_size=None, device=None, register: bool = True):
        if attack not in WORKER_ATTACKS:
            raise ValueError(f"The requested attack is not implemented; available attacks are: {list(WORKER_ATTACKS)}")
        super().__init__(rank, world_size, num_workers, batch_size, model, dataset, loss, train_size, device,
                         register)
        self.fw = fw
        self.attack_name = attack
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(10007 + rank)

    def compute_local_gradient(self, iter_num: int, model=None):
        grad, loss = super().compute_local_gradient(iter_num, model)
        est = None
        if self.attack_name in NEEDS_ESTIMATES:
            ests = [grad]
            for i in range(self.fw - 1):
                g, _ = super().compute_local_gradient(iter_num + i + 1, None)
                ests.append(g)
            est = torch.stack(ests)
        return apply_attack(self.attack_name, grad, est, self.gen), loss

    # explicit per-attack entry points (reference API)
    def random_attack(self, iter_num, model):
        return self._with("random", iter_num, model)

    def reverse_attack(self, iter_num, model):
        return self._with("reverse", iter_num, model)

    def partial_drop_attack(self, iter_num, model):
        return self._with("drop", iter_num, model)

    def little_is_enough_attack(self, iter_num, model):
        return self._with("lie", iter_num, model)

    def fall_empires_attack(self, iter_num, model):
        return self._with("empire", iter_num, model)

    def _with(self, name, iter_num, model):
        old, self.attack_name = self.attack_name, name
        try:
            return self.compute_gradients(iter_num, model)
        finally:
            self.attack_name = old
