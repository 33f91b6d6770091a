"""Byzantine parameter server (reference ``garfieldpp/byzServer.py:45-108``).

``get_model`` returns an attacked model (``random | reverse | drop``, plus ``nan`` /
``zero``) as ``(rank, tensor)`` — the reference returned a bare tensor, which broke
``Server.get_models`` (bug B4) — and ``get_latest_aggr_grad`` is attacked the same way.
"""
from __future__ import annotations

import torch

from garfield_amd.runtime.attacks import SERVER_ATTACKS
from garfield_amd.runtime.server import Server


class ByzServer(Server):
    def __init__(self, rank, world_size, num_workers, num_ps, byz_wrk, byz_ps, wrk_base_name, ps_base_name, batch,
                 model, dataset, optimizer, attack, *args, train_size=None, **kwargs):
        if attack not in SERVER_ATTACKS:
            raise ValueError(f"The requested attack is not implemented; available attacks are: {list(SERVER_ATTACKS)}")
        # set before the base constructor announces this server to its peers
        self.attack_name = attack
        self.gen = torch.Generator()
        self.gen.manual_seed(20011 + rank)
        super().__init__(rank, world_size, num_workers, num_ps, byz_wrk, byz_ps, wrk_base_name, ps_base_name, batch,
                         model, dataset, optimizer, train_size, *args, **kwargs)

    def _attack(self, t: torch.Tensor) -> torch.Tensor:
        return SERVER_ATTACKS[self.attack_name](t, generator=self.gen)

    def get_model(self):
        rank, m = super().get_model()
        return rank, self._attack(m)

    def get_latest_aggr_grad(self):
        rank, g = super().get_latest_aggr_grad()
        return rank, self._attack(g)

    # reference API
    def random_attack(self):
        return self.rank, SERVER_ATTACKS["random"](self._payload(), generator=self.gen)

    def reverse_attack(self):
        return self.rank, SERVER_ATTACKS["reverse"](self._payload())

    def partial_drop_attack(self):
        return self.rank, SERVER_ATTACKS["drop"](self._payload(), generator=self.gen)
