"""Byzantine-server mode (ByzSGD / GuanYu) over collectives.

Reference: ``applications/Garfield_CC/trainer.py:90-196`` (per parameter tensor:
every worker broadcasts its gradient to every PS replica inside a
``workers ∪ {ps}`` group, PS replicas ``all_gather`` their aggregated gradients and
apply ``--mar``, then every PS broadcasts to every worker, which applies ``--mar``
again) and the RPC ``ByzSGD`` trainer (``get_models`` + model GAR).

Collective form here, per step, on flat vectors (never per tensor):

1. worker ranks (``rank >= num_ps``) compute their logical workers' gradients into
   the exchange buffer ``X[k, world, ld]`` -- with the grouped executor (one HIP graph
   for the k workers, as in the plain engine) for the ResNet family; server ranks
   contribute zero rows, or host logical workers too with ``ps_workers=True`` (no
   idle GPUs: a server rank then trains like any worker rank);
2. ``X`` is all-gathered (RCCL full mesh) slot by slot, overlapped with compute;
3. every server replica runs the GAR (f = fw) on the worker rows only (a row
   table over the worker slots — no stacking copy) and applies its SGD update;
   simulated Byzantine servers (``ps_attack``, ranks < fps) then corrupt their model;
4. each server broadcasts its fp32 model (``num_ps`` broadcasts into ``M[num_ps, ld]``:
   only the server rows travel, ``num_ps * d * 4`` bytes received per rank) and every
   rank writes the model aggregation rule (``mar``, f = fps) over them into its own
   parameters (HIP coordinate-wise kernel writing straight into the flat fp32
   parameter buffer). Honest replicas therefore stay identical. With one server the
   rule over a single model is that model: the server keeps its update as it is and
   the others receive it straight into their parameters.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from garfield_amd.ops import gar
from garfield_amd.parallel.comm import DistContext, all_gather_rows, collectives_on
from garfield_amd.parallel.engine import COORD_RULES, WEIGHTED_RULES, EngineConfig, RobustDataParallel
from garfield_amd.runtime.attacks import SERVER_ATTACKS


@dataclass
class ByzPSConfig(EngineConfig):
    num_ps: int = 3
    fps: int = 1
    mar: str = "trimmed-mean"
    ps_attack: str = ""        # attack of the simulated Byzantine servers (ranks < fps)
    ps_workers: bool = False   # server ranks also host workers_per_rank logical workers


class ByzantinePSDataParallel(RobustDataParallel):
    # Every server replica aggregates ALL worker rows itself (all-gather form): sharding the
    # servers' GAR across replicas would let one Byzantine server corrupt its shard of
    # every honest server's aggregate, which is the failure this mode exists to tolerate.
    _supports_sharding = False

    def __init__(self, model: nn.Module, loss_fn, ctx: DistContext, cfg: ByzPSConfig):
        top = ctx.world_size if cfg.ps_workers else ctx.world_size - 1   # someone must compute gradients
        if not (0 < cfg.num_ps <= top):
            raise ValueError(f"need 0 < num_ps <= {top} (world {ctx.world_size}, ps_workers={cfg.ps_workers}), "
                             f"got num_ps={cfg.num_ps}")
        self.num_ps = cfg.num_ps
        super().__init__(model, loss_fn, ctx, cfg)
        self.is_ps = ctx.rank < cfg.num_ps
        self.worker_ranks = list(range(0 if cfg.ps_workers else cfg.num_ps, ctx.world_size))
        self.computes = (not self.is_ps) or cfg.ps_workers
        self.n_w = self.k * len(self.worker_ranks)
        self.M = torch.zeros((self.num_ps, self.ld), dtype=torch.float32, device=self.device)
        self._ps_gen = torch.Generator(device=self.device)
        self._ps_gen.manual_seed(cfg.seed + 31 * ctx.rank)

    def _check_gar(self) -> None:
        from garfield_amd import aggregators

        cfg = self.cfg
        n_w = cfg.workers_per_rank * (self.ctx.world_size - (0 if cfg.ps_workers else cfg.num_ps))
        msg = aggregators.get(cfg.gar).check(gradients=[torch.zeros(1)] * n_w, f=cfg.f, **cfg.gar_kwargs)
        if msg is not None:
            raise ValueError(f"GAR {cfg.gar!r} with {n_w} worker gradients: {msg}")
        msg = aggregators.get(cfg.mar).check(gradients=[torch.zeros(1)] * cfg.num_ps, f=cfg.fps)
        if msg is not None:
            raise ValueError(f"MAR {cfg.mar!r} with {cfg.num_ps} servers: {msg}")

    def graph_capturable(self) -> bool:
        return False  # per-worker graphs: servers and workers run different bodies (grouped: see _compute)

    def _worker_rows(self) -> list:
        return [self.X[j, r, : self.d] for j in range(self.k) for r in self.worker_ranks]

    def _compute(self, batches) -> torch.Tensor:
        """This rank's logical workers -> exchange rows (+ the slot all-gathers)."""
        if self._gexec is not None and self._groupable(batches):
            self._stage_grouped(batches)
            self._grouped_compute()
            self._attack_local_rows()
            works = [w for w in (self._gather_slot(j) for j in range(self.k)) if w is not None]
            for w in works:
                w.wait()
            return self._gloss.mean()
        losses = self.compute_local(batches)
        return torch.stack(losses).float().mean()

    def step(self, batches) -> torch.Tensor:
        self._agree_tuning()
        cfg = self.cfg
        # 1-2: gradients (worker ranks) + exchange (everyone)
        if self.computes:
            loss = self._compute(batches)
        else:
            works = [all_gather_rows(self.X[j], self.rank, async_op=True) for j in range(self.k)] \
                if collectives_on(self.world) else []
            for w in works:
                w.wait()
            loss = torch.zeros((), device=self.device)
        # 3: servers aggregate + update
        if self.is_ps:
            self._server_update()
            if cfg.ps_attack and self.rank < cfg.fps:
                v = self.flat.data[: self.d]
                v.copy_(SERVER_ATTACKS[cfg.ps_attack](v, generator=self._ps_gen))
        # 4: model exchange (the servers' rows only) + model aggregation on every rank
        self._exchange_models()
        self.step_count += 1
        return loss

    def _exchange_models(self) -> None:
        import torch.distributed as dist

        if self.num_ps == 1:   # the rule over one model is that model
            if collectives_on(self.world):
                dist.broadcast(self.flat.data, src=0)
                if not self.is_ps:
                    self.sync_shadow()
            return
        if self.is_ps:
            self.M[self.rank].copy_(self.flat.data)
        if collectives_on(self.world):
            works = [dist.broadcast(self.M[p], src=p, async_op=True) for p in range(self.num_ps)]
            for w in works:
                w.wait()
        self._write_mar([self.M[p, : self.d] for p in range(self.num_ps)])
        self.sync_shadow()   # master weights were rewritten by the model aggregation

    def _server_update(self) -> None:
        rows = self._worker_rows()
        self._collude(rows, [j * self.world + r for j in range(self.k) for r in self.worker_ranks])
        self._update_from_rows(rows)

    def _write_mar(self, models: list) -> None:
        cfg = self.cfg
        out = self.flat.data[: self.d]
        kw = {} if cfg.mar in ("average", "median", "average-nan") else {"f": cfg.fps}
        if self.device.type == "cuda" and cfg.mar in COORD_RULES and cfg.mar not in ("bulyan", "condense"):
            modes = gar._MODE
            beta = len(models) - cfg.fps
            self._C.gpu_coordwise(models, modes[cfg.mar], cfg.fps, beta, None, 0, 0, 1.0, out)
        else:
            agg = gar.aggregate(cfg.mar, models, **kw)
            with torch.no_grad():
                out.copy_(agg)
