"""Asynchronous (fastest-quorum) aggregation on collectives.

Reference: the RPC parameter server waits for the fastest ``n - f`` workers and
aggregates only their gradients (``pytorch_impl/libs/garfieldpp/server.py:134-155``,
``get_gradients(iter, num_wait_wrk)``). The synchronous collective engine
(``engine.py``) always waits for every row; here a straggling rank does not hold the
others back:

* one process group per source rank: rank r's k gradient rows travel in a
  ``broadcast`` on group r, so a late root only delays its own group's stream;
* every rank posts the receives of step t for all other roots BEFORE its own
  forward/backward (the roots' sends never wait for a straggler's compute), then
  sends its own rows;
* the leader (rank ``cfg.leader``, the reference's PS role) takes the first
  ``quorum`` roots whose rows arrived (its own included) and broadcasts that set on
  a decision group; every rank aggregates exactly those ``quorum * k`` rows, so all
  replicas apply the same update. Rows outside the set still land (in order, on
  their group's stream) and are simply not used;
* receive buffers alternate by step parity; a group's broadcasts run in order, so a
  late step-t broadcast completes before step t + 2 reuses the buffer.

A straggler that is not the leader therefore costs the others nothing: it receives
the decision and the chosen rows when it gets there and applies the same update;
when the decision of a step is already there (and excludes it) before it computes,
it skips that step's forward/backward and catches up.
If the leader itself is slow everyone waits for it, as for the reference's PS.
``finish()`` drains the in-flight broadcasts (call it before shutting the group down).

``cfg.straggler_delay`` ({rank: seconds}) sleeps after the compute of those ranks:
a fault-injection knob for tests and demos.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist
from torch import nn

from garfield_amd import aggregators
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel
from garfield_amd.runtime.attacks import NEEDS_ESTIMATES


@dataclass
class QuorumConfig(EngineConfig):
    quorum: int | None = None     # ranks whose rows are aggregated each step (default: all)
    leader: int = 0               # rank that decides the quorum set
    poll_s: float = 2e-4          # polling interval while waiting for arrivals / decisions
    catchup_poll_s: float = 5e-3  # how long a rank left out of the last quorum looks for the next decision
    straggler_delay: dict = field(default_factory=dict)   # {rank: seconds} fault injection


class QuorumDataParallel(RobustDataParallel):
    """Robust DP whose GAR uses the rows of the fastest ``quorum`` ranks (see module doc)."""

    _supports_sharding = False

    def __init__(self, model: nn.Module, loss_fn, ctx: DistContext, cfg: QuorumConfig):
        if not ctx.is_distributed:
            raise ValueError("the quorum engine needs an initialised process group")
        q = ctx.world_size if cfg.quorum is None else int(cfg.quorum)
        if not 1 <= q <= ctx.world_size:
            raise ValueError(f"quorum must be in [1, {ctx.world_size}], got {q}")
        if not 0 <= cfg.leader < ctx.world_size:
            raise ValueError(f"leader rank {cfg.leader} out of range")
        self.q = q
        super().__init__(model, loss_fn, ctx, cfg)
        W, k, ld = self.world, self.k, self.ld
        # every rank creates the groups in the same order (collective calls)
        self._groups = [dist.new_group(list(range(W))) for _ in range(W)]
        self._gdec = dist.new_group(list(range(W)))
        self._buf = torch.zeros((2, W, k, ld), dtype=self.X.dtype, device=self.device)
        self._dec = torch.zeros((2, W), dtype=torch.int32, device=self.device)
        self._inflight: list = []
        self._own = [None, None]   # this rank's send of each parity buffer
        self._dec_send = [None, None]   # the leader's decision broadcast of each parity
        self.last_quorum: list[int] = list(range(self.world))
        self.skipped = 0           # steps this rank skipped because it was behind (catch-up)

    def _check_gar(self) -> None:
        cfg = self.cfg
        n_q = cfg.workers_per_rank * (self.q if hasattr(self, "q") else self.ctx.world_size)
        msg = aggregators.get(cfg.gar).check(gradients=[torch.zeros(1)] * n_q, f=cfg.f, **cfg.gar_kwargs)
        if msg is not None:
            raise ValueError(f"GAR {cfg.gar!r} with a quorum of {n_q} gradients: {msg}")

    def graph_capturable(self) -> bool:
        return False

    def _gather_slot(self, j: int):
        return None   # rows leave in one broadcast per rank after the compute (step())

    def _compute(self, batches) -> torch.Tensor:
        if self._gexec is not None and self._groupable(batches):
            self._stage_grouped(batches)
            self._grouped_compute()
            self._attack_local_rows()
            return self._gloss.mean()
        return torch.stack(self.compute_local(batches)).float().mean()

    def step(self, batches) -> torch.Tensor:
        self._agree_tuning()
        cfg, W, r0 = self.cfg, self.world, self.rank
        par = self.step_count % 2
        buf, dec = self._buf[par], self._dec[par]
        self._inflight = [w for w in self._inflight if not w.is_completed()]
        # 1. receives of this step, posted before the compute
        works = {}
        for r in range(W):
            if r != r0:
                works[r] = dist.broadcast(buf[r], src=r, group=self._groups[r], async_op=True)
        dec_work = None if r0 == cfg.leader else dist.broadcast(dec, src=cfg.leader, group=self._gdec, async_op=True)
        # 2. compute (+ injected straggling), 3. send this rank's rows. A rank that is
        # behind and already knows it is outside this step's quorum skips the compute
        # (catch-up; its rows are sent unchanged, nobody reads them)
        late = False
        if dec_work is not None:
            if r0 not in self.last_quorum:   # left out last step: give the decision a moment to land
                t_end = time.monotonic() + cfg.catchup_poll_s
                while not dec_work.is_completed() and time.monotonic() < t_end:
                    time.sleep(cfg.poll_s)
            if dec_work.is_completed():
                dec_work.wait()
                late = not int(dec[r0])
        if late:
            loss = torch.full((), float("nan"), device=self.device)
            self.skipped += 1
        else:
            loss = self._compute(batches)
            delay = cfg.straggler_delay.get(r0, 0.0)
            if delay:
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                time.sleep(delay)
        if self._own[par] is not None:   # step t - 2's send of this buffer
            self._own[par].wait()
        if not late:
            buf[r0].copy_(self.X[:, r0])
        works[r0] = self._own[par] = dist.broadcast(buf[r0], src=r0, group=self._groups[r0], async_op=True)
        # 4. the quorum set: decided by the leader from arrival order, followed by the others
        if r0 == cfg.leader:
            arrived = [r0]
            while len(arrived) < self.q:
                for r in range(W):
                    if r not in arrived and works[r].is_completed():
                        arrived.append(r)
                        if len(arrived) == self.q:
                            break
                else:
                    time.sleep(cfg.poll_s)
            chosen = sorted(arrived)
            mask = torch.zeros(W, dtype=torch.int32)
            mask[chosen] = 1
            if self._dec_send[par] is not None:   # step t - 2's decision left this buffer
                self._dec_send[par].wait()
            dec.copy_(mask)
            # asynchronous: on RCCL a synchronous broadcast would hold the leader's stream
            # until every rank, a straggler included, has posted its receive
            self._dec_send[par] = dist.broadcast(dec, src=r0, group=self._gdec, async_op=True)
        else:
            dec_work.wait()
            chosen = [r for r, v in enumerate(dec.tolist()) if v]
        for r in chosen:
            if r != r0:
                works[r].wait()
        self._inflight += [works[r] for r in range(W) if r not in chosen and r != r0]
        self.last_quorum = chosen
        # 5. GAR over the chosen rows in slot order (slot j * world + r, as the synchronous
        # engine's [n, d] input) + the update. A colluding attack rewrites its row: on a
        # copy, since buf[r0] is the source of this rank's still-running broadcast and a
        # late receiver must get the honest row (and attack it itself, identically)
        slots = [j * W + r for j in range(self.k) for r in chosen]
        rows = [buf[s % W, s // W, : self.d] for s in slots]
        colluders = {s for s, a in cfg.byzantine.items() if a in NEEDS_ESTIMATES}
        rows = [r.clone() if s in colluders else r for r, s in zip(rows, slots)]
        self._collude(rows, slots)
        self._update_from_rows(rows)
        self.step_count += 1
        return loss

    def finish(self) -> None:
        """Wait for every broadcast still in flight (late rows of stragglers)."""
        for w in self._inflight + [w for w in self._own + self._dec_send if w is not None]:
            w.wait()
        self._inflight, self._own, self._dec_send = [], [None, None], [None, None]
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
