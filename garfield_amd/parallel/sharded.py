"""Sharded robust aggregation: every rank aggregates 1/world of the coordinates.

The redundant form of the engine (``engine.RobustDataParallel`` with
``shard_gar=False``) all-gathers every worker's full gradient to every rank, so
each rank receives ``(world - 1) * k * d`` values per step and runs the whole
GAR itself: at 8 MI355X, 8 workers per GPU and ResNet-50 (d = 23.5M, bf16) that is
2.6 GB per rank per step over xGMI, the same order as the compute step.

Every rule the engine runs is either coordinate-wise or decides from per-pair
squared distances, and squared distances are additive over coordinate blocks:
``||g_i - g_j||^2 = sum_s ||g_i^(s) - g_j^(s)||^2``. So, per step:

1. ``all_to_all_single``: rank r receives coordinate shard r of all n gradients
   (``k * d * (world-1)/world`` values out and in per rank, ~8x less than the
   all-gather at 8 GPUs);
2. distance-based rules (Krum/Multi-Krum, Bulyan's selection, Brute): each rank
   computes the partial Gram matrix of its shard (split-K MFMA kernel), the
   ``[n, n]`` partials are all-gathered (a few KB) and summed in rank order, so
   every rank sees the same matrix and makes the same selection; Aksel does the
   same with its per-row distances to the coordinate-wise median;
3. the combine / coordinate-wise kernel and the fused SGD update run on the
   shard only (fp32 master shard, momentum shard: optimizer state is sharded);
4. ``all_gather_into_tensor`` of the updated fp32 master shards; the bf16 working
   weights are re-cast locally.

Replicas stay bit-identical (they all receive the same all-gathered master).
Reference: the PS pull/aggregate/push loop of ``garfieldpp/server.py:112-159`` and
Garfield_CC's per-tensor gather/broadcast (``Garfield_CC/trainer.py:55-207``).
Condense draws its per-coordinate coin with the shard-local coordinate index, so
its mask differs from the unsharded run's (same Bernoulli(p) law).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from garfield_amd import _native
from garfield_amd.ops import gar
from garfield_amd.ops import reference as ref

DISTANCE_RULES = {"krum", "brute", "bulyan"}
SUPPORTED = DISTANCE_RULES | {"average", "aksel", "median", "trimmed-mean", "averaged-median", "average-nan",
                              "condense"}


def shard_pad(world: int, base: int = 64) -> int:
    """Row padding such that every shard is a whole number of 64-element (16-byte aligned) blocks."""
    return base * world


class ShardedAggregator:
    """All-to-all of the local gradient rows, sharded GAR, sharded SGD, all-gather."""

    def __init__(self, engine):
        e = engine
        self.e = e
        self.world, self.rank, self.k, self.n = e.world, e.rank, e.k, e.n
        if e.ld % self.world:
            raise ValueError("sharded aggregation needs the row length padded to a multiple of the world size")
        self.S = e.ld // self.world
        dev, dt = e.device, e.X.dtype
        self.send = torch.empty((self.world, self.k, self.S), dtype=dt, device=dev)
        self.recv = torch.empty((self.world, self.k, self.S), dtype=dt, device=dev)
        # slot j * world + src  ->  recv[src, j]  (the unsharded engine's row order)
        self.rows = [self.recv[s % self.world, s // self.world] for s in range(self.n)]
        self.lo = self.rank * self.S
        self.sl = slice(self.lo, self.lo + self.S)
        self.gagg = torch.zeros(self.S, dtype=torch.float32, device=dev)
        self._one = torch.ones(1, dtype=torch.float32, device=dev)
        self._ws = None
        self._avg = torch.full((self.n,), 1.0 / self.n, dtype=torch.float32, device=dev)

    # ------------------------------------------------------------------ #

    def exchange(self) -> None:
        """all_to_all: shard s of every local row goes to rank s."""
        e = self.e
        local = e.X.view(self.k, self.world, self.S)
        if self.world == 1:   # single rank (tests): the shard is the whole row
            self.recv.copy_(local.transpose(0, 1))
            return
        self.send.copy_(local.transpose(0, 1))
        dist.all_to_all_single(self.recv.view(-1), self.send.view(-1))

    def _sum_over_ranks(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's ``t`` summed in rank order (identical result on every rank)."""
        if self.world == 1:
            return t.clone()
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1))
        return out.sum(0)

    def _concat_ranks(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1))
        return out.view(-1, *t.shape[1:])

    # ------------------------------------------------------------------ #

    def aggregate_and_update(self, first: bool) -> None:
        e, cfg = self.e, self.e.cfg
        self.exchange()
        if e.device.type == "cuda":
            self._gpu(cfg, first)
        else:
            self._cpu(cfg, first)
        self._gather_master()

    def _gather_master(self) -> None:
        e = self.e
        full = e.flat.data
        if self.world > 1:
            mine = full[self.sl]
            if full.device.type == "cpu":
                mine = mine.clone()  # gloo rejects an input aliasing the output
            dist.all_gather_into_tensor(full, mine)
        if e._shadow is not None:
            with torch.no_grad():
                e._shadow.copy_(full)

    # ------------------------------------------------------------------ #
    # GPU: the HIP building blocks on the shard

    def _gpu(self, cfg, first: bool) -> None:
        e, C = self.e, self.e._C
        rule, f, kw = cfg.gar, cfg.f, dict(cfg.gar_kwargs)
        rows = gar.prepare(self.rows)
        if self._ws is None:
            self._ws = gar.Workspace(self.n, self.S, e.device)
        ws = self._ws
        param, mom = e.flat.data[self.sl], e.mom
        args = (cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
        if rule in ("average", "krum", "brute", "aksel"):
            w = self._gpu_weights(C, rows, ws, rule, f, kw)
            e.last_weights = w
            C.gpu_combine_sgd(self.rows, w, param, mom, None, None, *args)
            return
        g = self.gagg
        modes = gar._MODE
        if rule == "bulyan":
            m = cfg.m if cfg.m is not None else self.n - f - 2
            t = self.n - 2 * f - 2
            W = ws.get("bulyan_W", t * self.n)
            C.gpu_bulyan_select(self._total_gram(C, rows, ws), self.n, f, m, t, W)
            C.gpu_coordwise(self.rows, modes["bulyan-tail"], f, t - 2 * f, W, t, 0, 1.0, g)
        elif rule == "median":
            C.gpu_coordwise(self.rows, modes["median"], 0, 0, None, 0, 0, 1.0, g)
        elif rule == "trimmed-mean":
            C.gpu_coordwise(self.rows, modes["trimmed-mean"], f, 0, None, 0, 0, 1.0, g)
        elif rule == "averaged-median":
            C.gpu_coordwise(self.rows, modes["averaged-median"], f, kw.get("beta") or self.n - f, None, 0, 0, 1.0, g)
        elif rule == "average-nan":
            C.gpu_coordwise(self.rows, modes["average-nan"], 0, 0, None, 0, 0, 1.0, g)
        elif rule == "condense":
            C.gpu_coordwise(self.rows, modes["condense"], f, 0, None, 0, cfg.seed + e.step_count,
                            float(kw.get("p", 0.9)), g)
        else:
            raise ValueError(f"sharded aggregation does not support {rule!r}")
        C.gpu_combine_sgd([g], self._one, param, mom, None, None, *args)

    def _total_gram(self, C, rows, ws) -> torch.Tensor:
        g = gar._gram_into(C, rows, ws)
        return self._sum_over_ranks(g)

    def _gpu_weights(self, C, rows, ws, rule, f, kw) -> torch.Tensor:
        n = self.n
        if rule == "average":
            return self._avg
        w = ws.get("weights", n)
        if rule == "krum":
            m = self.e.cfg.m if self.e.cfg.m is not None else n - f - 2
            order = ws.get("order", n, torch.int32)
            scores = ws.get("scores", n)
            C.gpu_krum_select(self._total_gram(C, rows, ws), n, f, m, w, order, scores)
        elif rule == "brute":
            if n > 64:
                raise ValueError("brute: n must be <= 64 on the GPU")
            best = ws.get("brute_best", 1, torch.int64)
            C.gpu_brute_select(self._total_gram(C, rows, ws), n, f, best, w)
        else:  # aksel: distances to the coordinate-wise median, summed over shards
            c = (n + 1) // 2 if kw.get("mode", "mid") == "mid" else n - f
            med = ws.get("aksel_med", self.S)
            C.gpu_coordwise(self.rows, gar._MODE["median"], 0, 0, None, 0, 0, 1.0, med)
            grid = C.sqdist_grid(self.S)
            slabs = ws.get("aksel_slabs", grid * n)
            C.gpu_sqdist(self.rows, med, slabs)
            allslabs = self._concat_ranks(slabs.view(grid, n))
            dists = ws.get("aksel_dists", n)
            C.gpu_aksel_select(allslabs.contiguous().view(-1), n, c, w, dists)
        return w

    # ------------------------------------------------------------------ #
    # CPU (gloo): the same decomposition with the C++ / oracle building blocks

    def _cpu(self, cfg, first: bool) -> None:
        e = self.e
        rule, f, kw = cfg.gar, cfg.f, dict(cfg.gar_kwargs)
        X = torch.stack([r.float() for r in self.rows])            # [n, S] shard
        n = self.n
        if rule in DISTANCE_RULES or rule == "aksel":
            if rule == "aksel":
                med = gar.aggregate("median", X)
                part = ((X.double() - med.double()) ** 2).sum(1)
                part = torch.where(torch.isfinite(part), part, torch.full_like(part, math.inf))
                dist_ = self._sum_over_ranks(part)
                c = (n + 1) // 2 if kw.get("mode", "mid") == "mid" else n - f
                order = sorted(range(n), key=lambda j: (float(dist_[j]), j))
                w = torch.zeros(n, dtype=torch.float32)
                w[order[:c]] = 1.0 / c
                C = _native.require_for(X.device)
                g = C.cpu_combine(X, w) if C is not None else (w[:, None] * X).sum(0)
            else:
                D = self._sum_over_ranks(gar.pairwise_distances(X))
                m = cfg.m if cfg.m is not None else n - f - 2
                C = _native.require_for(X.device)
                if rule == "bulyan":
                    t = n - 2 * f - 2
                    if C is not None:
                        W = C.cpu_bulyan_weights(D, f, m, t)
                        g = C.cpu_coordwise(X, gar._MODE["bulyan-tail"], f, t - 2 * f, W.reshape(-1), t, 0, 1.0)
                    else:
                        g = gar._torch_closest_mean(ref.bulyan_weights(D, f, m).float() @ X, t - 2 * f)
                    w = None
                else:
                    if rule == "krum":
                        w = C.cpu_krum_weights(D, f, m)[0] if C is not None else ref.krum_weights(D, f, m).float()
                    else:
                        w = C.cpu_brute_weights(D, f) if C is not None else ref.brute_weights(D, f).float()
                    g = C.cpu_combine(X, w) if C is not None else (w[:, None] * X).sum(0)
            e.last_weights = w if rule != "bulyan" else None
        elif rule == "average":
            g = gar.aggregate("average", X).float()
        else:
            gkw = dict(kw)
            if rule not in ("median", "average-nan"):
                gkw["f"] = f
            if rule == "condense":
                gkw.setdefault("seed", cfg.seed + e.step_count)
            g = gar.aggregate(rule, X, **gkw).float()
        self._sgd_cpu(g, first)

    def _sgd_cpu(self, g: torch.Tensor, first: bool) -> None:
        cfg = self.e.cfg
        p, buf = self.e.flat.data[self.sl], self.e.mom
        with torch.no_grad():
            if cfg.weight_decay:
                g = g + cfg.weight_decay * p
            if cfg.momentum:
                if first:
                    buf.copy_(g)
                else:
                    buf.mul_(cfg.momentum).add_(g, alpha=1 - cfg.dampening)
                g = g + cfg.momentum * buf if cfg.nesterov else buf
            p.add_(g, alpha=-cfg.lr)

    def momentum_vector(self) -> torch.Tensor:
        """The full (unsharded) momentum buffer, all-gathered (checkpoints)."""
        if self.world == 1:
            return self.e.mom
        out = torch.empty(self.world * self.S, dtype=self.e.mom.dtype, device=self.e.mom.device)
        dist.all_gather_into_tensor(out, self.e.mom.clone())
        return out
