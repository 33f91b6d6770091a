"""Byzantine-resilient data-parallel training engine (collective form).

The reference trains with a parameter server that pulls every worker's gradient
over RPC, aggregates with a GAR and pushes the model back
(``applications/Aggregathor/trainer.py:231-243``, ``garfieldpp/server.py``), or,
in Garfield_CC, gathers every parameter tensor to rank 0 and broadcasts it back
(``applications/Garfield_CC/trainer.py:55-207``).

MI355X design:

1. every rank hosts ``workers_per_rank`` *logical workers* (f = 2 Multi-Krum needs
   n >= 7 gradients even on one GPU); each runs fwd/bwd on its own micro-batch
   (bf16 autocast) with ``p.grad`` aliased into one flat fp32 buffer;
2. the flat gradient is cast into this rank's row of slot j of the exchange
   buffer ``X[k, world, ld]`` and slot j is all-gathered (RCCL, async) while the
   next logical worker computes — only the last slot's transfer is exposed;
3. every rank runs the SAME deterministic HIP GAR on ``X`` viewed as ``[n, d]``
   (replicated-server semantics: no model broadcast needed);
4. the fused combine + SGD(momentum, weight decay) kernel updates the flat fp32
   master weights in one pass; replicas stay bit-identical.

Byzantine workers are simulated per global slot (``byzantine={slot: attack}``).
"""
from __future__ import annotations

import contextlib
import gc
import math
import os
import weakref
from dataclasses import dataclass, field

import torch
import torch.distributed as dist
import torch.nn as nn

from garfield_amd import _native
from garfield_amd.ops import gar
from garfield_amd.parallel.comm import DistContext, all_gather_rows, collectives_on
from garfield_amd.runtime.attacks import NEEDS_ESTIMATES, apply_attack
from garfield_amd.utils.flat import FlatParams
from garfield_amd.utils.profiling import PhaseTimer

# MIOpen's CK grouped-conv backward-weight solver is not HIP-graph-replay safe on
# ROCm 7 / gfx950: from the second replay of a captured backward it leaves whole
# bf16 weight gradients non-finite (diagnosed with scripts/debug_graph.py: fp32 and
# BatchNorm-free nets are unaffected, disabling only this solver fixes VGG/ResNet).
# It must be disabled before MIOpen picks solvers for the process, i.e. before
# the first convolution; users may override the variable explicitly.
os.environ.setdefault("MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS", "0")

WEIGHTED_RULES = {"average", "krum", "brute", "aksel"}
_LP_MODULES = (nn.modules.conv._ConvNd, nn.Linear)
COORD_RULES = {"median", "trimmed-mean", "averaged-median", "average-nan", "condense", "bulyan"}
LAYERWISE_RULES = {"krum", "bulyan", "brute", "aksel"}   # per-layer != flat only for distance-based rules
# Layer-wise Krum as device operations (gar_layerwise.hip: one segmented Gram launch, a batched
# selection, one segmented combine + SGD); "0" runs the per-segment loop (the reference form).
LW_DEVICE = os.environ.get("GARFIELD_LW_DEVICE", "1") != "0"
LW_JOB = 32768   # coordinates per job of the segmented kernels (a multiple of 64)


def lw_job_ranges(x0: int, x1: int, origin: int = 0) -> list:
    """[x0, x1) cut at the multiples of LW_JOB of the global coordinate (``origin``: the global
    coordinate of local 0): every job boundary inside a segment is then a multiple of 64 whatever the
    sharding, so the layer-wise tail's MFMA / exact split of the coordinates is sharding-invariant."""
    out, a = [], x0
    while a < x1:
        e = min(((a + origin) // LW_JOB + 1) * LW_JOB - origin, x1)
        out.append((a, e))
        a = e
    return out
# fp32 (no autocast) worker batching on the GPU (the reference's precision): "1" (default) the grouped
# NHWC executor on the fp32 kernels (conv_f32.hip, split-bf16 MFMA; bn_nhwc.hip in fp32), "0" the
# per-worker path.
FP32_GROUPED = os.environ.get("GARFIELD_FP32_GROUPED", "1")
# sharded steps with a comm stream: the grouped step captured as stages cut at the bucket boundaries,
# so the next forward's early layers run beside the late buckets' updates / all-gathers ("0": one graph)
STAGE_FORWARD = os.environ.get("GARFIELD_STAGE_FORWARD", "1") != "0"


@contextlib.contextmanager
def _capture_guard():
    """No cyclic garbage collection while HIP graphs are captured: a dead cycle holding a previous
    engine's graphs or events (freed by the collector at an arbitrary allocation) would destroy them
    in the middle of this capture (torch 2.10's torch.cuda.graph no longer collects first). Dead
    cycles are collected once before the capture instead."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


@dataclass
class EngineConfig:
    gar: str = "krum"
    f: int = 2
    m: int | None = None
    gar_kwargs: dict = field(default_factory=dict)
    workers_per_rank: int = 8
    lr: float = 0.1
    momentum: float = 0.9
    dampening: float = 0.0
    weight_decay: float = 5e-4
    nesterov: bool = False
    exchange_dtype: torch.dtype = torch.bfloat16
    autocast_dtype: torch.dtype | None = torch.bfloat16
    byzantine: dict = field(default_factory=dict)   # global slot -> attack name
    channels_last: bool = False
    seed: int = 1234
    cuda_graph: bool = False          # capture the whole step in a HIP graph after one eager step
    drop_bn_counters: bool = True     # BatchNorm num_batches_tracked += 1 is a launch per BN per worker
    profile_phases: bool = False      # HIP-event timers: compute / exchange / gar_update (see phase_times())
    lp_weights: bool = True           # bf16/fp16 working copies of conv/linear weights, refreshed by the update kernel
    # run the k local workers as ONE grouped NHWC batch (per-worker BN statistics and
    # per-worker weight gradients; parallel/grouped.py) when the model supports it.
    # None: on for GPU runs, off on CPU.
    worker_batching: bool | None = None
    # world > 1: aggregate sharded (all-to-all of coordinate shards, partial Gram
    # all-reduce, sharded update, all-gather of the master; parallel/sharded.py)
    # instead of all-gathering every gradient to every rank. None: on when world > 1.
    shard_gar: bool | None = None
    # Garfield_CC's per-layer aggregation (reference trainer.py:90-140: the GAR runs on each
    # parameter tensor separately). Differs from the flat rule for the distance-based GARs
    # (Krum, Bulyan, Brute, Aksel); identical for the coordinate-wise ones. Redundant
    # (unsharded) aggregation only.
    layerwise: bool = False
    # estimates of the colluding attacks (lie, empire), applied to the EXCHANGED rows so
    # they do not depend on how slots are placed on ranks: "fw" = the reference's
    # (byzWorker.py:108-143: the attacker's own honest gradient + fw - 1 other honest
    # gradients, here the lowest honest slots), "all" = every honest gradient
    collusion: str = "fw"
    # CPU rehearsal of the GPU's working-weight exchange: install the shadow (here fp32, the
    # master's dtype) on the CPU too, so the sharded path's weight all-gathers and compact
    # all-reduce of the non-shadowed parameters run in the multi-rank gloo tests
    shadow_cpu: bool = False


class _SlotIssuer:
    """Starts the per-slot all-gathers in slot order 0..k-1 on EVERY rank.

    Collectives pair up by call order, not by tensor: the local compute order puts a
    rank's Byzantine slots last (so colluders see the honest estimates) and differs
    between ranks, so a slot's all-gather is deferred until every lower slot has
    been issued."""

    def __init__(self, eng):
        self.eng = eng
        self.done = set()
        self.next = 0

    def ready(self, j: int) -> list:
        self.done.add(j)
        works = []
        while self.next in self.done:
            w = self.eng._gather_slot(self.next)
            if w is not None:
                works.append(w)
            self.next += 1
        return works


def _same_view(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.data_ptr() == b.data_ptr() and a.shape == b.shape and a.stride() == b.stride()
            and a.dtype == b.dtype)


def _stacked_view(ts):
    """The [k*B, ...] tensor the k equal-shaped tensors ``ts`` are consecutive row blocks of
    (views of one buffer), or None."""
    t0 = ts[0]
    B = t0.shape[0]
    if B == 0:
        return None
    for j, t in enumerate(ts):
        if (t.shape != t0.shape or t.stride() != t0.stride() or t.dtype != t0.dtype
                or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr()
                or t.storage_offset() != t0.storage_offset() + j * B * t0.stride(0)):
            return None
    return t0.as_strided((len(ts) * B, *t0.shape[1:]), t0.stride(), t0.storage_offset())


class RobustDataParallel:
    """Robust DP over one process per device (see module docstring)."""

    _supports_grouping = True   # subclasses with their own step() opt out
    _supports_sharding = True

    def __init__(self, model: nn.Module, loss_fn, ctx: DistContext, cfg: EngineConfig):
        self.ctx = ctx
        self.cfg = cfg
        self.device = ctx.device
        self.model = model.to(self.device)
        self._grouping = self._want_grouping(self.model)
        if (cfg.channels_last and self.device.type == "cuda") or self._grouping:
            self.model = self.model.to(memory_format=torch.channels_last)
        self.loss_fn = loss_fn
        if cfg.drop_bn_counters:
            for mod in self.model.modules():
                if isinstance(mod, nn.modules.batchnorm._BatchNorm) and mod.momentum is not None:
                    mod.num_batches_tracked = None  # only read when momentum is None
        self._sharded = self._want_sharded()
        from garfield_amd.parallel.sharded import shard_pad

        pad = shard_pad(ctx.world_size) if self._sharded else 64
        self.flat = FlatParams(self.model, device=self.device, with_grad=False, pad=pad)
        if ctx.is_distributed:
            dist.broadcast(self.flat.data, src=0)
        self.d, self.ld = self.flat.d, self.flat.ld
        # readers of the weights join a staged step first (weak: no engine <-> FlatParams cycle)
        self.flat.before_read = weakref.WeakMethod(self.synchronize)
        self.work_params = list(self.flat.params)   # what forward/backward sees (see _install_shadow)
        self._shadow = None
        self._install_shadow()
        self.k = cfg.workers_per_rank
        self.world = ctx.world_size
        self.rank = ctx.rank
        self.n = self.k * self.world
        if self.n > gar.LARGE_ROWS and self.device.type == "cuda":
            raise ValueError(f"at most {gar.LARGE_ROWS} logical workers per job on the GPU path, got {self.n}")
        # momentum: the whole vector, or this rank's shard when the aggregation is sharded
        self.mom = torch.zeros(self.ld // self.world if self._sharded else self.ld, dtype=torch.float32,
                               device=self.device)
        # exchange buffer X[k, world, ld]: row (j, rank) is local worker j's gradient; the
        # sharded form keeps the local rows only (X[k, 1, ld]) and all-to-alls shards of them
        self.xr = 0 if self._sharded else self.rank
        self.X = torch.zeros((self.k, 1 if self._sharded else self.world, self.ld), dtype=cfg.exchange_dtype,
                             device=self.device)
        self.G = None if self._sharded else self.X.view(self.n, self.ld)[:, : self.d]  # [n, d] GAR input
        # local slot order: honest workers first so colluders see their estimates
        self.local_slots = sorted(range(self.k), key=lambda j: (self.slot(j) in cfg.byzantine, j))
        self.step_count = 0
        self.last_weights = None
        self._C = _native.require_for(self.device) if self.device.type == "cuda" else None
        self._one = torch.ones(1, dtype=torch.float32, device=self.device)
        self._gagg = torch.zeros(self.ld, dtype=torch.float32, device=self.device) \
            if cfg.gar in COORD_RULES else None
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(cfg.seed + 7919 * self.rank)
        self._check_gar()
        self.timer = PhaseTimer(self.device, cfg.profile_phases)
        self._graph = None
        self._graph_failed = False
        self._tuning_agreed = False
        self._routed: set = set()     # (rows, sample shape) of grouped steps routed to the per-worker path
        self._static = None
        self._static_loss = None
        self._gexec = None
        if self._grouping:
            self._init_grouped(loss_fn)
        self._shard = None
        if self._sharded:
            from garfield_amd.parallel.sharded import ShardedAggregator

            bounds = self._gexec.bucket_offsets() if self._gexec is not None else ()
            self._shard = ShardedAggregator(self, bounds)

    # ------------------------------------------------------------------ #

    def _want_grouping(self, model: nn.Module) -> bool:
        from garfield_amd.parallel import grouped

        wb = self.cfg.worker_batching
        if wb is None:
            wb = self.device.type == "cuda"
        self._fp32_nhwc = False         # the grouped NHWC executor in fp32 (own kernels)
        if not (wb and self._supports_grouping):
            return False
        if self.device.type == "cuda":
            # bf16 activations with bf16 working weights (the grouped kernels' contract)
            if self.cfg.lp_weights and self.cfg.autocast_dtype == torch.bfloat16:
                return grouped.supports(model)
            # the reference's fp32: fp32 activations and weights on the fp32 grouped kernels
            if self.cfg.autocast_dtype is None and not self.cfg.lp_weights and FP32_GROUPED != "0":
                if grouped.supports(model):
                    self._fp32_nhwc = True
                    return True
            return False
        return grouped.supports(model)

    def _want_sharded(self) -> bool:
        from garfield_amd.parallel.sharded import SUPPORTED, layerwise_device_ok

        sg = self.cfg.shard_gar
        if sg is None:   # default: on for multi-rank jobs
            sg = self.ctx.is_distributed   # (or the one-rank run of the multi-rank collectives)
        if not (sg and self._supports_sharding):
            return False
        if self.ctx.world_size > 1 and not self.ctx.is_distributed:
            raise ValueError("sharded aggregation over several ranks needs an initialised process group")
        if self.cfg.gar not in SUPPORTED:
            raise ValueError(f"sharded aggregation does not support {self.cfg.gar!r} (shard_gar=False)")
        if (self.cfg.layerwise and self.cfg.gar in LAYERWISE_RULES and self.device.type == "cuda"
                and not layerwise_device_ok(self.cfg.gar, self.cfg.workers_per_rank * self.ctx.world_size,
                                            self.cfg.f)):
            if self.cfg.shard_gar:   # asked for explicitly: say why it cannot be honoured
                raise ValueError(f"shard_gar=True: the sharded layer-wise {self.cfg.gar!r} kernels do not take n="
                                 f"{self.cfg.workers_per_rank * self.ctx.world_size}, f={self.cfg.f} (leave shard_gar "
                                 f"unset to run the unsharded per-segment loop)")
            return False   # beyond the segmented device kernels: the unsharded per-segment loop
        return True

    def _gather_slot(self, j: int):
        """Start the all-gather of local worker j's slot (unsharded form only)."""
        if self._sharded or not collectives_on(self.world):
            return None
        return all_gather_rows(self.X[j], self.rank, async_op=True)

    def synchronize(self) -> None:
        """Make the current stream wait for every update, weight all-gather and BatchNorm-affine
        scatter of the last step still in flight on the comm stream. A staged sharded step
        returns before its layer3/layer4 buckets are updated (the next step's forward stages wait
        on them on the device); any other reader of ``model.parameters()`` / ``flat.data`` calls
        this first. The flat-vector readers (``flat.vector``, ``flat.reference_vector``,
        checkpoints) and ``evaluate`` do so themselves."""
        if getattr(self, "_shard", None) is not None:
            self._shard.join()

    def set_lr(self, lr: float) -> None:
        """Learning rate of the next updates (a scheduler hook): the fused combine + SGD
        kernel reads ``cfg.lr`` at every launch (the GAR and update are never captured)."""
        self.cfg.lr = float(lr)

    def momentum_vector(self) -> torch.Tensor:
        """The full momentum buffer (all-gathered when the optimizer state is sharded)."""
        return self._shard.momentum_vector() if self._shard is not None else self.mom

    def _init_grouped(self, loss_fn) -> None:
        from garfield_amd.ops.grouped import GradSink
        from garfield_amd.parallel.grouped import GroupedResNet

        offsets = {id(p): off for p, off in zip(self.work_params, self.flat.offsets)}
        nrow = self.X.shape[1]
        sink = GradSink(self.X.view(-1), nrow * self.ld, self.xr * self.ld, offsets, self.k)
        # bucket marks (sharded multi-rank exchange): the backward records an event when
        # it has written the gradients of layer4 + fc, then of layer3
        from garfield_amd.parallel.sharded import overlap_enabled

        buckets = ("layer4", "layer3") if self._sharded else ()
        self._gexec = GroupedResNet(self.model, self.k, sink, loss_fn, marks=buckets, offsets=offsets,
                                    signals=overlap_enabled(self.ctx.world_size))
        self._gx = self._gy = None
        self._gsrc = None
        self._gsrc_refs = None
        self._gloss = torch.zeros(self.k, dtype=torch.float32, device=self.device)
        self._ggraph = None

    def _install_shadow(self) -> None:
        """Low-precision working weights for the matmul-shaped layers.

        Under autocast every conv/linear weight is cast fp32 → bf16 on each forward
        and the bf16 weight gradient cast back to fp32 on each backward: two
        elementwise kernels per layer per logical worker (~900 launches and ~4.7 ms
        per ResNet-50 step on MI355X, see profiles/). Instead, those layers get
        bf16 parameters that are views of one flat ``shadow`` buffer laid out like the
        fp32 master buffer. The fused GAR update kernel writes the shadow in the same
        pass that updates the master weights, so the forward reads bf16 directly and
        the backward produces bf16 gradients that the flatten kernel copies into the
        exchange row as they are. The numbers are the same as with autocast: the cast
        is the same round-to-nearest-even, and autocast's weight gradient is the bf16
        gradient of that cast. BatchNorm and other parameters stay fp32 views of the
        master buffer."""
        lp = self.cfg.autocast_dtype
        if self.cfg.shadow_cpu and self.device.type == "cpu":
            lp = torch.float32
        elif not (self.cfg.lp_weights and self.device.type == "cuda" and lp in (torch.bfloat16, torch.float16)):
            return
        index = {id(p): i for i, p in enumerate(self.flat.params)}
        self._shadow = torch.zeros(self.ld, dtype=lp, device=self.device)
        views = list(self.flat.views(self._shadow))
        replaced = {}
        for mod in self.model.modules():
            if not isinstance(mod, _LP_MODULES):
                continue
            for name in ("weight", "bias"):
                p = mod._parameters.get(name)
                if p is None or id(p) not in index:
                    continue
                i = index[id(p)]
                if id(p) not in replaced:
                    replaced[id(p)] = nn.Parameter(views[i], requires_grad=True)
                    self.work_params[i] = replaced[id(p)]
                mod._parameters[name] = replaced[id(p)]
        self.sync_shadow()

    def shadow_param_ids(self) -> set:
        """ids of the working parameters that are views of the shadow (the rest are fp32 master
        views the forward reads directly)."""
        if self._shadow is None:
            return set()
        lo, hi = self._shadow.data_ptr(), self._shadow.data_ptr() + self._shadow.numel() * self._shadow.element_size()
        return {id(p) for p in self.work_params if lo <= p.data_ptr() < hi}

    def sync_shadow(self) -> None:
        """Refresh the low-precision working weights from the fp32 master weights
        (only needed after the master buffer is written outside the update kernel)."""
        shard = getattr(self, "_shard", None)
        if shard is not None:
            shard.master_stale = False   # the whole master was just written
        if self._shadow is not None:
            with torch.no_grad():
                self._shadow.copy_(self.flat.data)

    def slot(self, j: int) -> int:
        """Global slot id (row of the [n, d] GAR input) of local worker j."""
        return j * self.world + self.rank

    def _check_gar(self) -> None:
        from garfield_amd import aggregators

        rule = aggregators.get(self.cfg.gar)
        kw = dict(self.cfg.gar_kwargs)
        if self.cfg.m is not None:
            kw["m"] = self.cfg.m
        msg = rule.check(gradients=[torch.zeros(1)] * self.n, f=self.cfg.f, **kw)
        if msg is not None:
            raise ValueError(f"GAR {self.cfg.gar!r} with n={self.n}: {msg}")

    # ------------------------------------------------------------------ #

    def compute_local(self, batches) -> list:
        """Forward/backward of every local logical worker; returns the loss tensors.

        Autograd's per-parameter gradients are "stolen" (``p.grad = None`` before each
        backward, so no accumulate kernel runs) and one multi-tensor HIP kernel
        flattens + casts them into this worker's exchange row. One autocast region
        spans all local workers so the bf16 weight casts are cached across them.
        The all-gather of each slot starts as soon as its row is ready."""
        self.model.train()
        works, losses = [], []
        cuda = self.device.type == "cuda"
        amp = (torch.autocast("cuda", dtype=self.cfg.autocast_dtype)
               if (self.cfg.autocast_dtype is not None and cuda) else contextlib.nullcontext())
        params = self.work_params
        issue = _SlotIssuer(self)
        with amp:
            for j in self.local_slots:
                x, y = batches[j]
                for p in params:
                    p.grad = None
                loss = self.loss_fn(self.model(x), y)
                loss.backward()
                losses.append(loss.detach())
                # the honest gradient goes into the row; a Byzantine slot's row is then
                # attacked from it (sharded: at exchange time, bucket by bucket)
                self._write_row(self.X[j, self.xr, : self.d])
                if self._shard is None:
                    self._attack_rows(0, self.d, (j,))
                works += issue.ready(j)
        for p in params:
            p.grad = None
        for w in works:
            w.wait()
        return losses

    def _write_row(self, row: torch.Tensor) -> None:
        if self.device.type == "cuda":
            grads = []
            for p in self.work_params:
                g = p.grad
                grads.append(g if g is not None else torch.zeros_like(p))
            self._C.gpu_flatten_cast(grads, row)   # fp32 and bf16 sources, one launch
        else:
            self.flat.grads_flat(row, self.work_params)

    def _grad_vector(self) -> torch.Tensor:
        """Current local gradient as one fp32 vector (memory order)."""
        out = torch.empty(self.d, dtype=torch.float32, device=self.device)
        self._write_row(out)
        return out

    def aggregate_and_update(self) -> None:
        """Run the GAR on the gathered [n, d] gradients and apply the SGD update."""
        cfg = self.cfg
        first = self.step_count == 0
        if self._shard is not None:
            self._shard.aggregate_and_update(first)   # starts the exchange unless already started
            self.step_count += 1
            return
        self._collude([self.G[s] for s in range(self.n)])
        rule = cfg.gar
        kw = dict(cfg.gar_kwargs)
        if cfg.layerwise and rule in LAYERWISE_RULES:
            self._layerwise_update(rule, kw, first)
            self.step_count += 1
            return
        if self.device.type == "cuda" and self.n > gar.MAX_ROWS:
            self._large_update(rule, kw, first)
        elif self.device.type == "cuda":
            C = self._C
            param, mom = self.flat.data[: self.d], self.mom[: self.d]
            if rule in WEIGHTED_RULES:
                w = self._weights(rule, kw)
                self.last_weights = w
                C.gpu_combine_sgd(self.G, w, param, mom, None, self._shadow, cfg.lr, cfg.momentum, cfg.dampening,
                                  cfg.weight_decay, cfg.nesterov, first)
            else:
                g = self._gagg[: self.d]
                self._coordinate(rule, kw, g)
                C.gpu_combine_sgd(self._gagg.view(1, self.ld)[:, : self.d], self._one, param, mom, None, self._shadow,
                                  cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
        else:
            gkw = dict(kw)
            if rule not in ("average", "median", "average-nan"):
                gkw["f"] = cfg.f
            if cfg.m is not None and rule in ("krum", "bulyan"):
                gkw["m"] = cfg.m
            if rule == "condense":
                gkw.setdefault("seed", cfg.seed + self.step_count)
            g = gar.aggregate(rule, self.G.float(), **gkw).float()
            self._sgd_cpu(g, first)
        self.step_count += 1

    def _large_update(self, rule: str, kw: dict, first: bool) -> None:
        """More than MAX_ROWS (128) rows on the GPU (up to LARGE_ROWS = 1024, e.g. Bulyan with
        32 workers per GPU on 8 GPUs): the [n, d] set as one matrix on ``gar_large.hip``
        (compacted-weight combine, radix-select coordinate rules, split-K MFMA Gram for the
        selections), the aggregate rounded to the exchange dtype, then the fused update."""
        cfg = self.cfg
        if rule in WEIGHTED_RULES:
            w = self._weights(rule, kw)
            self.last_weights = w
            g = gar.combine(self.G, w)
        else:
            self.last_weights = None
            g = gar.aggregate(rule, self.G, **self._rule_kwargs())
        self._C.gpu_combine_sgd([g.contiguous()], self._one, self.flat.data[: self.d], self.mom[: self.d], None,
                                self._shadow, cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov,
                                first)

    def _layerwise_update(self, rule: str, kw: dict, first: bool) -> None:
        """The GAR on every parameter tensor's slice of the [n, d] rows (each parameter is
        one contiguous segment of the memory-order flat layout), then one update.

        GPU Krum runs as three device launches over all segments (``_layerwise_device``);
        otherwise a loop over the segments: weighted rules compute each segment's weights and
        combine it in fp32 (exactly the arithmetic of the device path), other rules aggregate
        the segment with the rule itself."""
        cfg = self.cfg
        gkw = dict(kw, f=cfg.f)
        if cfg.m is not None and rule in ("krum", "bulyan"):
            gkw["m"] = cfg.m
        cuda = self.device.type == "cuda"
        if cuda and LW_DEVICE and self.n <= gar.MAX_ROWS and (rule == "krum" or (rule == "bulyan" and self.n <= 64)):
            self._layerwise_device(rule, first)
            return
        g = self._gagg if self._gagg is not None else torch.zeros(self.ld, dtype=torch.float32, device=self.device)
        self._gagg = g
        ws = []
        for off, numel in self._segments():
            seg = self.G[:, off:off + numel]
            if rule in WEIGHTED_RULES:
                w = self._weights(rule, kw, seg if cuda else seg.float())
                ws.append(w.clone())
                gar.combine_into(seg, w, g[off:off + numel])
            else:
                g[off:off + numel].copy_(gar.aggregate(rule, seg if cuda else seg.float(), **gkw).float())
        self.last_weights = torch.stack(ws) if ws else None
        if cuda:
            self._C.gpu_combine_sgd(g.view(1, self.ld)[:, : self.d], self._one, self.flat.data[: self.d],
                                    self.mom[: self.d], None, self._shadow, cfg.lr, cfg.momentum, cfg.dampening,
                                    cfg.weight_decay, cfg.nesterov, first)
        else:
            self._sgd_cpu(g[: self.d], first)

    def _segments(self) -> list:
        """(offset, numel) of every parameter segment, by offset."""
        return sorted(zip(self.flat.offsets, self.flat.numels))

    def _layerwise_device(self, rule: str, first: bool) -> None:
        """Layer-wise Krum / Bulyan on device: per-segment Grams (one launch over a job table + one
        segmented reduction), every segment's selection in one batched launch, then Krum: one
        segmented combine fused with the SGD update; Bulyan: one segmented tail launch (each
        coordinate's t selection means with its segment's W, their averaged median) + the update."""
        cfg = self.cfg
        C = self._C
        lw = getattr(self, "_lw", None)
        if lw is None:
            segs = self._segments()
            jobs, seg_lo = [], [0]
            for s, (off, numel) in enumerate(segs):
                jobs.extend((a, e, s) for a, e in lw_job_ranges(off, off + numel))
                seg_lo.append(len(jobs))
            offs = [o for o, _ in segs] + [segs[-1][0] + segs[-1][1]]
            L, n = len(segs), self.n
            np_ = C.gram_padded(n)
            dev = self.device
            lw = self._lw = dict(
                jobs=torch.tensor(jobs, dtype=torch.int64, device=dev),
                seg_lo=torch.tensor(seg_lo, dtype=torch.int32, device=dev),
                seg_off=torch.tensor(offs, dtype=torch.int64, device=dev),
                slabs=torch.empty(len(jobs) * C.gram_slab_floats(n), dtype=torch.float32, device=dev),
                gram=torch.empty(L * np_ * np_, dtype=torch.float32, device=dev),
                w=torch.empty((L, n), dtype=torch.float32, device=dev),
                order=torch.empty((L, n), dtype=torch.int32, device=dev),
                scores=torch.empty((L, n), dtype=torch.float32, device=dev), L=L)
        n, f = self.n, cfg.f
        m = cfg.m if cfg.m is not None else n - f - 2
        G = self.G[:, : self.d]
        C.gpu_lw_gram(G, lw["jobs"], lw["seg_lo"], lw["slabs"], lw["gram"])
        if rule == "bulyan":
            t = n - 2 * f - 2
            W = lw.get("W")
            if W is None:
                W = lw["W"] = torch.empty((lw["L"], t, n), dtype=torch.float32, device=self.device)
            if self._gagg is None:
                self._gagg = torch.zeros(self.ld, dtype=torch.float32, device=self.device)
            g = self._gagg[: self.d]
            C.gpu_bulyan_select(lw["gram"], n, f, m, t, W, lw["L"])
            C.gpu_lw_bulyan_tail(G, lw["jobs"], W, t, t - 2 * f, g)
            C.gpu_combine_sgd(g.view(1, -1), self._one, self.flat.data[: self.d], self.mom[: self.d], None,
                              self._shadow, cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov,
                              first)
            self.last_weights = None
            return
        C.gpu_krum_select(lw["gram"], n, f, m, lw["w"], lw["order"], lw["scores"], lw["L"])
        C.gpu_lw_combine_sgd(G, lw["jobs"], lw["seg_off"], 0, lw["w"], self.flat.data[: self.d], self.mom[: self.d],
                             self._shadow, cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
        self.last_weights = lw["w"]

    def _weights(self, rule: str, kw: dict, G=None) -> torch.Tensor:
        f = self.cfg.f
        G = self.G if G is None else G
        if rule == "average":
            w = getattr(self, "_avg_w", None)
            if w is None:
                w = torch.full((self.n,), 1.0 / self.n, dtype=torch.float32, device=self.device)
                self._avg_w = w
            return w
        if rule == "krum":
            return gar.krum_weights(G, f, self.cfg.m)
        if rule == "brute":
            return gar.brute_weights(G, f)
        return gar.aksel_weights(G, f, kw.get("mode", "mid"))

    def _coordinate(self, rule: str, kw: dict, out: torch.Tensor, G=None) -> None:
        """Coordinate-wise rule (or Bulyan) over ``G`` (default: the [n, d] exchange rows;
        else a list of rows) into the fp32 vector ``out``."""
        C, f = self._C, self.cfg.f
        modes = gar._MODE
        G = self.G if G is None else G
        n = len(G) if isinstance(G, (list, tuple)) else G.shape[0]
        if rule == "bulyan":
            t = n - 2 * f - 2
            W = gar.bulyan_weights(G, f, self.cfg.m)
            C.gpu_coordwise(G, modes["bulyan-tail"], f, t - 2 * f, W.reshape(-1), t, 0, 1.0, out)
        elif rule == "median":
            C.gpu_coordwise(G, modes["median"], 0, 0, None, 0, 0, 1.0, out)
        elif rule == "trimmed-mean":
            C.gpu_coordwise(G, modes["trimmed-mean"], f, 0, None, 0, 0, 1.0, out)
        elif rule == "averaged-median":
            beta = kw.get("beta") or n - f
            C.gpu_coordwise(G, modes["averaged-median"], f, beta, None, 0, 0, 1.0, out)
        elif rule == "average-nan":
            C.gpu_coordwise(G, modes["average-nan"], 0, 0, None, 0, 0, 1.0, out)
        elif rule == "condense":
            C.gpu_coordwise(G, modes["condense"], f, 0, None, 0, self.cfg.seed + self.step_count,
                            float(kw.get("p", 0.9)), out)
        else:
            raise ValueError(rule)

    def _rule_kwargs(self) -> dict:
        cfg = self.cfg
        kw = dict(cfg.gar_kwargs)
        if cfg.gar not in ("average", "median", "average-nan"):
            kw["f"] = cfg.f
        if cfg.m is not None and cfg.gar in ("krum", "bulyan"):
            kw["m"] = cfg.m
        if cfg.gar == "condense":
            kw.setdefault("seed", cfg.seed + self.step_count)
        return kw

    def _update_from_rows(self, rows: list) -> None:
        """GAR over an explicit list of gradient rows (any subset of the slots, e.g. the
        Byzantine-PS workers or a quorum) + the SGD update of this replica."""
        cfg = self.cfg
        first = self.step_count == 0
        param, mom = self.flat.data[: self.d], self.mom[: self.d]
        if self.device.type == "cuda":
            C = self._C
            if cfg.gar in WEIGHTED_RULES:
                if cfg.gar == "krum":
                    w = gar.krum_weights(rows, cfg.f, cfg.m)
                elif cfg.gar == "brute":
                    w = gar.brute_weights(rows, cfg.f)
                elif cfg.gar == "aksel":
                    w = gar.aksel_weights(rows, cfg.f, cfg.gar_kwargs.get("mode", "mid"))
                else:
                    w = torch.full((len(rows),), 1.0 / len(rows), device=self.device)
                self.last_weights = w
                C.gpu_combine_sgd(rows, w, param, mom, None, self._shadow, cfg.lr, cfg.momentum, cfg.dampening,
                                  cfg.weight_decay, cfg.nesterov, first)
                return
            if self._gagg is None:
                self._gagg = torch.zeros(self.ld, dtype=torch.float32, device=self.device)
            g = self._gagg[: self.d]
            if len(rows) <= gar.MAX_ROWS:   # fp32 aggregate, as the synchronous step's
                self._coordinate(cfg.gar, dict(cfg.gar_kwargs), g, rows)
            else:
                g.copy_(gar.aggregate(cfg.gar, rows, **self._rule_kwargs()))
            C.gpu_combine_sgd([g], self._one, param, mom, None, self._shadow, cfg.lr, cfg.momentum, cfg.dampening,
                              cfg.weight_decay, cfg.nesterov, first)
        else:
            # as a [rows, d] fp32 matrix: the aggregate keeps fp32 (a list of 16-bit rows
            # would round it to the rows' dtype), as the synchronous step's
            g = gar.aggregate(cfg.gar, torch.stack([r.float() for r in rows]), **self._rule_kwargs()).float()
            self._sgd_cpu(g, first)

    def _sgd_cpu(self, g: torch.Tensor, first: bool) -> None:
        cfg = self.cfg
        p, buf = self.flat.data[: self.d], self.mom[: self.d]
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
            if self._shadow is not None:
                self._shadow[: self.d].copy_(p)

    def _eager_step(self, batches) -> torch.Tensor:
        self._join()
        with self.timer.phase("compute+exchange"):
            losses = self.compute_local(batches)
        with self.timer.phase("gar_update"):
            self.aggregate_and_update()
        return torch.stack(losses).float().mean()

    def phase_times(self) -> dict:
        """Mean ms per step of each phase (needs ``profile_phases=True``)."""
        return self.timer.summary()

    def graph_capturable(self) -> bool:
        random_attacks = {"random", "drop"} & set(self.cfg.byzantine.values())
        return (self.cfg.cuda_graph and self.device.type == "cuda" and not self._graph_failed
                and not random_attacks)

    def step(self, batches) -> torch.Tensor:
        """One synchronous robust training step; returns the mean local loss (device tensor).

        With ``cuda_graph`` the first step runs eagerly (warm-up: MIOpen algorithm
        selection, workspace allocation); then each local worker's forward +
        backward + flatten-cast into its exchange row is captured into its own HIP
        graph (one shared memory pool) and replayed: ~960 kernel launches per
        ResNet-50 worker become one graph launch. The RCCL all-gathers (overlapped
        with the next worker's graph) and the GAR + update stay eager (a handful
        of launches), so no collective is ever captured. New input tensors are
        copied into the static buffers.

        With worker batching (``_grouped_step``) the k local workers are one
        batched forward/backward instead, captured as ONE graph."""
        self._agree_tuning()
        if self._gexec is not None and self._groupable(batches):
            return self._grouped_step(batches)
        if not self.graph_capturable() or self.step_count == 0:
            return self._eager_step(batches)
        if self._graph is not None and not self._static_fits(batches):
            return self._eager_step(batches)   # e.g. a short last batch: the graphs keep their shapes
        if self._graph is None:
            self._capture(batches)
            if self._graph is None:
                return self._eager_step(batches)
        self._join()
        works = []
        issue = _SlotIssuer(self)
        with self.timer.phase("compute"):
            for j in self.local_slots:
                sx, sy = self._static[j]
                x, y = batches[j]
                # engine-owned static inputs: the caller's tensors are only ever read
                sx.copy_(x, non_blocking=True)
                sy.copy_(y, non_blocking=True)
                self._graph[j].replay()
                works += issue.ready(j)
        with self.timer.phase("exchange_wait"):
            for w in works:
                w.wait()
        with self.timer.phase("gar_update"):
            self.aggregate_and_update()
        return self._static_loss.mean()

    # ------------------------------------------------------------------ #
    # Worker batching: the k local workers as one grouped batch

    def _agree_tuning(self) -> None:
        """Once, at the start of the second step (before any capture): every rank adopts rank 0's
        measured kernel choices (``ops/tuning.py``), so all ranks replay the same kernels."""
        if self.step_count >= 1 and not self._tuning_agreed:
            self._tuning_agreed = True
            if self.device.type == "cuda" and collectives_on(self.world):
                from garfield_amd.ops import tuning

                tuning.agree()

    def _groupable(self, batches) -> bool:
        if len(batches) != self.k:
            return False
        x0, y0 = batches[0]
        if not (x0.dim() == 4 and all(x.shape == x0.shape and y.shape == y0.shape for x, y in batches)):
            return False
        return self._grouped_fits(x0.shape[0], tuple(x0.shape[1:]))

    def _grouped_fits(self, batch: int, sample_shape: tuple) -> bool:
        """Capacity routing, decided before anything runs or is captured: a grouped step whose largest
        tensor would pass the kernels' 32-bit indexing (e.g. 16 ImageNet workers x 250 images on one GPU:
        a 3.2e9-element stem activation) runs its workers one at a time instead (warned once)."""
        from garfield_amd.parallel import grouped
        from garfield_amd.utils.logging import warning

        rows = self.k * int(batch)
        if grouped.fits(self.model, rows, sample_shape):
            return True
        key = (rows, sample_shape)
        if key not in self._routed:
            self._routed.add(key)
            warning(f"grouped step of {self.k} workers x {batch} images {sample_shape}: its largest tensor has "
                    f"{grouped.largest_index(self.model, rows, sample_shape)} elements (> {grouped.INDEX_LIMIT}, the "
                    f"kernels' 32-bit indexing); running the workers one at a time")
        return False

    def _ensure_gbuf(self, B: int, sample_shape: tuple, label_shape: tuple = (), label_dtype=torch.int64) -> None:
        shape = (self.k * B, *sample_shape)
        if self._gx is None or tuple(self._gx.shape) != shape:
            fp32 = getattr(self, "_fp32_nhwc", False)
            dt = torch.bfloat16 if (self.device.type == "cuda" and not fp32) else torch.float32
            self._gx = torch.empty(shape, dtype=dt, device=self.device, memory_format=torch.channels_last)
            self._gy = torch.empty((self.k * B, *label_shape), dtype=label_dtype, device=self.device)
            self._ggraph = None
            self._gsrc = None

    def grouped_inputs(self, batch: int, sample_shape, label_dtype=torch.int64):
        """The grouped step's static input buffers ([k*batch, *sample_shape] channels_last, bf16 or
        fp32 by the step's precision, and the labels) for a producer that writes each step's batch in place
        (``data.fresh.DeviceBatches.attach``): no staging copy. None when the step is not grouped."""
        if self._gexec is None or not self._grouped_fits(int(batch), tuple(sample_shape)):
            return None
        self._ensure_gbuf(int(batch), tuple(sample_shape), (), label_dtype)
        return self._gx, self._gy

    def _stage_grouped(self, batches) -> None:
        """Concatenate the k micro-batches into the static grouped input buffers
        (skipped when the caller passes the very same, unmodified tensors again)."""
        x0, y0 = batches[0]
        B = x0.shape[0]
        self._ensure_gbuf(B, tuple(x0.shape[1:]), tuple(y0.shape[1:]), y0.dtype)
        key = tuple((id(x), x._version, id(y), y._version) for x, y in batches)
        if key != self._gsrc:
            with torch.no_grad():
                gx, gy = _stacked_view([x for x, _ in batches]), _stacked_view([y for _, y in batches])
                if gx is not None and gy is not None:
                    # the k batches are one buffer (DeviceBatches): written in place already, or 2 copies
                    if not _same_view(gx, self._gx):
                        self._gx.copy_(gx)
                    if not _same_view(gy, self._gy):
                        self._gy.copy_(gy)
                else:
                    for j, (x, y) in enumerate(batches):
                        self._gx[j * B:(j + 1) * B].copy_(x)
                        self._gy[j * B:(j + 1) * B].copy_(y)
            self._gsrc = key
            self._gsrc_refs = [t for xy in batches for t in xy]  # keep ids valid while cached

    def _grouped_compute(self) -> None:
        """The k local workers' forward/backward as one grouped pass (HIP graph from the
        second step on); every worker's gradient lands in its exchange row."""
        if (self.device.type == "cuda" and self.cfg.cuda_graph and not self._graph_failed and self.step_count >= 1
                and self._ggraph is None and getattr(self._gexec, "graph_safe", True)):
            self._capture_grouped()
        if self._shard is not None:   # this step's updates may run beside the next forward's stages
            self._shard.staged = isinstance(self._ggraph, list)
        if isinstance(self._ggraph, list):   # staged: each stage waits for the buckets it reads
            waits = self._shard.stage_waits(self._gexec.stage_ends(self.ld))
            main = torch.cuda.current_stream(self.device)
            for g, ev in zip(self._ggraph, waits):
                if ev is not None:
                    main.wait_event(ev)
                g.replay()
            self._gexec.replayed()
        elif self._ggraph is not None:
            self._join()
            self._ggraph.replay()
            self._gexec.replayed()   # the bucket signals captured in the graph fired once more
        else:
            self._join()
            self._gexec.run(self._gx, self._gy, self._gloss)

    def _staging(self) -> bool:
        """Whether the grouped step is captured as stages cut at the bucket boundaries (the
        sharded exchange with its comm stream and stream-ordered collectives, bf16)."""
        return (STAGE_FORWARD and self._shard is not None and self._shard.staging_ok()
                and hasattr(self._gexec, "run_stages") and self._gexec.stageable(self._gx))

    def _join(self) -> None:
        """The main stream waits for the previous step's buckets still in flight on the comm stream."""
        if self._shard is not None:
            self._shard.join()

    def _grouped_step(self, batches) -> torch.Tensor:
        self._stage_grouped(batches)
        works = []
        with self.timer.phase("compute"):
            self._grouped_compute()
            if self._shard is not None:   # buckets leave as the backward finishes them
                self._shard.start_exchange(self._gexec.mark_events())
            else:
                self._attack_local_rows()
                works = [w for w in (self._gather_slot(j) for j in range(self.k)) if w is not None]
        with self.timer.phase("exchange_wait"):
            for w in works:
                w.wait()
        with self.timer.phase("gar_update"):
            self.aggregate_and_update()
        gl = self._gloss
        if gl.is_cuda and gl.dtype == torch.float32 and gl.is_contiguous():
            return _native.native().gpu_mean_f32(gl)   # the reported loss without an ATen reduction
        return gl.mean()

    _DEFAULT_GEN = object()

    def _attack_rows(self, lo: int, hi: int, slots=None, gen=_DEFAULT_GEN) -> None:
        """Simulated Byzantine workers of this rank (``slots``: local worker ids, default
        all), on coordinates [lo, hi) of their rows, which hold their honest gradient.
        Every attack is coordinate-wise. The colluding attacks are skipped here: they
        run on the exchanged rows (``_collude``)."""
        cfg = self.cfg
        hi = min(hi, self.d)
        if lo >= hi or not cfg.byzantine:
            return
        gen = self._gen if gen is RobustDataParallel._DEFAULT_GEN else gen
        for j in (self.local_slots if slots is None else slots):
            attack = cfg.byzantine.get(self.slot(j))
            if attack is None or attack in NEEDS_ESTIMATES:
                continue
            row = self.X[j, self.xr, lo:hi]
            row.copy_(apply_attack(attack, row.float(), None, gen))

    def _attack_local_rows(self) -> None:
        """Overwrite the simulated Byzantine workers' rows (after the honest rows exist)."""
        self._attack_rows(0, self.d)

    def _collude(self, rows, slots=None) -> None:
        """The colluding attacks (lie, empire) on exchanged rows: ``rows[i]`` is (a
        coordinate slice of) the row of global slot ``slots[i]`` (default: i) and still
        holds that worker's honest gradient. Every rank holding the rows computes the
        same result (deterministic, coordinate-wise), so the sharded form (each owner on
        its coordinate shard) equals the redundant one.

        Estimates (``cfg.collusion``): "fw" follows the reference
        (``byzWorker.py:108-143``): the attacker's own honest gradient plus fw - 1 other
        honest gradients (here: the lowest honest slots), fw = the Byzantine workers
        among the rows; "all": every honest row."""
        byz = self.cfg.byzantine
        if not byz:
            return
        slots = list(range(len(rows))) if slots is None else list(slots)
        targets = [(i, byz[s]) for i, s in enumerate(slots) if byz.get(s) in NEEDS_ESTIMATES]
        if not targets:
            return
        honest = [i for i, s in enumerate(slots) if s not in byz]
        fw = sum(1 for s in slots if s in byz)
        peers = honest if self.cfg.collusion == "all" else honest[: max(fw - 1, 0)]
        if rows[0].is_cuda and rows[0].dtype in (torch.bfloat16, torch.float16, torch.float32) \
                and len(peers) + len(targets) <= gar.MAX_ROWS:
            # one fused pass per attack kind (gar_combine.hip k_collude): every Byzantine row from the
            # estimates read once, in the exchange dtype, no fp32 copies
            from garfield_amd.runtime.attacks import EMPIRE_EPS, LIE_Z

            for kind, param in (("lie", LIE_Z), ("empire", EMPIRE_EPS)):
                tg = [rows[i] for i, a in targets if a == kind]
                if tg:
                    self._C.gpu_collude([rows[i] for i in peers] + tg, len(peers), kind == "empire", param)
            return
        ests = [rows[i].float() for i in peers]
        for i, attack in targets:
            g = rows[i].float()
            rows[i].copy_(apply_attack(attack, g, torch.stack([g, *ests]), self._gen))

    def _capture_grouped(self) -> None:
        """Capture the grouped forward/backward (+ gradient scatter) as one HIP graph."""
        from garfield_amd.utils.logging import warning

        bns = [m for m in self.model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)
               and m.running_mean is not None]
        saved = [(m.running_mean.clone(), m.running_var.clone()) for m in bns]
        torch.cuda.synchronize()
        try:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):  # warm-up on the capture stream (per-stream library state)
                self._gexec.run(self._gx, self._gy, self._gloss)
            s.synchronize()
            mode = "thread_local" if collectives_on(self.world) else "global"
            if self._staging():
                # one graph per stage (shared memory pool), cut at the bucket boundaries of the
                # forward: the next step's early layers need not wait for the late buckets' updates
                graphs, pool, stages = [], None, self._gexec.run_stages(self._gx, self._gy, self._gloss)
                done = False
                with _capture_guard():
                    while not done:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode=mode):
                            done = next(stages, None) is None
                        graphs.append(g)
                        pool = g.pool()
                torch.cuda.current_stream(self.device).wait_stream(s)
                self._ggraph = graphs
            else:
                g = torch.cuda.CUDAGraph()
                with _capture_guard(), torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                    self._gexec.run(self._gx, self._gy, self._gloss)
                torch.cuda.current_stream(self.device).wait_stream(s)
                self._ggraph = g
        except Exception as e:  # capture unsupported: stay eager
            warning(f"HIP graph capture of the grouped step failed, running eagerly: {e!r}")
            self._graph_failed = True
            self._ggraph = None
        torch.cuda.synchronize()
        with torch.no_grad():  # the warm-up pass must not count as an extra step of the running statistics
            for m, (rm, rv) in zip(bns, saved):
                m.running_mean.copy_(rm)
                m.running_var.copy_(rv)

    def _worker_body(self, j: int, x, y, loss_out: torch.Tensor) -> None:
        """fwd + bwd of local worker j, gradient flattened (and attacked) into its row."""
        amp = (torch.autocast("cuda", dtype=self.cfg.autocast_dtype, cache_enabled=False)
               if self.cfg.autocast_dtype is not None else contextlib.nullcontext())
        for p in self.work_params:
            p.grad = None
        with amp:
            loss = self.loss_fn(self.model(x), y)
        loss.backward()
        loss_out.copy_(loss.detach().float())
        self._write_row(self.X[j, self.xr, : self.d])
        if self._shard is None:
            self._attack_rows(0, self.d, (j,), gen=None)   # captured: deterministic attacks only
        for p in self.work_params:
            p.grad = None

    def _static_fits(self, batches) -> bool:
        if len(batches) != len(self._static):
            return False
        return all(x.shape == sx.shape and y.shape == sy.shape and x.dtype == sx.dtype and y.dtype == sy.dtype
                   for (x, y), (sx, sy) in zip(batches, self._static))

    def _capture(self, batches) -> None:
        from garfield_amd.utils.logging import warning

        # engine-owned static inputs (never the caller's tensors: a loader's views must not be overwritten)
        self._static = [(x.clone(memory_format=torch.preserve_format), y.clone()) for x, y in batches]
        self._static_loss = torch.zeros(self.k, dtype=torch.float32, device=self.device)
        self.model.train()
        torch.cuda.synchronize()
        graphs = [None] * self.k
        pool = None
        try:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            # warm-up ON THE CAPTURE STREAM (lazy per-stream library state: BLAS / MIOpen
            # workspaces, algorithm caches) before any capture
            with torch.cuda.stream(s):
                for j in self.local_slots:
                    x, y = self._static[j]
                    self._worker_body(j, x, y, self._static_loss[j])
            s.synchronize()
            for j in self.local_slots:
                g = torch.cuda.CUDAGraph()
                mode = "thread_local" if collectives_on(self.world) else "global"  # RCCL watchdog thread
                with _capture_guard(), torch.cuda.graph(g, stream=s, pool=pool, capture_error_mode=mode):
                    x, y = self._static[j]
                    self._worker_body(j, x, y, self._static_loss[j])
                if pool is None:
                    pool = g.pool()
                graphs[j] = g
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._graph = graphs
        except Exception as e:  # capture unsupported: stay eager
            warning(f"HIP graph capture failed, running eagerly: {e!r}")
            self._graph_failed = True
            self._graph = None
            torch.cuda.synchronize()

    # ------------------------------------------------------------------ #

    def sync_master(self) -> None:
        """Collective in sharded multi-rank runs: refresh the fp32 master weights outside
        this rank's shards (the step all-gathers the bf16 working weights only)."""
        if self._shard is not None:
            self._shard.sync_master()

    def flat_model(self) -> torch.Tensor:
        """Reference-layout flat parameter vector (a view; clone to keep). Collective in
        sharded multi-rank runs (see ``sync_master``)."""
        self.sync_master()
        return self.flat.vector()

    def replica_checksum(self) -> float:
        self.sync_master()
        return float(self.flat.vector().double().sum())

    @torch.no_grad()
    def evaluate(self, batches, binary: bool = False) -> float:
        self._join()
        self.model.eval()
        correct = total = 0
        amp = (torch.autocast("cuda", dtype=self.cfg.autocast_dtype)
               if (self.cfg.autocast_dtype is not None and self.device.type == "cuda") else contextlib.nullcontext())
        for x, y in batches:
            with amp:
                out = self.model(x.to(self.device)).float()
            pred = out.round() if binary else out.argmax(1)
            correct += int((pred.view_as(y) == y.to(self.device)).sum())
            total += y.numel()
        self.model.train()
        return 100.0 * correct / max(total, 1)


def synthetic_batches(k: int, batch: int, shape, num_classes: int, device, seed: int = 0, channels_last=False,
                      learnable: bool = True):
    """k fixed synthetic (input, label) micro-batches resident on ``device``.

    With ``learnable`` the labels are a fixed function of the input (argmax of a
    fixed random projection, shared by all workers), so training makes progress."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    proj = torch.randn(int(torch.tensor(shape).prod()), num_classes,
                       generator=torch.Generator().manual_seed(424242))
    out = []
    for _ in range(k):
        x = torch.randn((batch, *shape), generator=g)
        if learnable:
            y = (x.flatten(1) @ proj).argmax(1)
        else:
            y = torch.randint(0, num_classes, (batch,), generator=g)
        x = x.to(device)
        if channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        out.append((x, y.to(device)))
    return out


def gar_overhead(step_ms: float, avg_step_ms: float) -> float:
    return 100.0 * (step_ms - avg_step_ms) / avg_step_ms if avg_step_ms > 0 else math.nan
