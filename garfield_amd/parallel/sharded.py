"""Sharded, bucketed robust aggregation: every rank aggregates 1/world of the coordinates.

The redundant form of the engine (``engine.RobustDataParallel`` with
``shard_gar=False``) all-gathers every worker's full gradient to every rank, so
each rank receives ``(world - 1) * k * d`` values per step and runs the whole
GAR itself: at 8 MI355X, 8 workers per GPU and ResNet-50 (d = 23.5M, bf16) that is
2.6 GB per rank per step over xGMI, the same order as the compute step.

Every rule the engine runs is either coordinate-wise or decides from per-pair
squared distances, and squared distances are additive over coordinate blocks:
``||g_i - g_j||^2 = sum_s ||g_i^(s) - g_j^(s)||^2``. So, per step:

1. the flat vector is cut into BUCKETS at layer boundaries, in the order the
   backward finishes them (layer4 + fc first: 64% of ResNet-50's parameters);
   each bucket is cut into ``world`` equal shards and rank r owns shard r of
   every bucket;
2. a bucket is exchanged as soon as the backward has written it: the grouped
   executor's captured graph bumps a device-side counter when its backward crosses
   the bucket boundary (``parallel/signals.py``), a comm stream waits for it ON THE
   DEVICE, applies the simulated attacks to that slice and sends the whole bucket in
   ONE group of RCCL point-to-point transfers straight from the exchange rows (each
   local row's shard ``dst`` is contiguous; this rank's own shard is read in place and
   never moves; through torch.distributed: a ``[dst, worker, shard]`` pack and one
   ``all_to_all_single``) -- so most of the exchange runs under the rest of the backward (every collective
   of the step is issued from the comm stream: a HIP event dependency on the main
   stream would slow the next graph replay, see signals.py);
3. distance-based rules (Krum/Multi-Krum, Bulyan's selection, Brute): each rank
   adds the partial Gram matrices of its shards (split-K MFMA kernel, one per
   bucket as it lands), the ``[n, n]`` partials are all-gathered (a few KB) and
   summed in rank order, so every rank sees the same matrix and makes the same
   selection; Aksel does the same with its per-row distances to the median;
4. the combine / coordinate-wise kernel and the fused SGD update run bucket by
   bucket on the owned shard (fp32 master shard, momentum shard: optimizer state
   is sharded) and write the bf16 working weights of the shard in the same pass;
5. the updated bf16 working weights are all-gathered per bucket (2 bytes per
   parameter, not the 4-byte fp32 master), each as soon as its bucket's update is
   queued (low coordinates first); the few fp32 parameters the forward reads
   directly (BatchNorm affine) travel in one small all-reduce.
   The fp32 master outside the owned shards is refreshed lazily
   (``sync_master``) for checkpoints and the reference-layout flat vector.

Replicas stay bit-identical (same gathered bytes everywhere).
Reference: the PS pull/aggregate/push loop of ``garfieldpp/server.py:112-159`` and
Garfield_CC's per-tensor gather/broadcast (``Garfield_CC/trainer.py:55-207,
288-314``). Condense draws its per-coordinate coin with the shard-local coordinate
index, so its mask differs from the unsharded run's (same Bernoulli(p) law).
"""
from __future__ import annotations

import contextlib
import math
import os

import torch
import torch.distributed as dist

from garfield_amd import _native
from garfield_amd.ops import gar
from garfield_amd.ops import reference as ref
from garfield_amd.parallel.comm import collectives_on, gloo_backend, world1_collectives
from garfield_amd.parallel.rccl import direct_backend
from garfield_amd.parallel.signals import Handoff

DISTANCE_RULES = {"krum", "brute", "bulyan"}
LAYERWISE_RULES = {"krum", "bulyan", "brute", "aksel"}
SUPPORTED = DISTANCE_RULES | {"average", "aksel", "median", "trimmed-mean", "averaged-median", "average-nan",
                              "condense"}


def layerwise_device_ok(rule: str, n: int, f: int) -> bool:
    """Whether the sharded GPU layer-wise path's device kernels take this configuration:
    the segmented Gram (``gpu_lw_gram``) and the batched selections need n <= MAX_ROWS, the
    layer-wise Bulyan tail t = n - 2f - 2 <= 64 selected rows, Brute's subset search n <= 64.
    Other configurations keep the unsharded engine's per-segment loop."""
    if n > gar.MAX_ROWS:
        return False
    if rule == "bulyan":
        return n - 2 * f - 2 <= 64
    if rule == "brute":
        return n <= 64
    return True


def shard_pad(world: int, base: int = 64) -> int:
    """Row padding such that every shard is a whole number of 64-element (16-byte aligned) blocks."""
    return base * world


def overlap_enabled(world: int = 1) -> bool:
    """Whether each bucket's exchange starts INSIDE the step's backward: the grouped
    executor's captured graph carries a device-side counter signal per bucket mark
    (``parallel/signals.py``) and the comm stream waits for it on the device. On by
    default when there is something to overlap (world > 1, or the one-rank run of the
    multi-rank collectives, ``comm.world1_collectives``); ``GARFIELD_OVERLAP=1`` forces it
    (e.g. the world-1 loopback exchange), ``0`` disables it."""
    v = os.environ.get("GARFIELD_OVERLAP", "")
    if v == "":
        return collectives_on(world)
    return v != "0"


class _Bucket:
    """One layer bucket [lo, hi) of the flat vector, cut into ``world`` shards of S.

    This rank's own shard never moves (its rows are read in place from the exchange rows).
    ``send[i, j]`` = local worker j's shard for the i-th OTHER rank in rank order (torch.distributed
    path only: packed so the whole bucket leaves in ONE ``all_to_all_single`` with an empty chunk for
    this rank), ``recv[pos[src], j]`` = shard ``rank`` of source rank src's local worker j (the row of
    global slot j * world + src), pos[src] = src below this rank, src - 1 above it; with ``slots`` =
    world the last slot holds this rank's own rows for the one-matrix (more than MAX_ROWS rows) path."""

    def __init__(self, lo: int, hi: int, world: int, rank: int, k: int, dev, dt, coll: bool, pack: bool,
                 slots: int):
        self.lo, self.hi = lo, hi
        self.S = (hi - lo) // world
        self.own = slice(lo + rank * self.S, lo + (rank + 1) * self.S)
        self.send = torch.empty((world - 1, k, self.S), dtype=dt, device=dev) if coll and pack else None
        self.recv = torch.empty((slots, k, self.S), dtype=dt, device=dev) if coll else None
        self.p2p = None        # the direct exchange's (sends, to, recvs, from) lists
        self.moff = 0          # offset of this bucket's shard in the momentum buffer
        self.works: list = []
        self.rows: list = []
        self.gagg = None
        self.done = None


class ShardedAggregator:
    """Bucketed all-to-all of the local gradient rows, sharded GAR, sharded SGD,
    all-gather of the working weights (see the module docstring)."""

    def __init__(self, engine, boundaries=()):
        e = engine
        self.e = e
        self.world, self.rank, self.k, self.n = e.world, e.rank, e.k, e.n
        if e.ld % self.world:
            raise ValueError("sharded aggregation needs the row length padded to a multiple of the world size")
        align = shard_pad(self.world)
        cuts = sorted({min(e.ld, ((int(b) + align - 1) // align) * align) for b in boundaries} - {0, e.ld})
        edges = [0, *cuts, e.ld]
        dev, dt = e.device, e.X.dtype
        # every collective of the step is issued from the comm stream (so RCCL's internal
        # stream depends on it, never on the main stream: parallel/signals.py), which
        # follows the main stream through device-side hand-offs
        # (world 1 without the loopback exchange: nothing to overlap, and a second active
        # queue alone costs the main stream's graph ~4-5 % (profiles/r3/probe_cross_stream.log):
        # everything stays on the main stream)
        # the one-rank run of the multi-rank collectives (GARFIELD_COLL_WORLD1=1 on a one-rank
        # process group, tests and traces: real RCCL calls, no shortcut taken for world 1)
        forced = self.world == 1 and world1_collectives()
        side = dev.type == "cuda" and (self.world > 1 or loopback_enabled() or overlap_enabled(self.world) or forced)
        self._comm_stream = torch.cuda.Stream(dev) if side else None
        self._handoff = Handoff(dev) if side else None
        # RCCL kernels straight onto the comm stream (rccl.py, GARFIELD_DIRECT_RCCL=1); None:
        # torch.distributed
        self._rccl = direct_backend(self.world, self.rank, side, forced and dev.type == "cuda")
        # whether the step issues its collectives (several ranks, or the forced one-rank run)
        self._coll = self.world > 1 or forced
        # ready order of the backward: highest coordinates (last layers) first
        # receive slot of each source rank (this rank's own rows: the last slot, one-matrix path only)
        self._pos = [src if src < self.rank else src - 1 for src in range(self.world)]
        self._pos[self.rank] = self.world - 1
        slots = self.world if self.n > gar.MAX_ROWS else self.world - 1
        self.buckets = [_Bucket(edges[i], edges[i + 1], self.world, self.rank, self.k, dev, dt, self._coll,
                                self._rccl is None, slots) for i in reversed(range(len(edges) - 1))]
        off = 0
        for b in sorted(self.buckets, key=lambda b: b.lo):
            b.moff = off
            off += b.S
        self.S = off                                   # owned coordinates = ld / world
        for b in self.buckets:
            b.rows = self._rows_of(b)
            if self._rccl is not None:
                b.p2p = self._p2p_of(b)
        self._one = torch.ones(1, dtype=torch.float32, device=dev)
        self._avg = torch.full((self.n,), 1.0 / self.n, dtype=torch.float32, device=dev)
        self._ws = {}
        self._started = False
        self._gathers: list = []
        self._scatters: list = []
        self._ready: list = []      # (bucket lo, event) of buckets finished on the comm stream
        self.staged = False         # the engine replays the next forward in bucket stages
        self.master_stale = False
        self._init_fp32_sync()

    # ------------------------------------------------------------------ #
    # layout

    def _rows_of(self, b: _Bucket) -> list:
        """Row (global slot j * world + src) -> its shard of bucket b, in slot order. This rank's
        own workers' rows are read in place from the exchange rows (the own shard never moves)."""
        e = self.e
        if not self._coll:
            return [e.X[j, 0, b.lo:b.hi] for j in range(self.k)]
        rows = []
        for s in range(self.n):
            src, j = s % self.world, s // self.world
            rows.append(e.X[j, 0, b.own] if src == self.rank else b.recv[self._pos[src], j])
        return rows

    def _p2p_of(self, b: _Bucket):
        """The direct exchange of bucket b as point-to-point transfers with no packing copy:
        local worker j's shard dst (contiguous in its exchange row) goes to rank dst, and
        source rank src's worker j lands in recv[pos[src], j]; pairs match in issue order."""
        e, W = self.e, self.world
        sends, to, recvs, frm = [], [], [], []
        for d in range(1, W):
            dst = (self.rank + d) % W            # staggered peers: every rank starts on a different link
            src = (self.rank - d) % W
            for j in range(self.k):
                sends.append(e.X[j, 0, b.lo + dst * b.S:b.lo + (dst + 1) * b.S])
                to.append(dst)
                recvs.append(b.recv[self._pos[src], j])
                frm.append(src)
        return sends, to, recvs, frm

    def _init_fp32_sync(self) -> None:
        """fp32 parameters the forward reads directly (not mirrored by the bf16 working
        weights): per bucket, their owned values travel in one all-reduce of a compact
        vector right after the bucket's weight all-gather."""
        e = self.e
        for b in self.buckets:
            b.np = None
        if e._shadow is None or not self._coll:
            return
        lp = e.shadow_param_ids()
        idx = []
        for p, wp, off, numel in zip(e.flat.params, e.work_params, e.flat.offsets, e.flat.numels):
            if id(wp) not in lp:
                idx.append(torch.arange(off, off + numel))
        if not idx:
            return
        gidx = torch.cat(idx)
        own = torch.zeros(e.ld, dtype=torch.bool)
        for b in self.buckets:
            own[b.own] = True
        for b in self.buckets:
            bidx = gidx[(gidx >= b.lo) & (gidx < b.hi)]
            if bidx.numel() == 0:
                continue
            b.np = (bidx.to(e.device), torch.nonzero(own[bidx]).flatten().to(e.device),
                    bidx[own[bidx]].to(e.device), torch.zeros(bidx.numel(), dtype=torch.float32, device=e.device))

    # ------------------------------------------------------------------ #
    # exchange

    @contextlib.contextmanager
    def _on_comm(self):
        """Make the comm stream current, after everything the main stream has queued so far
        (device-side hand-off). Collectives issued inside run after that work and leave the
        main stream free of cross-stream dependencies; ``work.wait()`` outside (main
        stream current) brings their results back."""
        if self._comm_stream is None:
            yield
            return
        main = torch.cuda.current_stream(self.e.device)
        self._handoff.to_comm(main, self._comm_stream)
        with torch.cuda.stream(self._comm_stream):
            yield

    def start_exchange(self, events=None) -> None:
        """Issue every bucket's exchange, in ready order: the simulated attacks on the
        bucket's slice of the local rows, then ONE group of transfers per bucket (3 per
        step for the ResNets). On the direct RCCL path that group is the point-to-point
        sends of each local row's shards straight from the exchange rows (no packing copy:
        on a memory-bound backward the copy alone cost as much HBM time as the transfer)
        and this rank's own shard stays where it is; through torch.distributed it is a pack
        into ``send[dst, j]`` and one ``all_to_all_single``. ``events[i]`` (optional) marks
        the point of the backward where bucket i's rows are complete; the comm stream
        waits on it, so the exchange overlaps the rest of the backward."""
        e = self.e
        side = self._comm_stream is not None
        use_events = (side and events is not None and overlap_enabled(self.world)
                      and len(events) >= len(self.buckets))
        if side and not use_events:   # after the whole backward
            self._handoff.to_comm(torch.cuda.current_stream(e.device), self._comm_stream)
        for i, b in enumerate(self.buckets):
            if side:
                s = self._comm_stream
                if use_events:
                    events[i].wait_on(s)      # a point inside the step's graph (signals.DeviceSignal)
                ctx = torch.cuda.stream(s)
            else:
                ctx = _nullctx()
            with ctx:
                e._attack_rows(b.lo, b.hi)
                b.works = []
                if self._coll and self._rccl is not None:   # straight from the exchange rows
                    self._rccl.exchange(*b.p2p, self._comm_stream)
                elif self._coll:
                    local = e.X[:, 0, b.lo:b.hi].view(self.k, self.world, b.S).transpose(0, 1)   # [dst, j, S]
                    r, W = self.rank, self.world
                    if r > 0:
                        b.send[:r].copy_(local[:r])
                    if r < W - 1:
                        b.send[r:].copy_(local[r + 1:])
                    split = [0 if q == r else self.k * b.S for q in range(W)]   # nothing to or from itself
                    w = dist.all_to_all_single(b.recv[:W - 1].view(-1), b.send.view(-1), split, split,
                                               async_op=True)
                    if side:     # the COMM stream waits for RCCL's internal stream (the main stream only
                        w.wait()  # ever waits on the comm stream's events: the cheap direction, signals.py)
                    else:
                        b.works.append(w)
                if side:
                    b.done = torch.cuda.Event(enable_timing=_TIMING)
                    b.done.record(s)
        self._started = True

    def _wait(self, b: _Bucket) -> None:
        for w in b.works:
            w.wait()
        b.works = []
        if b.done is not None:
            torch.cuda.current_stream(self.e.device).wait_event(b.done)   # main waits on comm: cheap
        self.e._collude(b.rows)   # colluding attacks on this rank's coordinate shard of every row

    def _sum_over_ranks(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's ``t`` summed in rank order (identical result on every rank)."""
        if not self._coll:
            return t.clone()
        return self._gather_ranks(t).sum(0)

    def _concat_ranks(self, t: torch.Tensor) -> torch.Tensor:
        if not self._coll:
            return t
        return self._gather_ranks(t).view(-1, *t.shape[1:])

    def _gather_ranks(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape]: every rank's t (a small all-gather issued from the comm stream)."""
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        src = t.contiguous().view(-1)
        with self._on_comm():
            if self._rccl is not None:
                self._rccl.all_gather(src, out.view(-1), self._comm_stream)
                work = None
            else:
                work = dist.all_gather_into_tensor(out.view(-1), src, async_op=True)
                if self._comm_stream is not None:   # the comm stream waits, then the main stream on it
                    work.wait()
                    work = None
        self._back_to_main(work)
        return out

    def _back_to_main(self, work=None) -> None:
        """The main stream waits for what was issued on the comm stream (and for a
        torch.distributed work): an event the MAIN stream waits on."""
        if work is not None:
            work.wait()
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.e.device).wait_stream(self._comm_stream)

    # ------------------------------------------------------------------ #

    def aggregate_and_update(self, first: bool) -> None:
        e, cfg = self.e, self.e.cfg
        if not self._started:
            self.start_exchange()
        self._gathers = []
        if cfg.layerwise and cfg.gar in LAYERWISE_RULES:   # per-tensor == flat for the coordinate rules
            self._layerwise(cfg, first)
        elif e.device.type == "cuda":
            self._gpu(cfg, first)
        else:
            self._cpu(cfg, first)
        self._started = False
        self._finish_gathers()

    def _gather_bucket(self, b: _Bucket, handoff: bool = True) -> None:
        """Start the all-gather of bucket b's updated parameters (the bf16 working weights
        when the forward reads those, else the fp32 master) as soon as its update is
        queued, then the compact all-reduce of the bucket's fp32 parameters the forward
        reads directly (BatchNorm affine): on RCCL it runs beside the remaining buckets'
        updates. ``handoff=False``: the update was issued on the comm stream itself."""
        e = self.e
        if not self._coll:
            return
        buf = e._shadow if e._shadow is not None else e.flat.data
        full, mine = buf[b.lo:b.hi], buf[b.own]
        ctx = self._on_comm() if handoff else torch.cuda.stream(self._comm_stream)
        with ctx:
            if self._rccl is not None:   # in place: this rank's block is its own shard
                self._rccl.all_gather(mine, full, self._comm_stream)
            else:
                if gloo_backend():
                    mine = mine.clone()  # gloo rejects an input aliasing the output
                w = dist.all_gather_into_tensor(full, mine, async_op=True)
                if self._comm_stream is not None:
                    w.wait()    # stream-ordered on the comm stream, as the direct path
                else:
                    self._gathers.append(w)
            if b.np is not None:
                idx, own_pos, own_idx, nb = b.np
                nb.zero_()
                nb[own_pos] = e.flat.data[own_idx]
                if self._rccl is not None:   # stream-ordered: scattered back on the comm stream
                    self._rccl.all_reduce_sum(nb, self._comm_stream)
                    e.flat.data[idx] = nb
                elif self._comm_stream is not None:
                    dist.all_reduce(nb, async_op=True).wait()
                    e.flat.data[idx] = nb
                else:
                    self._gathers.append(dist.all_reduce(nb, async_op=True))
                    self._scatters.append(b)

    def _finish_gathers(self) -> None:
        """Wait for the weight all-gathers and compact all-reduces: stream-ordered on RCCL
        (the main stream waits for the comm stream, or, with the next forward staged, each
        stage waits for its buckets' events: ``stage_waits``), host-side for torch.distributed."""
        e = self.e
        if not self._coll:
            if e._shadow is not None and e.device.type != "cuda":
                with torch.no_grad():
                    e._shadow.copy_(e.flat.data)
            return
        for w in self._gathers:
            w.wait()
        self._gathers = []
        for b in self._scatters:
            idx, _, _, nb = b.np
            e.flat.data[idx] = nb
        self._scatters = []
        if not self._ready:
            self._back_to_main()
        if e._shadow is not None:
            self.master_stale = True

    # ------------------------------------------------------------------ #
    # the next step's forward, staged at the bucket boundaries

    def staging_ok(self) -> bool:
        """Whether the updates can run beside the next forward: a comm stream, and every
        collective stream-ordered on it (the direct RCCL path; torch.distributed's works waited on
        by the comm stream; or nothing to exchange)."""
        return self._comm_stream is not None

    def _update_buckets(self, fn) -> None:
        """``fn(b)`` issues bucket b's update; buckets in update order (low coordinates first).
        With the next forward staged (``self.staged``), the first bucket's update stays on the
        main stream and the others run on the comm stream (one device-side hand-off), each
        bucket followed by its weight all-gather and an event (``self._ready``) that the next
        forward's stage reading it waits on: the stem-to-layer2 forward runs while the
        layer3/layer4 updates and all-gathers are still in flight."""
        order = self._update_order()
        staged = self.staged and self.staging_ok()
        for i, b in enumerate(order):
            if staged and i > 0:
                if i == 1:
                    self._handoff.to_comm(torch.cuda.current_stream(self.e.device), self._comm_stream)
                with torch.cuda.stream(self._comm_stream):
                    fn(b)
                self._gather_bucket(b, handoff=False)
            else:
                fn(b)
                self._gather_bucket(b)
            if staged and (i > 0 or self._coll):
                ev = torch.cuda.Event(enable_timing=_TIMING)
                ev.record(self._comm_stream)
                self._ready.append((b.lo, ev))

    def stage_waits(self, ends: list) -> list:
        """For each stage of the next forward (``ends[i]``: where the parameters it reads end),
        the event it must wait on (None: nothing pending): the last comm-stream bucket that
        starts below that end (the comm stream finishes buckets in coordinate order)."""
        out = []
        for hi in ends:
            ev = None
            for lo, e in self._ready:
                if lo < hi:
                    ev = e
            out.append(ev)
        self._ready = []
        return out

    def join(self) -> None:
        """The main stream waits for every pending bucket (a step that is not staged, or any
        reader of the parameters)."""
        if self._ready:
            main = torch.cuda.current_stream(self.e.device)
            for _, ev in self._ready:
                main.wait_event(ev)
            self._ready = []

    def quiesce(self) -> None:
        """Order torch.distributed collectives issued next after this aggregator's direct
        ones (same communicator): the main stream waits for the comm stream."""
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.e.device).wait_stream(self._comm_stream)
        self._ready = []

    def sync_master(self) -> None:
        """Collective: refresh the fp32 master outside this rank's shards (checkpoints,
        the reference-layout flat vector). Every rank must call it."""
        self.quiesce()
        if not self.master_stale or not self._coll:
            self.master_stale = False
            return
        data = self.e.flat.data
        for b in sorted(self.buckets, key=lambda b: b.lo):
            mine = data[b.own]
            if gloo_backend():
                mine = mine.clone()
            dist.all_gather_into_tensor(data[b.lo:b.hi], mine)
        self.master_stale = False

    # ------------------------------------------------------------------ #
    # GPU: the HIP building blocks, bucket by bucket

    def _wsp(self, b: _Bucket):
        ws = self._ws.get(b.lo)
        if ws is None:
            ws = self._ws[b.lo] = gar.Workspace(self.n, b.S, self.e.device)
        return ws

    def _param(self, b: _Bucket):
        e = self.e
        mom = e.mom[b.moff:b.moff + b.S]
        shadow = e._shadow[b.own] if e._shadow is not None else None
        return e.flat.data[b.own], mom, shadow

    def _gpu(self, cfg, first: bool) -> None:
        if self.n > gar.MAX_ROWS:
            return self._gpu_large(cfg, first)
        e, C = self.e, self.e._C
        rule, f, kw = cfg.gar, cfg.f, dict(cfg.gar_kwargs)
        n = self.n
        args = (cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
        modes = gar._MODE
        if rule in DISTANCE_RULES or rule == "aksel":
            total = None
            slabs = []
            for b in self.buckets:   # partial statistics as the buckets land
                self._wait(b)
                rows = gar.prepare(b.rows)
                ws = self._wsp(b)
                if rule == "aksel":
                    med = ws.get("aksel_med", b.S)
                    C.gpu_coordwise(b.rows, modes["median"], 0, 0, None, 0, 0, 1.0, med)
                    grid = C.sqdist_grid(b.S)
                    sl = ws.get("aksel_slabs", grid * n)
                    C.gpu_sqdist(b.rows, med, sl)
                    slabs.append(sl.view(grid, n))
                else:
                    g = gar._gram_into(C, rows, ws)
                    total = g.clone() if total is None else total.add_(g)
            if rule == "aksel":
                c = (n + 1) // 2 if kw.get("mode", "mid") == "mid" else n - f
                allslabs = self._concat_ranks(torch.cat(slabs))
                w = self._ws_any().get("weights", n)
                dists = self._ws_any().get("aksel_dists", n)
                C.gpu_aksel_select(allslabs.contiguous().view(-1), n, c, w, dists)
            else:
                total = self._sum_over_ranks(total)
                w = self._select(C, total, rule, f, cfg)
            if rule != "bulyan":
                e.last_weights = w

                def combine(b):
                    p, mom, sh = self._param(b)
                    C.gpu_combine_sgd(b.rows, w, p, mom, None, sh, *args)
                self._update_buckets(combine)
                return
            t = n - 2 * f - 2

            def tail(b):
                g = self._gagg(b)
                C.gpu_coordwise(b.rows, modes["bulyan-tail"], f, t - 2 * f, w, t, 0, 1.0, g)
                p, mom, sh = self._param(b)
                C.gpu_combine_sgd([g], self._one, p, mom, None, sh, *args)
            self._update_buckets(tail)
            return
        if rule == "average":
            e.last_weights = self._avg
        for b in self.buckets:   # coordinate-wise aggregation as the buckets land
            self._wait(b)
            if rule == "average":
                continue
            g = self._gagg(b)
            if rule == "median":
                C.gpu_coordwise(b.rows, modes["median"], 0, 0, None, 0, 0, 1.0, g)
            elif rule == "trimmed-mean":
                C.gpu_coordwise(b.rows, modes["trimmed-mean"], f, 0, None, 0, 0, 1.0, g)
            elif rule == "averaged-median":
                C.gpu_coordwise(b.rows, modes["averaged-median"], f, kw.get("beta") or n - f, None, 0, 0, 1.0, g)
            elif rule == "average-nan":
                C.gpu_coordwise(b.rows, modes["average-nan"], 0, 0, None, 0, 0, 1.0, g)
            elif rule == "condense":
                C.gpu_coordwise(b.rows, modes["condense"], f, 0, None, 0, cfg.seed + e.step_count + 7919 * b.lo,
                                float(kw.get("p", 0.9)), g)
            else:
                raise ValueError(f"sharded aggregation does not support {rule!r}")

        def update(b):
            p, mom, sh = self._param(b)
            if rule == "average":
                C.gpu_combine_sgd(b.rows, self._avg, p, mom, None, sh, *args)
            else:
                C.gpu_combine_sgd([self._gagg(b)], self._one, p, mom, None, sh, *args)
        self._update_buckets(update)

    def _matrix(self, b: _Bucket) -> torch.Tensor:
        """Bucket b's received shards as ONE [n, S] matrix (row pos[src] * k + j: the receive
        buffer as it lands, this rank's own rows copied into the last slot)."""
        if not self._coll:
            return torch.stack(b.rows)
        b.recv[self.world - 1].copy_(self.e.X[:, 0, b.own])
        return b.recv.view(self.n, b.S)

    def _gpu_large(self, cfg, first: bool) -> None:
        """More than MAX_ROWS rows (e.g. 8 GPUs x 32 workers): each bucket's shards as one
        matrix on the gar_large.hip kernels (split-K MFMA Gram and W·X with fp32 output,
        compacted combine, radix-select coordinate rules). Selections are made in slot order (the
        partial Grams permuted once), then mapped back to the matrix's row order."""
        e, C = self.e, self.e._C
        rule, f, kw = cfg.gar, cfg.f, dict(cfg.gar_kwargs)
        n, k, world = self.n, self.k, self.world
        args = (cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
        perm = torch.tensor([self._pos[s % world] * k + s // world for s in range(n)], device=e.device)
        mats = {}
        for b in self.buckets:
            self._wait(b)
            mats[b.lo] = self._matrix(b)
        if rule == "brute":   # C(n, f) subsets of n > 128 rows: the device search takes n <= 64
            raise ValueError(f"brute: n must be <= 64 on the GPU (n = {n})")
        if rule in ("krum", "bulyan"):
            total = None
            for b in self.buckets:
                g = gar.large_gram(mats[b.lo])                  # MFMA, fp32 (gar_large.hip)
                total = g if total is None else total.add_(g)
            gs = self._sum_over_ranks(total)[perm][:, perm]          # slot order on every rank
            m = cfg.m if cfg.m is not None else n - f - 2
            if rule == "krum":
                ws = gar.large_select(gs, f, m)
            else:
                W = gar.large_select(gs, f, m, bulyan=True)
                Wm = torch.empty_like(W)
                Wm[:, perm] = W
                t, beta = n - 2 * f - 2, n - 4 * f - 2
                e.last_weights = None
                for b in self._update_order():
                    V = gar.large_wx(Wm, mats[b.lo])               # [t, S] fp32 on MFMA (bounded: one shard)
                    g = self._gagg(b)
                    C.gpu_large_coord(V, 2, 0, beta, g)
                    p, mom, sh = self._param(b)
                    C.gpu_combine_sgd([g], self._one, p, mom, None, sh, *args)
                    self._gather_bucket(b)
                return
        elif rule == "average":
            ws = torch.full((n,), 1.0 / n, dtype=torch.float32, device=e.device)
        else:
            ws = None
        if ws is not None:
            e.last_weights = ws
            wm = torch.empty_like(ws)
            wm[perm] = ws
        for b in self._update_order():
            X = mats[b.lo]
            out = torch.empty(b.S, dtype=X.dtype, device=e.device)
            if ws is not None:
                C.gpu_large_combine(X, wm, out)
            elif rule in gar._LARGE_MODE:
                beta = kw.get("beta") or n - f
                C.gpu_large_coord(X, gar._LARGE_MODE[rule], f, beta, out)
            else:
                raise ValueError(f"sharded aggregation of more than {gar.MAX_ROWS} rows does not support {rule!r}")
            p, mom, sh = self._param(b)
            C.gpu_combine_sgd([out], self._one, p, mom, None, sh, *args)
            self._gather_bucket(b)

    def _update_order(self) -> list:
        """Buckets by ascending coordinates: the next forward reads the low ones first."""
        return sorted(self.buckets, key=lambda b: b.lo)

    def _ws_any(self):
        return self._wsp(self.buckets[0])

    def _gagg(self, b: _Bucket) -> torch.Tensor:
        if b.gagg is None:
            b.gagg = torch.zeros(b.S, dtype=torch.float32, device=self.e.device)
        return b.gagg

    def _select(self, C, gram_total, rule, f, cfg) -> torch.Tensor:
        n = self.n
        ws = self._ws_any()
        m = cfg.m if cfg.m is not None else n - f - 2
        if rule == "krum":
            w = ws.get("weights", n)
            order = ws.get("order", n, torch.int32)
            scores = ws.get("scores", n)
            C.gpu_krum_select(gram_total, n, f, m, w, order, scores)
            return w
        if rule == "brute":
            if n > 64:
                raise ValueError("brute: n must be <= 64 on the GPU")
            w = ws.get("weights", n)
            best = ws.get("brute_best", 1, torch.int64)
            C.gpu_brute_select(gram_total, n, f, best, w)
            return w
        t = n - 2 * f - 2   # bulyan
        W = ws.get("bulyan_W", t * n)
        C.gpu_bulyan_select(gram_total, n, f, m, t, W)
        return W

    # ------------------------------------------------------------------ #
    # Layer-wise rules, sharded. Per-parameter-segment squared distances are additive over the
    # coordinate shards too, so each rank adds the partial Grams of its owned coordinates per
    # segment ([L, n, n]; Aksel: the [L, n] partial distances to the coordinate-wise median), the
    # partials are summed over ranks in rank order, every rank selects every segment
    # (identically), and each rank aggregates + updates its owned coordinates with their
    # segment's selection (Krum / Brute / Aksel: weights; Bulyan: W [t, n] and the tail).

    def _lw_plan(self):
        """Per bucket: the owned range's pieces of every parameter segment (local coordinates)."""
        plan = getattr(self, "_lwp", None)
        if plan is not None:
            return plan
        e = self.e
        from garfield_amd.parallel.engine import lw_job_ranges

        segs = sorted(zip(e.flat.offsets, e.flat.numels))
        offs = [o for o, _ in segs] + [segs[-1][0] + segs[-1][1]]
        L = len(segs)
        plan = {"L": L, "offs": offs, "buckets": {}, "seg_id": {}}
        for b in self.buckets:
            o0, o1 = b.own.start, b.own.stop
            jobs, seg_lo = [], [0]
            sid = torch.full((b.S,), L, dtype=torch.int64)   # L: padding past the last segment
            for si in range(L):
                x0, x1 = max(offs[si], o0), min(offs[si + 1], o1)
                if x1 > x0:
                    sid[x0 - o0:x1 - o0] = si
                jobs.extend((a - o0, e - o0, si) for a, e in lw_job_ranges(x0, x1))
                seg_lo.append(len(jobs))
            plan["buckets"][b.lo] = (jobs, seg_lo)
            plan["seg_id"][b.lo] = sid.to(e.device)
        if e.device.type == "cuda":
            C, dev, n = e._C, e.device, self.n
            np_ = C.gram_padded(n)
            plan["seg_off"] = torch.tensor(offs, dtype=torch.int64, device=dev)
            for lo, (jobs, seg_lo) in list(plan["buckets"].items()):
                J = max(len(jobs), 1)
                plan["buckets"][lo] = dict(
                    J=len(jobs),
                    jobs=torch.tensor(jobs if jobs else [(0, 0, 0)], dtype=torch.int64, device=dev),
                    seg_lo=torch.tensor(seg_lo, dtype=torch.int32, device=dev),
                    slabs=torch.empty(J * C.gram_slab_floats(n), dtype=torch.float32, device=dev),
                    gram=torch.empty(L * np_ * np_, dtype=torch.float32, device=dev))
            plan["w"] = torch.empty((L, n), dtype=torch.float32, device=dev)
            plan["order"] = torch.empty((L, n), dtype=torch.int32, device=dev)
            plan["scores"] = torch.empty((L, n), dtype=torch.float32, device=dev)
            plan["best"] = torch.empty(1, dtype=torch.int64, device=dev)
            plan["np"] = np_
        self._lwp = plan
        return plan

    _AKSEL_CHUNK = 1 << 20   # coordinates per distance chunk: n x 1M x 8 B of transient memory

    def _lw_aksel_weights(self, cfg, plan, buckets) -> torch.Tensor:
        """Layer-wise Aksel: per segment, the c rows closest (squared distance, summed over the owned
        coordinates of every rank) to the coordinate-wise median get weight 1/c (ties by slot).
        ``buckets`` yields (bucket lo, its [n] owned row shards) one bucket at a time (on the GPU as
        each lands); the distances are accumulated per coordinate chunk, so the transient memory is
        one chunk of the rows, not fp32/fp64 copies of every bucket."""
        n, L = self.n, plan["L"]
        e = self.e
        D = torch.zeros((n, L + 1), dtype=torch.float64, device=e.device)
        for lo, rows in buckets:
            S = rows[0].numel()
            if e.device.type == "cuda":
                med = self._ws_any().get("lw_aksel_med", S)[:S]
                e._C.gpu_coordwise(rows, gar._MODE["median"], 0, 0, None, 0, 0, 1.0, med)
            else:
                med = gar.aggregate("median", torch.stack([r.float() for r in rows])).float()
            sid = plan["seg_id"][lo]
            for a in range(0, S, self._AKSEL_CHUNK):
                z = min(S, a + self._AKSEL_CHUNK)
                X = torch.stack([r[a:z] for r in rows]).float()
                D.index_add_(1, sid[a:z], ((X - med[a:z]) ** 2).double())
        D = self._sum_over_ranks(D[:, :L].t().contiguous())
        D = torch.where(torch.isfinite(D), D, torch.full_like(D, math.inf))
        c = (n + 1) // 2 if dict(cfg.gar_kwargs).get("mode", "mid") == "mid" else n - cfg.f
        idx = torch.sort(D, dim=1, stable=True).indices[:, :c]
        return torch.zeros((L, n), dtype=torch.float32, device=D.device).scatter_(1, idx, 1.0 / c)

    def _layerwise(self, cfg, first: bool) -> None:
        e = self.e
        rule = cfg.gar
        n, f = self.n, cfg.f
        m = cfg.m if cfg.m is not None else n - f - 2
        t = n - 2 * f - 2
        plan = self._lw_plan()
        L = plan["L"]
        if e.device.type == "cuda":
            C = e._C
            args = (cfg.lr, cfg.momentum, cfg.dampening, cfg.weight_decay, cfg.nesterov, first)
            if rule == "aksel":
                def landed():
                    for b in self.buckets:
                        self._wait(b)
                        yield b.lo, b.rows
                plan["w"].copy_(self._lw_aksel_weights(cfg, plan, landed()))
            else:
                total = None
                for b in self.buckets:          # partial per-segment Grams as the buckets land
                    self._wait(b)
                    bp = plan["buckets"][b.lo]
                    if bp["J"] == 0:
                        continue
                    C.gpu_lw_gram(b.rows, bp["jobs"], bp["seg_lo"], bp["slabs"], bp["gram"])
                    total = bp["gram"].clone() if total is None else total.add_(bp["gram"])
                if total is None:
                    total = torch.zeros_like(next(iter(plan["buckets"].values()))["gram"])
                total = self._sum_over_ranks(total)
                if rule == "bulyan":
                    W = plan.get("W")
                    if W is None:
                        W = plan["W"] = torch.empty((L, t, n), dtype=torch.float32, device=e.device)
                    C.gpu_bulyan_select(total, n, f, m, t, W, L)
                    e.last_weights = None
                    for b in self._update_order():
                        bp = plan["buckets"][b.lo]
                        g = self._gagg(b)
                        if bp["J"]:
                            C.gpu_lw_bulyan_tail(b.rows, bp["jobs"][: bp["J"]], W, t, t - 2 * f, g)
                        p, mom, sh = self._param(b)
                        C.gpu_combine_sgd([g], self._one, p, mom, None, sh, *args)
                        self._gather_bucket(b)
                    return
                if rule == "brute":
                    np2 = plan["np"] ** 2
                    for si in range(L):
                        C.gpu_brute_select(total[si * np2:(si + 1) * np2], n, f, plan["best"], plan["w"][si])
                else:
                    C.gpu_krum_select(total, n, f, m, plan["w"], plan["order"], plan["scores"], L)
            e.last_weights = plan["w"]
            for b in self._update_order():
                bp = plan["buckets"][b.lo]
                if bp["J"]:
                    p, mom, sh = self._param(b)
                    C.gpu_lw_combine_sgd(b.rows, bp["jobs"][: bp["J"]], plan["seg_off"], b.own.start, plan["w"],
                                         p, mom, sh, *args)
                self._gather_bucket(b)
            return
        # CPU (gloo): per-segment partial squared distances of the owned coordinates (fp64)
        for b in self.buckets:
            self._wait(b)
        Xs = {b.lo: torch.stack([r.float() for r in b.rows]) for b in self.buckets}   # [n, S] owned shards
        Cn = _native.require_for(torch.empty(0))
        if rule == "aksel":
            W = self._lw_aksel_weights(cfg, plan, ((b.lo, list(Xs[b.lo])) for b in self.buckets))
        else:
            D = torch.zeros((L, n, n), dtype=torch.float64)
            for b in self.buckets:
                X = Xs[b.lo].double()
                for a, z, si in plan["buckets"][b.lo][0]:
                    Y = X[:, a:z]
                    sq = (Y * Y).sum(1)
                    D[si] += sq[:, None] + sq[None, :] - 2.0 * (Y @ Y.T)
            D = self._sum_over_ranks(D)
            W = torch.zeros((L, t, n) if rule == "bulyan" else (L, n), dtype=torch.float32)
            for si in range(L):
                Ds = D[si].clamp_min(0)
                Ds.fill_diagonal_(math.inf)
                if rule == "krum":
                    W[si] = ref.krum_weights(Ds, f, m).float()
                elif rule == "brute":
                    W[si] = (Cn.cpu_brute_weights(Ds, f) if Cn is not None else ref.brute_weights(Ds, f)).float()
                else:
                    W[si] = (Cn.cpu_bulyan_weights(Ds, f, m, t) if Cn is not None
                             else ref.bulyan_weights(Ds, f, m)).float().view(t, n)
        e.last_weights = None if rule == "bulyan" else W
        for b in self._update_order():
            X = Xs[b.lo]
            g = torch.zeros(b.S, dtype=torch.float32)
            for a, z, si in plan["buckets"][b.lo][0]:
                if rule != "bulyan":
                    g[a:z] = (W[si][:, None] * X[:, a:z]).sum(0)
                elif Cn is not None:
                    g[a:z] = Cn.cpu_coordwise(X[:, a:z], gar._MODE["bulyan-tail"], f, t - 2 * f, W[si].reshape(-1), t,
                                              0, 1.0).float()
                else:
                    g[a:z] = gar._torch_closest_mean(W[si] @ X[:, a:z], t - 2 * f).float()
            self._sgd_cpu(b, g, first)
            self._gather_bucket(b)

    # ------------------------------------------------------------------ #
    # CPU (gloo): the owned shards concatenated, the C++ / oracle building blocks

    def _cpu(self, cfg, first: bool) -> None:
        e = self.e
        for b in self.buckets:
            self._wait(b)
        order = sorted(self.buckets, key=lambda b: b.lo)
        X = torch.cat([torch.stack([r.float() for r in b.rows]) for b in order], dim=1)   # [n, S] owned
        g = self._cpu_rule(cfg, X)
        pos = 0
        for b in order:
            self._sgd_cpu(b, g[pos:pos + b.S], first)
            self._gather_bucket(b)
            pos += b.S

    def _cpu_rule(self, cfg, X: torch.Tensor) -> torch.Tensor:
        e = self.e
        rule, f, kw = cfg.gar, cfg.f, dict(cfg.gar_kwargs)
        n = self.n
        if rule in DISTANCE_RULES or rule == "aksel":
            C = _native.require_for(X.device)
            if rule == "aksel":
                med = gar.aggregate("median", X)
                part = ((X.double() - med.double()) ** 2).sum(1)
                part = torch.where(torch.isfinite(part), part, torch.full_like(part, math.inf))
                dist_ = self._sum_over_ranks(part)
                c = (n + 1) // 2 if kw.get("mode", "mid") == "mid" else n - f
                order = sorted(range(n), key=lambda j: (float(dist_[j]), j))
                w = torch.zeros(n, dtype=torch.float32)
                w[order[:c]] = 1.0 / c
                e.last_weights = w
                return C.cpu_combine(X, w) if C is not None else (w[:, None] * X).sum(0)
            D = self._sum_over_ranks(gar.pairwise_distances(X))
            m = cfg.m if cfg.m is not None else n - f - 2
            if rule == "bulyan":
                t = n - 2 * f - 2
                e.last_weights = None
                if C is not None:
                    W = C.cpu_bulyan_weights(D, f, m, t)
                    return C.cpu_coordwise(X, gar._MODE["bulyan-tail"], f, t - 2 * f, W.reshape(-1), t, 0, 1.0)
                return gar._torch_closest_mean(ref.bulyan_weights(D, f, m).float() @ X, t - 2 * f)
            if rule == "krum":
                w = C.cpu_krum_weights(D, f, m)[0] if C is not None else ref.krum_weights(D, f, m).float()
            else:
                w = C.cpu_brute_weights(D, f) if C is not None else ref.brute_weights(D, f).float()
            e.last_weights = w
            return C.cpu_combine(X, w) if C is not None else (w[:, None] * X).sum(0)
        if rule == "average":
            return gar.aggregate("average", X).float()
        gkw = dict(kw)
        if rule not in ("median", "average-nan"):
            gkw["f"] = f
        if rule == "condense":
            gkw.setdefault("seed", cfg.seed + e.step_count)
        return gar.aggregate(rule, X, **gkw).float()

    def _sgd_cpu(self, b: _Bucket, g: torch.Tensor, first: bool) -> None:
        cfg = self.e.cfg
        p, buf, _ = self._param(b)
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
            sh = self.e._shadow
            if sh is not None:
                sh[b.own].copy_(p)

    # ------------------------------------------------------------------ #
    # optimizer state in the reference layout (checkpoints)

    def momentum_vector(self) -> torch.Tensor:
        """The full (unsharded) momentum buffer, all-gathered (collective)."""
        self.quiesce()
        e = self.e
        out = torch.zeros(e.ld, dtype=e.mom.dtype, device=e.mom.device)
        for b in sorted(self.buckets, key=lambda b: b.lo):
            mine = e.mom[b.moff:b.moff + b.S].clone()
            if not self._coll:
                out[b.lo:b.hi] = mine
            else:
                dist.all_gather_into_tensor(out[b.lo:b.hi], mine)
        return out

    def load_momentum(self, full: torch.Tensor) -> None:
        self.quiesce()
        e = self.e
        for b in self.buckets:
            e.mom[b.moff:b.moff + b.S].copy_(full[b.own])


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


# GARFIELD_EXCHANGE_TIMING=1: the per-bucket "exchange issued" events are timing events
# (scripts/overlap_timing.py reads them against the step's start and its backward's end)
_TIMING = os.environ.get("GARFIELD_EXCHANGE_TIMING", "0") == "1"


def loopback_enabled() -> bool:
    """GARFIELD_LOOPBACK_EXCHANGE=1 at world 1: run the exchange machinery of a multi-rank
    step (comm stream, in-graph bucket signals, device-side hand-offs, per-bucket events)
    with nothing to move, since a rank's own shard is read in place (traces, tests)."""
    return os.environ.get("GARFIELD_LOOPBACK_EXCHANGE", "0") == "1"
