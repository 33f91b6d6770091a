"""Garfield_CC: Byzantine-resilient training over collectives (one process per GPU).

Reference: ``pytorch_impl/applications/Garfield_CC/trainer.py`` (flags ``--master
--rank --dataset --batch --num_ps --num_workers --fw --fps --model --loss --lr
--momentum --wd --epochs --aggregator --mar --backend --bench --log``; per-parameter
``dist.gather``/``broadcast`` on gloo because "NCCL does not support gather").

Here every gradient exchange is ONE flat all-gather per logical-worker slot over
RCCL (``--backend nccl``, default on GPU) or gloo, and:

* ``--num_ps 0`` (or 1 with ``--fps 0``): replicated-server robust DP — every rank is
  a worker (``--workers_per_rank`` logical workers) and runs the GAR redundantly
  (``parallel.engine.RobustDataParallel``);
* ``--num_ps P >= 2``: Byzantine-server mode — ranks < P are server replicas, the
  others workers; servers aggregate worker gradients with ``--aggregator`` and every
  rank aggregates the servers' models with ``--mar`` (``parallel.byzps``).

Launch: ``torchrun --nproc-per-node 8 -m garfield_amd.apps.garfield_cc ...`` (reads
RANK / WORLD_SIZE / LOCAL_RANK), or one process per node with ``--rank/--master``.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

from garfield_amd.apps.common import str2bool
from garfield_amd.data.datasets import CLASSES, DatasetManager
from garfield_amd.models import build_model
from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig
from garfield_amd.parallel.comm import init_distributed, shutdown
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel
from garfield_amd.parallel.quorum import QuorumConfig, QuorumDataParallel
from garfield_amd.utils.checkpoint import Checkpoints
from garfield_amd.utils.logging import info, set_rank_prefix


def multistep_lr(base: float, milestones, gamma: float, epoch: int) -> float:
    """Learning rate of 0-based ``epoch`` under the reference's schedule: ``MultiStepLR``
    whose ``scheduler.step()`` runs at the START of every epoch (Garfield_CC
    trainer.py:288-291), so the rate drops once epoch + 1 reaches a milestone."""
    return base * gamma ** sum(1 for m in milestones if epoch + 1 >= m)


def parse(argv=None):
    p = argparse.ArgumentParser(description="Garfield_CC (Garfield-MI355X, collectives)")
    p.add_argument("--master", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    p.add_argument("--port", type=int, default=int(os.environ.get("MASTER_PORT", 29500)))
    p.add_argument("--rank", type=int, default=None)
    p.add_argument("--dataset", default="cifar10")
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--num_ps", type=int, default=0)
    p.add_argument("--num_workers", type=int, default=None, help="worker ranks (default: world - num_ps)")
    p.add_argument("--workers_per_rank", type=int, default=1, help="logical workers hosted by each worker rank")
    p.add_argument("--fw", type=int, default=0)
    p.add_argument("--fps", type=int, default=0)
    p.add_argument("--model", default="resnet18")
    p.add_argument("--loss", default="cross-entropy")
    p.add_argument("--lr", type=float, default=0.1)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--wd", type=float, default=5e-4)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr_milestones", default=None,
                   help="comma-separated epochs where the learning rate is multiplied by --lr_gamma (default: "
                        "25,50 for resnet50, as the reference's MultiStepLR, trainer.py:273-274,290-291; none else)")
    p.add_argument("--lr_gamma", type=float, default=0.1)
    p.add_argument("--num_iter", type=int, default=0, help="stop after this many iterations (0: epochs)")
    p.add_argument("--aggregator", default="vanilla", help="GAR name; vanilla = average (reference default)")
    p.add_argument("--mar", default="median")
    p.add_argument("--attack", default="", help="attack of the fw Byzantine worker slots")
    p.add_argument("--ps_attack", default="", help="attack of the fps Byzantine servers")
    p.add_argument("--ps_workers", type=str2bool, default=False,
                   help="Byzantine-server mode: server ranks also host --workers_per_rank logical workers")
    p.add_argument("--quorum", type=int, default=0,
                   help="aggregate only the rows of the fastest QUORUM ranks each step (reference server.py:134-155, "
                        "fastest n - f; parallel/quorum.py); 0 = wait for every rank")
    p.add_argument("--straggler", default="", help="fault injection for --quorum: RANK:SECONDS[,RANK:SECONDS]")
    p.add_argument("--backend", default=None, help="nccl (RCCL) or gloo")
    p.add_argument("--exchange_dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--cuda_graph", type=str2bool, default=True)
    p.add_argument("--bench", type=str2bool, default=False)
    p.add_argument("--log", type=str2bool, default=False)
    p.add_argument("--acc_freq", type=int, default=0)
    p.add_argument("--layerwise", type=str2bool, default=False,
                   help="apply the GAR per parameter tensor like the reference (trainer.py:90-140); the default "
                        "aggregates the flat gradient (same result for coordinate-wise rules)")
    p.add_argument("--checkpoint", default="", help="checkpoint directory (reference-layout flat vector + "
                   "momentum + BatchNorm buffers; utils/checkpoint.py)")
    p.add_argument("--checkpoint_freq", type=int, default=0, help="save every this many iterations (0: at the end)")
    p.add_argument("--resume", type=str2bool, default=False, help="restore the newest checkpoint of --checkpoint")
    return p.parse_args(argv)


def main(argv=None, results: dict | None = None):
    a = parse(argv)
    if a.rank is not None:
        world = a.num_ps + (a.num_workers or 1)
        os.environ.update(RANK=str(a.rank), WORLD_SIZE=str(world), MASTER_ADDR=a.master, MASTER_PORT=str(a.port))
        os.environ.setdefault("LOCAL_RANK", str(a.rank % max(torch.cuda.device_count(), 1)))
    ctx = init_distributed(backend=a.backend)
    set_rank_prefix(f"[rank {ctx.rank}] " if ctx.world_size > 1 else "")
    torch.manual_seed(1234)
    ncls = CLASSES.get(a.dataset, 10)
    loss_fn = F.nll_loss if a.loss == "nll" else (F.binary_cross_entropy if a.loss == "binary-cross-entropy"
                                                    else F.cross_entropy)
    model = build_model(a.model, num_classes=ncls)
    xdt = torch.bfloat16 if a.exchange_dtype == "bf16" else torch.float32
    k = a.workers_per_rank
    mar = a.mar
    if mar in ("crash", "vanilla"):
        # crash-tolerant / vanilla servers (reference trainer.py:97,137,520-523): no Byzantine server, the
        # trusted PS 0 broadcasts its aggregate. Every server here computes the same deterministic
        # aggregate from the same gradients, so averaging the identical server models is that broadcast.
        if a.fps != 0:
            raise SystemExit(f"--mar {mar} tolerates no Byzantine server: use --fps 0")
        mar = "average"
    byz_mode = a.num_ps >= 2 or (a.num_ps == 1 and a.fps > 0)
    worker_ranks = list(range(a.num_ps, ctx.world_size)) if (byz_mode and not a.ps_workers) \
        else list(range(ctx.world_size))
    # Byzantine logical workers: the first fw global worker slots (slot = j * world + rank)
    slots = sorted(j * ctx.world_size + r for j in range(k) for r in worker_ranks)
    byz = {s: a.attack for s in slots[: a.fw]} if a.attack else {}
    # --aggregator vanilla is the reference default: plain averaging (trainer.py:83-84,444-445)
    gar_name = "average" if a.aggregator == "vanilla" else a.aggregator
    # f = fw as in the reference (gar(gradients, f=fw)); a rule whose check needs f >= 1 fails loudly
    common = dict(gar=gar_name, f=a.fw, workers_per_rank=k, lr=a.lr, momentum=a.momentum, weight_decay=a.wd,
                  exchange_dtype=xdt, byzantine=byz, cuda_graph=a.cuda_graph)
    if a.layerwise:
        common.update(layerwise=True)
    if byz_mode:
        eng = ByzantinePSDataParallel(model, loss_fn, ctx,
                                      ByzPSConfig(num_ps=a.num_ps, fps=a.fps, mar=mar, ps_attack=a.ps_attack,
                                                  ps_workers=a.ps_workers, **common))
    elif a.quorum:
        delays = {int(r): float(t) for r, t in (x.split(":") for x in a.straggler.split(",") if x)}
        eng = QuorumDataParallel(model, loss_fn, ctx, QuorumConfig(quorum=a.quorum, straggler_delay=delays, **common))
    else:
        eng = RobustDataParallel(model, loss_fn, ctx, EngineConfig(**common))
    # data: logical worker j of rank r trains on partition (its worker index)
    nwork = len(worker_ranks) * k
    my_index = worker_ranks.index(ctx.rank) if ctx.rank in worker_ranks else 0
    loaders = []
    for j in range(k):
        mgr = DatasetManager(a.dataset, a.batch, nwork, nwork, j * len(worker_ranks) + my_index, device=ctx.device)
        loaders.append(mgr.get_train_set())
    test = DatasetManager(a.dataset, a.batch, 1, 1, 0, device=ctx.device).get_test_set()
    iters = a.num_iter or a.epochs * min(len(ld) for ld in loaders)
    ck = Checkpoints(a.checkpoint) if a.checkpoint else None
    start = 0
    if ck is not None and a.resume and ck.latest() is not None:
        ck.restore(eng)
        start = eng.step_count
        if ctx.rank == 0:
            info(f"resumed from {ck.path(start)} (iteration {start})")
    per_epoch = max(min(len(ld) for ld in loaders), 1)
    ms = a.lr_milestones if a.lr_milestones is not None else ("25,50" if a.model == "resnet50" else "")
    milestones = [int(x) for x in ms.split(",") if x.strip()]
    lrs = []
    t0 = time.time()
    loss = None
    for i in range(start, iters):
        if i % per_epoch == 0 or i == start:   # the reference steps its scheduler at each epoch's start
            eng.set_lr(multistep_lr(a.lr, milestones, a.lr_gamma, i // per_epoch))
            lrs.append(eng.cfg.lr)
        batches = [ld[i] for ld in loaders]
        ts = time.perf_counter()
        loss = eng.step(batches)
        if a.bench:
            if ctx.device.type == "cuda":
                torch.cuda.synchronize()
            info(f"iteration {i}: {1000 * (time.perf_counter() - ts):.2f} ms")
        if a.log:
            info(f"iteration {i} loss {float(loss):.4f}")
        if a.acc_freq and (i % a.acc_freq == 0 or i == iters - 1) and ctx.rank == 0:
            info(f"iteration {i} accuracy {eng.evaluate(test, binary=ncls == 1):.2f} time {time.time() - t0:.1f}s")
        if ck is not None and a.checkpoint_freq and (i + 1) % a.checkpoint_freq == 0:
            ck.save(eng, write=ctx.rank == 0)   # every rank: collectives of the sharded engine
    if ck is not None and not a.checkpoint_freq:
        ck.save(eng, write=ctx.rank == 0)
    if hasattr(eng, "finish"):
        eng.finish()   # quorum engine: late rows still in flight
    acc = eng.evaluate(test, binary=ncls == 1)
    checksum = eng.replica_checksum()   # collective in sharded runs
    if ctx.rank == 0:
        info(f"final accuracy {acc:.2f} after {iters} iterations ({time.time() - t0:.1f}s)")
        info(f"replica checksum {checksum:.12e}")
    if results is not None:
        results.update(accuracy=acc, checksum=checksum, loss=float(loss) if loss is not None else None, lrs=lrs)
    shutdown(ctx)
    return acc


if __name__ == "__main__":
    main(sys.argv[1:])
