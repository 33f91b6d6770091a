#!/usr/bin/env python3
"""Headline benchmark: img/s of Byzantine-resilient ResNet-50 training with f=2
Multi-Krum on 1..8 MI355X (BASELINE.json), plus the GAR overhead vs ``average``.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it is
launched by ``torch.distributed.run`` with one rank per GPU (RCCL). W untimed warmup
steps, then EXACTLY K timed steps bracketed by barrier + synchronize, max over
ranks; rank 0 prints one JSON line.

Workload (fixed per GPU => weak scaling): each GPU hosts ``--workers-per-gpu``
logical workers (default 8, so f = 2 Multi-Krum's n >= 2f + 3 = 7 holds on one GPU),
each computing a full forward/backward of ResNet-50 (torchvision architecture,
10 classes, random init) on its own synthetic CIFAR-10-shape micro-batch of
``--batch`` images (default 250: the reference Garfield_CC ResNet-50 config,
``PT/applications/Garfield_CC/run_exp.sh``), bf16 autocast. Every step: the GPU's
logical workers run as ONE grouped NHWC forward/backward (per-worker BatchNorm
statistics and per-worker weight gradients, HIP BN/ReLU/residual kernels, one HIP
graph) -> per-worker bf16 gradient rows -> RCCL all-gather into the [n, d]
buffer -> HIP Multi-Krum (MFMA Gram, on-device selection) -> fused combine +
SGD(momentum 0.9, wd 5e-4) on fp32 master weights.
img/s = n_logical x batch / step time (whole job).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _self_launch() -> int | None:
    """``python bench.py --gpus N`` (N > 1) without a torchrun environment: start
    ``torch.distributed.run`` with N ranks on this node as a CHILD process and
    return its exit code. Runs before torch is imported, so nothing has touched
    the GPU yet (and it is never an exec)."""
    if "WORLD_SIZE" in os.environ:
        return None
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=1)
    known, _ = p.parse_known_args()
    if known.gpus <= 1:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


if __name__ == "__main__":
    _rc = _self_launch()
    if _rc is not None:
        sys.exit(_rc)

import torch  # noqa: E402
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from garfield_amd.models import build_model, num_parameters  # noqa: E402
from garfield_amd.parallel.comm import init_distributed, shutdown  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402

BASELINE_VALUE = None  # BASELINE.json "published": {} -> no reference number to divide by


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--dataset", default="cifar10", choices=["cifar10", "imagenet"])
    p.add_argument("--batch", type=int, default=250, help="micro-batch per logical worker")
    p.add_argument("--workers-per-gpu", type=int, default=8)
    p.add_argument("--gar", default="krum")
    p.add_argument("--f", type=int, default=2)
    p.add_argument("--exchange-dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                   help="fp32: the reference's precision end to end (no autocast, fp32 exchange rows, fp32 weights: "
                        "the grouped NHWC executor on the fp32 kernels)")
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--overhead", action="store_true",
                   help="also time the same job with the 'average' GAR and report the Krum overhead")
    p.add_argument("--cudnn-benchmark", action="store_true")
    p.add_argument("--no-graph", action="store_true", help="disable per-worker HIP graph capture (eager launches)")
    p.add_argument("--no-lp-weights", action="store_true",
                   help="autocast casts every conv/linear weight per worker instead of bf16 working weights")
    p.add_argument("--no-worker-batching", action="store_true",
                   help="run the logical workers one after the other (per-worker graphs) instead of as one grouped "
                        "NHWC batch with per-worker BatchNorm statistics and gradients")
    p.add_argument("--ref-impl", action="store_true",
                   help="also time the reference's algorithms run as-is (BASELINE.md (a)) and report the speedup")
    p.add_argument("--phases", action="store_true", help="report per-phase device time (compute / exchange / GAR)")
    p.add_argument("--layerwise", action="store_true",
                   help="the GAR on every parameter tensor separately (reference Garfield_CC --layerwise)")
    p.add_argument("--shard-gar", action="store_true",
                   help="force the sharded, bucketed aggregation even on one GPU (with GARFIELD_LOOPBACK_EXCHANGE=1 "
                        "the exchange is emulated by side-stream copies: overlap traces)")
    p.add_argument("--num-ps", type=int, default=0,
                   help="Byzantine-server mode (parallel/byzps.py): ranks < NUM_PS are server replicas")
    p.add_argument("--fps", type=int, default=0, help="Byzantine servers tolerated by the model aggregation")
    p.add_argument("--mar", default="median", help="model aggregation rule of the Byzantine-server mode")
    p.add_argument("--ps-workers", action="store_true", help="server ranks also host logical workers")
    p.add_argument("--ps-attack", default="", help="attack of the simulated Byzantine servers (ranks < fps), "
                                                   "e.g. reverse: the Byzantine-server mode's resilience check")
    p.add_argument("--checkpoint", default="", help="save a checkpoint here after the timed steps (untimed)")
    p.add_argument("--resume", default="", help="restore this checkpoint file before the warm-up")
    p.add_argument("--data", default="fresh", choices=["fresh", "static"],
                   help="fresh: every step draws new samples from a GPU-resident synthetic uint8 dataset with random "
                        "crop + flip + normalise (data_aug.hip, one launch); static: the same batches every step")
    p.add_argument("--dataset-size", type=int, default=0,
                   help="images in the synthetic dataset (default 50000 CIFAR-shape, 2000 ImageNet-shape)")
    p.add_argument("--attack", default="",
                   help="comma-separated attacks of the Byzantine logical workers (e.g. reverse,lie): worker slot i "
                        "(global slot order) runs attack i; the JSON reports the GAR weight they received")
    p.add_argument("--no-fp32", action="store_true",
                   help="skip the companion run at the reference's precision (fp32_ms_per_step / fp32_img_per_s: "
                        "the same job with fp32 activations, weights and exchange rows on the fp32 kernels)")
    p.add_argument("--lr", type=float, default=0.01,
                   help="0.01: the reference lr (0.2) diverges from random init on the synthetic data")
    return p.parse_args()


def timed_steps(eng, batches, steps, warmup, ctx, trend=None):
    """``batches``: the k micro-batches, or a callable returning the next step's."""
    nxt = batches if callable(batches) else (lambda: batches)
    for i in range(warmup):
        loss = eng.step(nxt())
        if trend is not None and i == 0:
            trend.append(float(loss))
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    if ctx.device.type == "cuda":
        if os.environ.get("GARFIELD_TRACE_MARK"):
            torch.cuda._sleep(1000)  # marker kernel: scripts/trace_summary.py keeps what follows
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = eng.step(nxt())
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    ctx.barrier()
    if ctx.device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if ctx.is_distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=ctx.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, float(loss)


def worker_loss(eng, ctx, loss):
    """Mean of ``loss`` over the ranks that compute gradients (collective): in the Byzantine-server
    mode a pure server rank computes none and reports nothing (its 0.0 is not a loss)."""
    computes = getattr(eng, "computes", True)
    if not ctx.is_distributed:
        return loss if computes else None
    t = torch.tensor([loss if computes else 0.0, 1.0 if computes else 0.0], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t)
    return float(t[0] / t[1]) if float(t[1]) > 0 else None


def build_job(a, ctx, model, shape, num_classes, fp32: bool):
    """The engine of the benchmarked job and its batch source; fp32: the reference's precision
    (no autocast, fp32 exchange rows and weights: the grouped NHWC executor on the fp32 kernels)."""
    exchange, lp = ("fp32", False) if fp32 else (a.exchange_dtype, not a.no_lp_weights)
    xdt = torch.bfloat16 if exchange == "bf16" else torch.float32
    amp = {} if not fp32 else {"autocast_dtype": None}
    cfg = EngineConfig(gar=a.gar, f=a.f, workers_per_rank=a.workers_per_gpu, lr=a.lr, momentum=0.9,
                       weight_decay=5e-4, exchange_dtype=xdt, channels_last=a.channels_last,
                       cuda_graph=not a.no_graph, profile_phases=a.phases, lp_weights=lp,
                       worker_batching=False if a.no_worker_batching else None,
                       shard_gar=True if a.shard_gar else None, layerwise=a.layerwise,
                       byzantine={i: name for i, name in enumerate(x for x in a.attack.split(",") if x)}, **amp)
    if a.num_ps:
        from dataclasses import asdict

        from garfield_amd.parallel.byzps import ByzantinePSDataParallel, ByzPSConfig

        eng = ByzantinePSDataParallel(model, F.cross_entropy, ctx,
                                      ByzPSConfig(**asdict(cfg), num_ps=a.num_ps, fps=a.fps, mar=a.mar,
                                                  ps_workers=a.ps_workers, ps_attack=a.ps_attack))
    else:
        eng = RobustDataParallel(model, F.cross_entropy, ctx, cfg)
    if a.data == "fresh":
        from garfield_amd.data.fresh import DeviceBatches

        size = a.dataset_size or (50000 if a.dataset == "cifar10" else 2000)
        feed = DeviceBatches.synthetic(size, shape, num_classes, a.workers_per_gpu, a.batch, ctx.device,
                                       seed=1000 + ctx.rank)
        if hasattr(eng, "grouped_inputs"):   # write each batch straight into the step's input buffers
            feed.attach(eng.grouped_inputs(a.batch, shape))
        batches = feed.next
        if fp32 and feed.out.dtype != torch.float32:   # not attached: the fp32 step takes fp32 inputs
            batches = lambda: [(x.float(), y) for x, y in feed.next()]  # noqa: E731
    else:
        batches = synthetic_batches(a.workers_per_gpu, a.batch, shape, num_classes, ctx.device,
                                    seed=1000 + ctx.rank, channels_last=a.channels_last)
        if fp32:
            batches = [(x.float(), y) for x, y in batches]
    return eng, batches, xdt, amp


def main():
    a = parse()
    ctx = init_distributed()
    if a.cudnn_benchmark:
        torch.backends.cudnn.benchmark = True
    world = ctx.world_size
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the process group has {world} ranks "
                         f"(WORLD_SIZE={os.environ.get('WORLD_SIZE')}); refusing to report a mislabelled number")
    if world > 1:
        assert ctx.is_distributed and dist.get_world_size() == a.gpus, "process group not initialised"
    shape = (3, 32, 32) if a.dataset == "cifar10" else (3, 224, 224)
    num_classes = 10 if a.dataset == "cifar10" else 1000
    torch.manual_seed(1234)
    model = build_model(a.model, num_classes=num_classes)
    d = num_parameters(model)
    fp32 = a.precision == "fp32"
    eng, batches, _, _ = build_job(a, ctx, model, shape, num_classes, fp32)
    if a.resume:
        from garfield_amd.utils.checkpoint import load_engine

        load_engine(a.resume, eng)
    trend = []
    elapsed, loss = timed_steps(eng, batches, a.steps, a.warmup, ctx, trend)
    loss = worker_loss(eng, ctx, loss)
    first = worker_loss(eng, ctx, trend[0] if trend else 0.0) if trend else None
    if a.checkpoint:
        from garfield_amd.utils.checkpoint import save_engine

        save_engine(a.checkpoint, eng, meta={"bench": vars(a)}, write=ctx.rank == 0)
    checksums = None
    if world > 1:   # untimed: the replicas must be bit-identical (Byzantine-server mode: every rank, attacker included)
        mine = torch.tensor([eng.replica_checksum()], dtype=torch.float64, device=ctx.device)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        checksums = [float(c.item()) for c in allc]
    n = getattr(eng, "n_w", eng.n)   # Byzantine-server mode: only the worker slots train
    imgs = n * a.batch * a.steps
    value = imgs / elapsed
    ms = 1000.0 * elapsed / a.steps
    extra = {}
    if checksums is not None:
        extra["replica_checksums"] = checksums
        extra["replicas_identical"] = len(set(checksums)) == 1
    if a.phases:
        eng.timer.reset()
        for _ in range(3):
            eng.step(batches() if callable(batches) else batches)
        extra["phase_ms"] = {k: round(v, 3) for k, v in eng.phase_times().items()}
    if a.overhead:
        # the same job (precision, exchange, executor, data) with the average GAR
        a_avg = argparse.Namespace(**{**vars(a), "gar": "average", "attack": "", "layerwise": False})
        torch.manual_seed(1234)
        eng_avg, b_avg, _, _ = build_job(a_avg, ctx, build_model(a.model, num_classes=num_classes), shape,
                                         num_classes, fp32)
        e_avg, _ = timed_steps(eng_avg, b_avg, a.steps, a.warmup, ctx)
        ms_avg = 1000.0 * e_avg / a.steps
        extra.update({"avg_ms_per_step": round(ms_avg, 3),
                      "gar_overhead_pct_vs_average": round(100.0 * (ms - ms_avg) / ms_avg, 3)})
    if a.ref_impl and ctx.world_size == 1:
        from garfield_amd.parallel.refimpl import ReferenceStyleDP

        torch.manual_seed(1234)
        ref = ReferenceStyleDP(build_model(a.model, num_classes=num_classes), F.cross_entropy, ctx.device,
                               a.workers_per_gpu, a.f, a.lr, gar=a.gar if a.gar in ("krum", "average") else "krum",
                               autocast_dtype=None if fp32 else torch.bfloat16)
        e_ref, _ = timed_steps(ref, batches, a.steps, a.warmup, ctx)
        ms_ref = 1000.0 * e_ref / a.steps
        extra["ref_impl_ms_per_step"] = round(ms_ref, 3)
        extra["ref_impl_img_per_s"] = round(n * a.batch / (ms_ref / 1000.0), 2)
        extra["speedup_vs_ref_impl"] = round(ms_ref / ms, 3)
    if a.attack:
        byz = dict(eng.cfg.byzantine)
        w = getattr(eng, "last_weights", None)
        extra["byzantine_workers"] = {str(k): v for k, v in byz.items()}
        if w is not None and w.dim() == 1:   # the last step's selection weights, global slot order
            wc = w.float().cpu()
            extra["byzantine_weight_max"] = float(wc[list(byz)].abs().max())
            extra["honest_weight_sum"] = round(float(wc.sum() - wc[list(byz)].sum()), 6)
    if not fp32 and not a.no_fp32 and not a.num_ps:
        # the reference's precision, same job, same invocation: fp32 activations / weights / exchange rows
        # on the fp32 kernels (conv_f32.hip: split-bf16 MFMA; bn_nhwc.hip and the rest in fp32)
        torch.manual_seed(1234)
        eng32, b32, _, _ = build_job(a, ctx, build_model(a.model, num_classes=num_classes), shape, num_classes, True)
        e32, loss32 = timed_steps(eng32, b32, a.steps, a.warmup, ctx)
        ms32 = 1000.0 * e32 / a.steps
        extra.update({"fp32_ms_per_step": round(ms32, 3), "fp32_img_per_s": round(n * a.batch / (ms32 / 1000.0), 2),
                      "fp32_final_loss": round(loss32, 4), "fp32_worker_batching": eng32._gexec is not None})
    if ctx.rank == 0:
        default = (a.model, a.gar, a.f, a.dataset) == ("resnet50", "krum", 2, "cifar10")
        gar_name = {"krum": "Multi-Krum"}.get(a.gar, a.gar)
        out = {
            "metric": "img/sec ResNet-50 f=2 Multi-Krum" if default else f"img/sec {a.model} f={a.f} {gar_name}",
            "value": round(value, 2),
            "unit": "img/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": a.precision,
            "data": f"synthetic (random {'CIFAR-10' if a.dataset == 'cifar10' else 'ImageNet'}-shape images, "
                    + ("fresh samples every step from a GPU-resident uint8 dataset with random crop + flip + "
                       "normalise, " if a.data == "fresh" else "the same batches every step, ")
                    + "random-init weights)",
            "config": {
                "model": f"{a.model} (torchvision architecture, {num_classes} classes, {d} params)",
                "global_batch": n * a.batch,
                "seq_len": None,
                "image_shape": list(shape),
                "parallelism": f"dp{world} (robust DP, {a.workers_per_gpu} logical workers/GPU, n={n})"
                               + (f", {a.num_ps} Byzantine-resilient server replicas (fps={a.fps}, mar={a.mar}"
                                  f"{', servers host workers' if a.ps_workers else ''}"
                                  f"{', server attack ' + a.ps_attack if a.ps_attack else ''})" if a.num_ps else ""),
                "process_group": {"backend": ctx.backend,
                                  "world_size": dist.get_world_size() if ctx.is_distributed else 1},
                "gar": a.gar + (" (layer-wise: per parameter tensor)" if a.layerwise else ""),
                "f": a.f,
                "batch_per_worker": a.batch,
                "exchange_dtype": a.exchange_dtype,
                "hip_graphs": bool(getattr(eng, "_graph", None) or getattr(eng, "_ggraph", None)),
                "worker_batching": eng._gexec is not None,
                "lp_weights": eng._shadow is not None,
                "optimizer": f"SGD lr={a.lr} momentum=0.9 wd=5e-4 (fused into the GAR combine kernel)",
            },
            # mean over the gradient-computing ranks (Byzantine-server mode: servers without workers excluded)
            "final_loss": round(loss, 4) if loss is not None else None,
            "first_loss": round(first, 4) if first is not None else None,   # loss of the first (warm-up) step
            **extra,
        }
        print(json.dumps(out), flush=True)
    shutdown(ctx)


if __name__ == "__main__":
    main()
