"""Census of the gemm_nt.hip calls of one grouped step: every (M, N, K, add, stats) problem the
step issues, how often, the configuration the step's tuner chose, and every valid configuration
timed on the same operands (20 back-to-back calls each, after a warm call).

    python scripts/gemm_census.py [--model resnet50] [--dataset cifar10] > census.txt

Runs the bench configuration's engine eagerly (no graph) for two steps, recording the calls of the
second one, then times the recorded problems on scratch outputs."""
import argparse
import collections

import torch
import torch.nn.functional as F

from garfield_amd import _native
from garfield_amd.models import build_model
from garfield_amd.ops import grouped
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--dataset", default="cifar10", choices=["cifar10", "imagenet"])
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=250)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shape = (3, 224, 224) if a.dataset == "imagenet" else (3, 32, 32)
    ncls = 1000 if a.dataset == "imagenet" else 10
    eng = RobustDataParallel(build_model(a.model, ncls), F.cross_entropy, DistContext(device=dev),
                             EngineConfig(gar="krum", f=2, workers_per_rank=a.workers, cuda_graph=False))
    b = synthetic_batches(a.workers, a.batch, shape, ncls, dev)
    eng.step(b)
    torch.cuda.synchronize()
    C = _native.native()
    real = C.gpu_gemm_nt
    calls = []

    class Rec:
        def __getattr__(self, k):
            return getattr(C, k)

        @staticmethod
        def gpu_gemm_nt(A, B, out, add, stats, rg, cfg, **kw):
            calls.append((tuple(A.shape), tuple(B.shape), add is not None, stats is not None, rg, cfg,
                          (A, B, out, add, stats, kw)))
            return real(A, B, out, add, stats, rg, cfg, **kw)

    orig = _native.native
    _native.native = lambda: Rec()
    try:
        eng.step(b)
        torch.cuda.synchronize()
    finally:
        _native.native = orig

    def timed(fn, reps=20):
        fn()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            fn()
        t1.record()
        t1.synchronize()
        return t0.elapsed_time(t1) * 1000.0 / reps   # us

    groups = collections.OrderedDict()
    for (sa, sb, add, st, rg, cfg, ops) in calls:
        key = (sa[0], sb[0], sa[1], add, st, rg)
        if key not in groups:
            groups[key] = [0, cfg, ops]
        groups[key][0] += 1
    print(f"{'M':>8} {'N':>6} {'K':>6} add st  calls  cfg  us(cfg)  best  us(best)  GFLOP  TF(cfg)")
    tot_cfg = tot_best = 0.0
    for (M, N, K, add, st, rg), (n, cfg, (A, B, out, addt, stats, kw)) in groups.items():
        scratch = torch.empty_like(out)
        addc = addt.clone() if addt is not None else None

        def run(c):
            stc = (torch.empty(C.gemm_nt_stats_geometry(c, M, N, K, rg)[2], dtype=torch.float32, device=dev)
                   if stats is not None else None)
            return lambda: real(A, B, addc if addc is not None else scratch, addc, stc, rg, c, **kw)

        t_cfg = timed(run(cfg))
        best, t_best = cfg, t_cfg
        for c in range(C.gemm_nt_num_cfg()):
            if c == cfg or not C.gemm_nt_valid(c, N, K) or (rg and C.gemm_nt_stats_rows(c) > rg):
                continue
            if kw.get("pro_groups") and not C.gemm_nt_pro_ok(c, K, M // kw["pro_groups"], kw["pro_groups"]):
                continue
            t = timed(run(c))
            if t < t_best:
                best, t_best = c, t
        gf = 2.0 * M * N * K / 1e9
        tot_cfg += n * t_cfg
        tot_best += n * t_best
        print(f"{M:>8} {N:>6} {K:>6} {int(add):>3} {int(st):>2} {n:>6} {cfg:>4} {t_cfg:>8.1f} {best:>5} {t_best:>9.1f} "
              f"{gf:>6.2f} {gf / t_cfg * 1000.0:>8.1f}")
    print(f"total per step: {tot_cfg:.1f} us with the step's choices, {tot_best:.1f} us with the best valid ones")
    _ = grouped


if __name__ == "__main__":
    main()
