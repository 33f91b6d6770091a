"""A/B of the weight-stationary 1x1 GEMM (gemm_nt.hip k_gemm_ws): LDS-DMA by builtin (variant 0) vs by
inline asm with counted waits (variant ws_asm=1). Every (M, N, K, epilogue) problem of the ResNet-50
CIFAR / ImageNet steps that the tuner gives a weight-stationary configuration: outputs (and statistics)
compared bit for bit between the variants, then each variant timed (HIP events, best of 3 x 10 calls).

    python scripts/ab_gemm_ws.py [--imagenet]"""
import sys

import torch

from garfield_amd import _native

C_ = _native.native()
dev = torch.device("cuda")
cifar = [(128000, 64, 64, "stats"), (128000, 256, 64, "stats"), (128000, 256, 64, "add"), (128000, 64, 64, "add"),
         (128000, 128, 256, "stats"), (128000, 256, 128, "add"), (32000, 512, 128, "stats"), (32000, 512, 128, "add"),
         (8000, 1024, 256, "plain"), (8000, 1024, 256, "add"), (128000, 64, 256, "plain")]
imagenet = [(6272000, 64, 64, "stats"), (6272000, 256, 64, "stats"), (6272000, 256, 64, "add"),
            (6272000, 256, 128, "add"), (1568000, 512, 128, "stats"), (1568000, 512, 128, "add"),
            (392000, 1024, 256, "stats"), (392000, 1024, 256, "add"), (6272000, 64, 64, "add")]
probs = cifar + (imagenet if "--imagenet" in sys.argv else [])
G = 8


def run(M, N, K, kind, cfg):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    add = torch.randn(M, N, device=dev).to(torch.bfloat16) if kind == "add" else None
    rg = M // G if kind == "stats" else 0
    out = {}
    for v in (0, 1):
        C_._set_kernel_variant("ws_asm", v)
        c = add.clone() if add is not None else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        st = torch.zeros(C_.gemm_nt_stats_geometry(cfg, M, N, K, rg)[2], device=dev) if rg else None
        C_.gpu_gemm_nt(a, b, c, c if add is not None else None, st, rg, cfg)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(10):
                C_.gpu_gemm_nt(a, b, c, c if add is not None else None, st, rg, cfg)
            t1.record()
            t1.synchronize()
            best = min(best, t0.elapsed_time(t1) / 10 * 1000)
        # one fresh call for the comparison (the timing calls accumulated into c when adding)
        c2 = add.clone() if add is not None else torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        st2 = torch.zeros_like(st) if st is not None else None
        C_.gpu_gemm_nt(a, b, c2, c2 if add is not None else None, st2, rg, cfg)
        torch.cuda.synchronize()
        out[v] = (c2, st2, best)
    C_._set_kernel_variant("ws_asm", 0)
    same = torch.equal(out[0][0], out[1][0]) and (out[0][1] is None or torch.equal(out[0][1], out[1][1]))
    byts = 2 * (M * K + N * K + M * N * (2 if kind == "add" else 1))
    return same, out[0][2], out[1][2], byts


ok = True
print(f"{'M':>8} {'N':>5} {'K':>4} {'epi':>5} {'cfg':>3}  {'v0 us':>8} {'v1 us':>8}  {'v0 TB/s':>7} {'v1 TB/s':>7}  same")
for M, N, K, kind in probs:
    for cfg in range(9, 15):
        if not C_.gemm_nt_valid(cfg, N, K):
            continue
        try:
            same, t0, t1, byts = run(M, N, K, kind, cfg)
        except RuntimeError as e:
            continue
        ok &= same
        print(f"{M:>8} {N:>5} {K:>4} {kind:>5} {cfg:>3}  {t0:8.1f} {t1:8.1f}  {byts / t0 / 1e6:7.2f} {byts / t1 / 1e6:7.2f}  {same}",
              flush=True)
print("ALL SAME" if ok else "MISMATCH")
