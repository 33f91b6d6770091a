"""Micro-benchmark: the grouped ResNet-50 step's 1x1 convolution GEMMs (8 workers x 250
CIFAR images) on hipBLASLt (torch.mm) vs the implicit-GEMM MFMA kernel (gpu_iconv as a
1x1 convolution, pixel tiles PM = 1/2/4) and, when built, the dedicated 1x1 kernel
(gpu_gemm1x1).  Forward y = x·Wᵀ and data gradient dx = dy·W; prints µs and the
fraction of the 6.3 TB/s achievable HBM rate the compulsory bytes represent."""
import time

import torch

from garfield_amd import _native

N = 2000
# (name, rows M, K = Cin, Cout, count per step)
SHAPES = [
    ("l1 1x1 64->64", N * 64, 64, 64, 1), ("l1 1x1 256->64", N * 64, 256, 64, 2),
    ("l1 1x1 64->256", N * 64, 64, 256, 4),
    ("l2 1x1 256->128", N * 64, 256, 128, 1), ("l2 1x1 512->128", N * 16, 512, 128, 3),
    ("l2 1x1 128->512", N * 16, 128, 512, 4),
    ("l3 1x1 512->256", N * 16, 512, 256, 1), ("l3 1x1 1024->256", N * 4, 1024, 256, 5),
    ("l3 1x1 256->1024", N * 4, 256, 1024, 6),
    ("l4 1x1 1024->512", N * 4, 1024, 512, 1), ("l4 1x1 2048->512", N, 2048, 512, 2),
    ("l4 1x1 512->2048", N, 512, 2048, 3),
]


def bench(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    dev = torch.device("cuda")
    C_ = _native.native()
    has_g = hasattr(C_, "gpu_gemm1x1")
    tot = {}
    for name, M, K, Co, cnt in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Co, K, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(M, Co, device=dev, dtype=torch.bfloat16)
        byf = 2 * (M * K + M * Co + Co * K)
        res = {}
        yref = torch.mm(x, w.t())
        dref = torch.mm(dy, w)
        res["mm fwd"] = bench(lambda: torch.mm(x, w.t()))
        res["mm dgrad"] = bench(lambda: torch.mm(dy, w))
        x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)          # [M, K, 1, 1] channels_last
        dy4 = dy.view(M, 1, 1, Co).permute(0, 3, 1, 2)
        w4 = w.view(Co, K, 1, 1)
        y4 = torch.empty((M, Co, 1, 1), device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        dx4 = torch.empty((M, K, 1, 1), device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        for pm in (11, 12, 14):
            f = lambda: C_.gpu_iconv(x4, w4, 1, 1, 1, 1, 0, 0, 1, 1, y4, None, pm, False)
            res[f"iconv{pm - 10} fwd"] = bench(f)
            f()
            err = (y4.view(M, Co).float() - yref.float()).abs().max().item()
            assert err < 0.05 * yref.float().abs().max().item() + 1e-2, (name, pm, err)
            g = lambda: C_.gpu_iconv(dy4, w4, 1, 1, 1, 1, 0, 0, 1, 1, dx4, None, pm, True)
            res[f"iconv{pm - 10} dgrad"] = bench(g)
            g()
            err = (dx4.view(M, K).float() - dref.float()).abs().max().item()
            assert err < 0.05 * dref.float().abs().max().item() + 1e-2, (name, pm, "dgrad", err)
        if has_g:
            y2 = torch.empty((M, Co), device=dev, dtype=torch.bfloat16)
            dx2 = torch.empty((M, K), device=dev, dtype=torch.bfloat16)
            f = lambda: C_.gpu_gemm1x1(x, w, y2, None, False)
            res["g1x1 fwd"] = bench(f)
            f()
            err = (y2.float() - yref.float()).abs().max().item()
            assert err < 0.05 * yref.float().abs().max().item() + 1e-2, (name, "g1x1", err)
            g = lambda: C_.gpu_gemm1x1(dy, w, dx2, None, True)
            res["g1x1 dgrad"] = bench(g)
            g()
            err = (dx2.float() - dref.float()).abs().max().item()
            assert err < 0.05 * dref.float().abs().max().item() + 1e-2, (name, "g1x1 dgrad", err)
        floor = byf / 6.3e12 * 1e6
        print(f"{name:18s} M={M:6d} K={K:5d} N={Co:5d} x{cnt} floor {floor:5.1f}us | "
              + " ".join(f"{k} {v:6.1f}" for k, v in res.items()), flush=True)
        for k, v in res.items():
            tot[k] = tot.get(k, 0.0) + cnt * v
    print("per-step totals (us):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
