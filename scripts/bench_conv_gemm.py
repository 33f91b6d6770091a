"""Micro-benchmark: forward / dgrad GEMM shapes of the grouped ResNet-50 step
(8 workers x 250 CIFAR images = 2000 images) on hipBLASLt vs rocBLAS."""
import time

import torch

N = 2000
# (name, rows M, K, Cout, count per step)
SHAPES = [
    ("stem 7x7/2", N * 256, 152, 64, 1),
    ("l1 1x1 64->64", N * 64, 64, 64, 1), ("l1 1x1 256->64", N * 64, 256, 64, 2),
    ("l1 3x3 64", N * 64, 576, 64, 3), ("l1 1x1 64->256", N * 64, 64, 256, 4),
    ("l2 1x1 256->128", N * 64, 256, 128, 1), ("l2 3x3/2 128", N * 16, 1152, 128, 1),
    ("l2 1x1 512->128", N * 16, 512, 128, 3), ("l2 3x3 128", N * 16, 1152, 128, 3),
    ("l2 1x1 128->512", N * 16, 128, 512, 4), ("l2 ds 256->512/2", N * 16, 256, 512, 1),
    ("l3 3x3 256", N * 4, 2304, 256, 6), ("l3 1x1 1024->256", N * 4, 1024, 256, 5),
    ("l3 1x1 256->1024", N * 4, 256, 1024, 6),
    ("l4 3x3 512", N, 4608, 512, 3), ("l4 1x1 2048->512", N, 2048, 512, 2), ("l4 1x1 512->2048", N, 512, 2048, 3),
]


def bench(fn, iters=20):
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
    libs = ["cublaslt", "cublas"]
    tot = {lib: 0.0 for lib in libs}
    for name, M, K, C, cnt in SHAPES:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(C, K, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, C, device=dev, dtype=torch.bfloat16)
        row = f"{name:20s} M={M:7d} K={K:5d} N={C:5d} x{cnt}:"
        for lib in libs:
            torch.backends.cuda.preferred_blas_library(lib)
            tf = bench(lambda: torch.mm(a, w.t()))
            tb = bench(lambda: torch.mm(dy, w))
            tot[lib] += cnt * (tf + tb)
            fl = 2 * M * K * C / 1e6
            row += f"  {lib}: fwd {tf:7.1f} us ({fl / tf:5.0f} TF/s) dgrad {tb:7.1f} us ({fl / tb:5.0f} TF/s)"
        print(row, flush=True)
    print("per-step totals (fwd + dgrad):", {k: f"{v / 1000:.2f} ms" for k, v in tot.items()})


if __name__ == "__main__":
    main()
