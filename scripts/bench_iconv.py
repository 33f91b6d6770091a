"""Micro-benchmark: implicit-GEMM MFMA convolution (gpu_iconv) vs im2col + hipBLASLt GEMM
on the 3x3 layers of the grouped ResNet-50 step (8 workers x 250 CIFAR images)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

N = int(os.environ.get("N", 2000))
# (name, H, C, Cout, stride)
SHAPES = [("l1 3x3 64", 8, 64, 64, 1), ("l2 3x3 128", 4, 128, 128, 1), ("l2 3x3/2 128", 8, 128, 128, 2),
          ("l3 3x3 256", 2, 256, 256, 1), ("l4 3x3 512", 1, 512, 512, 1)]


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
    C_ = _native.native()
    dev = torch.device("cuda")
    for name, H, C, Co, s in SHAPES:
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, C, 3, 3, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        Ho = (H + 2 - 3) // s + 1
        y = torch.empty(N, Co, Ho, Ho, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        col = torch.empty(N * Ho * Ho, 9 * C, dtype=torch.bfloat16, device=dev)
        w2 = w.permute(0, 2, 3, 1).reshape(Co, -1)

        def ref():
            C_.gpu_im2col(x, 3, 3, s, s, 1, 1, 1, 1, col)
            return torch.mm(col, w2.t())

        t_ref = bench(ref)
        row = f"{name:14s} M={N * Ho * Ho:7d} K={9 * C:5d} Cout={Co:4d}: im2col+gemm {t_ref:7.1f} us"
        for pm in (1, 2, 4):
            t = bench(lambda: C_.gpu_iconv(x, w, 3, 3, s, s, 1, 1, 1, 1, y, None, pm))
            row += f" | iconv pm={pm} {t:7.1f} us"
        print(row, flush=True)


if __name__ == "__main__":
    main()
