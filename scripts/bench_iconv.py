"""Micro-benchmark: implicit-GEMM MFMA convolution (gpu_iconv) vs im2col + hipBLASLt GEMM
(plain GEMM for 1x1 stride-1) on the convolution shapes of the grouped ResNet-50 step
(8 workers x 250 CIFAR images). Each variant is timed over a HIP graph of 50 calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

N = int(os.environ.get("N", 2000))
# (name, H, C, Cout, stride, kernel)
SHAPES = [("l1 3x3 64", 8, 64, 64, 1, 3), ("l2 3x3 128", 4, 128, 128, 1, 3), ("l2 3x3/2 128", 8, 128, 128, 2, 3),
          ("l3 3x3 256", 2, 256, 256, 1, 3), ("l4 3x3 512", 1, 512, 512, 1, 3),
          ("l1 1x1 64>256", 8, 64, 256, 1, 1), ("l1 1x1 256>64", 8, 256, 64, 1, 1),
          ("l2 1x1 128>512", 4, 128, 512, 1, 1), ("l2 1x1 512>128", 4, 512, 128, 1, 1),
          ("l3 1x1 256>1024", 2, 256, 1024, 1, 1), ("l3 1x1 1024>256", 2, 1024, 256, 1, 1),
          ("l4 1x1 512>2048", 1, 512, 2048, 1, 1), ("l4 1x1 2048>512", 1, 2048, 512, 1, 1)]


def bench(fn, iters=50):
    """Mean microseconds per call over a HIP graph of ``iters`` calls (no Python launch overhead)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    for name, H, C, Co, s, k in SHAPES:
        p = k // 2
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(Co, C, k, k, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        Ho = (H + 2 * p - k) // s + 1
        y = torch.empty(N, Co, Ho, Ho, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        col = torch.empty(N * Ho * Ho, k * k * C, dtype=torch.bfloat16, device=dev)
        w2 = w.permute(0, 2, 3, 1).reshape(Co, -1)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
        out = torch.empty(N * Ho * Ho, Co, dtype=torch.bfloat16, device=dev)

        def ref():
            if k == 1 and s == 1:
                return torch.mm(x2, w2.t(), out=out)
            C_.gpu_im2col(x, k, k, s, s, p, p, 1, 1, col)
            return torch.mm(col, w2.t(), out=out)

        t_ref = bench(ref)
        kind = "gemm" if (k == 1 and s == 1) else "im2col+gemm"
        row = f"{name:16s} M={N * Ho * Ho:7d} K={k * k * C:5d} Cout={Co:5d}: {kind} {t_ref:7.1f} us"
        for pm in (4, 11, 12, 14):
            t = bench(lambda: C_.gpu_iconv(x, w, k, k, s, s, p, p, 1, 1, y, None, pm))
            row += f" | iconv pm={pm} {t:7.1f} us"
        print(row, flush=True)


if __name__ == "__main__":
    main()
