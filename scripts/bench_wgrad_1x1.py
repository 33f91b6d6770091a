"""Micro-benchmark: per-worker weight gradients of the grouped ResNet-50 step's
convolutions (8 workers x 250 CIFAR images): strided-batched hipBLASLt GEMM (with the
split-K variants of ``_wgrad``) vs the implicit MFMA kernel ``gpu_iwgrad`` at each
pixel-split count. Each variant is timed over a HIP graph of 50 calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

G = 8
N = int(os.environ.get("N", 2000))
# (name, H, Cin, Cout, kernel)
SHAPES = [("l1 1x1 64>256", 8, 64, 256, 1), ("l1 1x1 256>64", 8, 256, 64, 1),
          ("l2 1x1 128>512", 4, 128, 512, 1), ("l2 1x1 512>128", 4, 512, 128, 1),
          ("l2 1x1 256>512", 4, 256, 512, 1),
          ("l3 1x1 256>1024", 2, 256, 1024, 1), ("l3 1x1 1024>256", 2, 1024, 256, 1),
          ("l4 1x1 512>2048", 1, 512, 2048, 1), ("l4 1x1 2048>512", 1, 2048, 512, 1),
          ("l3 3x3 256", 2, 256, 256, 3), ("l4 3x3 512", 1, 512, 512, 3)]


def bench(fn, iters=50):
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
    for name, H, C, Co, k in SHAPES:
        p = k // 2
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, Co, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        M = N * H * H // G
        K = k * k * C
        row = f"{name:16s} rows/worker={M:6d} K={K:5d} Cout={Co:5d}:"
        if k == 1:
            x2 = x.permute(0, 2, 3, 1).reshape(G, M, C)
            d2 = dy.permute(0, 2, 3, 1).reshape(G, M, Co)
            out = torch.empty(G, Co, C, dtype=torch.bfloat16, device=dev)
            t = bench(lambda: torch.bmm(d2.transpose(1, 2), x2, out=out))
            row += f" bmm {t:6.1f} us"
            for S in (2, 4):
                if M % S:
                    continue
                xs, ds = x2.reshape(G * S, M // S, C), d2.reshape(G * S, M // S, Co)
                t = bench(lambda: torch.sum(torch.bmm(ds.transpose(1, 2), xs).view(G, S, Co, C), 1, out=out))
                row += f" | bmm S={S} {t:6.1f}"
        out = torch.empty(G, Co, K, dtype=torch.bfloat16, device=dev)
        t = bench(lambda: C_.gpu_iwgrad(x, dy, k, k, 1, 1, p, p, 1, 1, G, out, 1))
        row += f" | iwgrad {t:6.1f}"
        for S in (2, 4, 8):
            part = torch.empty(S, G, Co, K, dtype=torch.float32, device=dev)
            t = bench(lambda: torch.sum(C_.gpu_iwgrad(x, dy, k, k, 1, 1, p, p, 1, 1, G, part, S) or part, 0,
                                        out=out))
            row += f" | iwgrad S={S} {t:6.1f}"
        print(row, flush=True)


if __name__ == "__main__":
    main()
