"""Micro-benchmark of the halo-staged 3x3 weight gradient (k_wgrad3x3) on the grouped ResNet-18 CIFAR
step's 3x3 / stride-1 layers (8 workers x 250 images): device time per call (HIP graph of 20 calls) per
kernel form (``_set_kernel_variant("wgrad3x3", v)``: 0 = 2 co x 2 ci fragments per wave, 1 = 4 co x 1
ci) and bitwise equality of the forms."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

G, N = 8, 2000
SHAPES = [("l1 64", 32, 64), ("l2 128", 16, 128), ("l3 256", 8, 256), ("l4 512", 4, 512)]


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (3 * iters) * 1e6


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    variants = [0]
    for name, H, C in SHAPES:
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        row = f"{name:8s} px/worker={N * H * H // G:6d}:"
        ref = None
        for S in (1, 4):
            for v in variants:
                shape = (G, C, 9 * C) if S == 1 else (S, G, C, 9 * C)
                out = torch.empty(shape, dtype=torch.bfloat16 if S == 1 else torch.float32, device=dev)
                t = bench(lambda: C_.gpu_iwgrad(x, dy, 3, 3, 1, 1, 1, 1, 1, 1, G, out, S))
                if ref is None or ref.shape != out.shape:
                    ref = out.clone()
                elif not torch.equal(out, ref):
                    row += " MISMATCH"
                row += f" S{S}v{v} {t:7.1f}"
        print(row, flush=True)


if __name__ == "__main__":
    main()
