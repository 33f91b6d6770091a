"""Micro-benchmark of the 1x1 weight-gradient kernel (k_iwgrad_1x1_wide) on the grouped ResNet-50 CIFAR
step's 1x1 layers with C, Cout % 128 (8 workers x 250 images): device time per call (HIP graph of 50
calls) at 1 and 2 pixel splits. Round 6 used it with a since-removed variant switch (bit 0: ring depth 2,
bit 1: LDS epilogue; the variants columns of profiles/r6/iwgrad_wide/micro_variants.txt); the depth-2 ring
was kept for splits of at most four 64-pixel stages."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

G, N = 8, 2000
SHAPES = [("l2 128>512", 4, 128, 512), ("l2 512>128", 4, 512, 128), ("l2 256>512", 4, 256, 512),
          ("l3 256>1024", 2, 256, 1024), ("l3 1024>256", 2, 1024, 256), ("l3 512>1024", 2, 512, 1024),
          ("l4 512>2048", 1, 512, 2048), ("l4 2048>512", 1, 2048, 512), ("l4 1024>2048", 1, 1024, 2048)]


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
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (3 * iters) * 1e6


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    tot = [0.0] * 4
    for name, H, C, Co in SHAPES:
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, Co, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        row = f"{name:14s} px/worker={N * H * H // G:5d}:"
        ref = None
        for S in (1, 2):
            for v in range(1):
                if S == 1:
                    out = torch.empty(G, Co, C, dtype=torch.bfloat16, device=dev)
                else:
                    out = torch.empty(S, G, Co, C, dtype=torch.float32, device=dev)
                t = bench(lambda: C_.gpu_iwgrad(x, dy, 1, 1, 1, 1, 0, 0, 1, 1, G, out, S))
                if S == 1:
                    tot[v] += t
                    if v == 0:
                        ref = out.clone()
                    elif not torch.equal(out, ref):
                        row += " MISMATCH"
                row += f" S{S}v{v} {t:6.1f}"
        print(row, flush=True)
    print("sum S=1 (us):", round(tot[0], 1))


if __name__ == "__main__":
    main()
