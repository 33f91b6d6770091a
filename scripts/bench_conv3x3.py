"""Micro-benchmark: 3x3 / stride-1 convolutions of the grouped CIFAR steps (8 workers x 250 images) on
the implicit-GEMM kernel (iconv_nhwc.hip, pm 12 / 14, data gradient with the weight read transposed)
vs the halo-staged kernel (conv3x3_nhwc.hip, pm 22 / 24, data gradient on the flipped weight), plus
the per-worker weight gradient of the same shapes. Device time per call over a HIP graph of 20 calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

N = int(os.environ.get("N", 2000))
G = 8
# (name, H, C, Cout)
SHAPES = [("r18 l1 32x32x64", 32, 64, 64), ("r18 l2 16x16x128", 16, 128, 128), ("r18 l3 8x8x256", 8, 256, 256),
          ("r18 l4 4x4x512", 4, 512, 512), ("r50 l1 8x8x64", 8, 64, 64), ("r50 l2 4x4x128", 4, 128, 128),
          ("r50 l3 2x2x256", 2, 256, 256)]


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
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    for name, H, C, Co in SHAPES:
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.empty(N, Co, H, H, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        dy = torch.randn(N, Co, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        wd = torch.empty((C, Co, 3, 3), dtype=torch.bfloat16, device=dev).contiguous(memory_format=torch.channels_last)
        C_.gpu_transpose_multi([w], [wd])
        flop = 2.0 * N * H * H * Co * 9 * C
        row = f"{name:18s} {flop / 1e9:6.1f} GFLOP:"
        pick = C_.conv3x3_pick(N, H, H, C, Co)
        for pm in (12, 14):
            t = bench(lambda: C_.gpu_iconv(x, w, 3, 3, 1, 1, 1, 1, 1, 1, y, None, pm))
            row += f" fwd pm{pm} {t:7.1f}us {flop / t / 1e6:5.0f}TF"
        if pick:
            ref = torch.empty_like(y)
            C_.gpu_iconv(x, w, 3, 3, 1, 1, 1, 1, 1, 1, ref, None, 14)
            for pm in (22, 24):
                if pm == 24 and pick != 4:
                    continue
                t = bench(lambda: C_.gpu_iconv(x, w, 3, 3, 1, 1, 1, 1, 1, 1, y, None, pm))
                err = ((y.float() - ref.float()).norm() / ref.float().norm()).item()
                row += f" | halo pm{pm} {t:7.1f}us {flop / t / 1e6:5.0f}TF (err {err:.1e})"
        print(row, flush=True)
        row = f"{'':18s} dgrad:"
        t = bench(lambda: C_.gpu_iconv(dy, w, 3, 3, 1, 1, 1, 1, 1, 1, dx, None, 14, True))
        row += f" tw pm14 {t:7.1f}us {flop / t / 1e6:5.0f}TF"
        if C_.conv3x3_pick(N, H, H, Co, C):
            t = bench(lambda: C_.gpu_iconv(dy, wd, 3, 3, 1, 1, 1, 1, 1, 1, dx, None, 0))
            row += f" | halo flipped {t:7.1f}us {flop / t / 1e6:5.0f}TF"
        rows = N // G * H * H
        for S in (1, 4, 16, 64):
            part = torch.empty(S, G, Co, 9 * C, device=dev)
            t = bench(lambda: C_.gpu_iwgrad(x, dy, 3, 3, 1, 1, 1, 1, 1, 1, G, part, S))
            row += f" | wgrad S{S} {t:7.1f}us {flop / t / 1e6:5.0f}TF"
        print(row, f"(rows/worker {rows})", flush=True)
        del x, y, dy, dx


if __name__ == "__main__":
    main()
