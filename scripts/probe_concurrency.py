"""Probe: how much do a layer's data-gradient GEMM (gemm_nt) and its per-worker 1x1 weight gradient
(k_iwgrad_1x1_wide) gain from running concurrently? Both captured 30 times in a HIP graph, either in
sequence on one stream or as two graph branches (fork / join on two streams). ResNet-50 CIFAR layer3 /
layer4 1x1 shapes, 8 workers x 250 images."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

G, N = 8, 2000
SHAPES = [("l4 conv3 512>2048", 1, 512, 2048), ("l4 conv1 2048>512", 1, 2048, 512), ("l3 conv3 256>1024", 2, 256, 1024),
          ("l3 conv1 1024>256", 2, 1024, 256)]


def timed_graph(body, iters=30):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            body()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (5 * iters) * 1e6


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    side = torch.cuda.Stream()
    for name, H, C, Co in SHAPES:
        x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(N, Co, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(C, Co, device=dev) * 0.05).to(torch.bfloat16)      # Wᵀ [C, Co]
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, Co)
        dx = torch.empty(dy2.shape[0], C, device=dev, dtype=torch.bfloat16)
        out = torch.empty(G, Co, C, dtype=torch.bfloat16, device=dev)
        cfg = C_.gemm_nt_pick(dy2.shape[0], C, Co, 0)

        def dgrad():
            C_.gpu_gemm_nt(dy2, wt, dx, None, None, 0, cfg)

        def wgrad():
            C_.gpu_iwgrad(x, dy, 1, 1, 1, 1, 0, 0, 1, 1, G, out, 1)

        def both_seq():
            dgrad()
            wgrad()

        def both_par():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            dgrad()
            with torch.cuda.stream(side):
                wgrad()
            cur.wait_stream(side)

        td, tw = timed_graph(dgrad), timed_graph(wgrad)
        ts, tp = timed_graph(both_seq), timed_graph(both_par)
        print(f"{name:20s} dgrad {td:6.1f} wgrad {tw:6.1f} | sequence {ts:6.1f} branches {tp:6.1f} "
              f"(gain {100 * (ts - tp) / ts:5.1f}%)", flush=True)


if __name__ == "__main__":
    main()
