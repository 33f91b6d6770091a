"""Micro-benchmark: per-worker weight-gradient GEMM shapes of the grouped ResNet-50
step (k = 8 workers x 250 CIFAR images): one strided-batched GEMM per layer vs a
split-K variant (batch k*S, fp32 sum over S)."""
import time

import torch

G = 8
# (Cout, K = kh*kw*Cin, rows per worker)
SHAPES = [(64, 152, 64000), (64, 576, 16000), (64, 256, 16000), (256, 64, 16000), (128, 1152, 4000),
          (512, 128, 4000), (256, 2304, 1000), (1024, 256, 1000), (512, 4608, 250), (2048, 512, 250)]


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
    tot_a = tot_b = 0.0
    for cout, K, M in SHAPES:
        dy = torch.randn(G, M, cout, device=dev, dtype=torch.bfloat16)
        col = torch.randn(G, M, K, device=dev, dtype=torch.bfloat16)
        a = bench(lambda: torch.bmm(dy.transpose(1, 2), col))
        best = (a, 1)
        for S in (2, 4, 8, 16):
            if M % S:
                continue
            dys = dy.view(G * S, M // S, cout)
            cols = col.view(G * S, M // S, K)
            t = bench(lambda: torch.bmm(dys.transpose(1, 2), cols).view(G, S, cout, K).float().sum(1))
            if t < best[0]:
                best = (t, S)
        tf = 2 * G * M * cout * K / (a * 1e-6) / 1e12
        print(f"Cout={cout:5d} K={K:5d} M={M:6d}: bmm {a:8.1f} us ({tf:6.1f} TF/s)  best split S={best[1]:2d} "
              f"{best[0]:8.1f} us", flush=True)
        tot_a += a
        tot_b += best[0]
    print(f"total: bmm {tot_a:.0f} us, best split {tot_b:.0f} us")


if __name__ == "__main__":
    main()
