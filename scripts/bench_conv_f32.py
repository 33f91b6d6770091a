"""Micro-benchmark: the fp32 (split-bf16) convolution kernels of conv_f32.hip on the grouped
ResNet-50 CIFAR step's shapes (8 workers x 250 images): forward / data gradient per kernel variant
(pm 11 / 12 / 13 / 14 / 15 = LDS-staged PM 1 / 2 (3-deep ring) / 2 (2-deep: two workgroups per CU) / 4 /
4 with a 3-deep ring; ks = split-K) and the
per-worker weight gradient, in ms and TFLOP/s of fp32 work."""
import sys

import torch

from garfield_amd import _native

C = _native.native()
dev = torch.device("cuda", 0)
N, G = 2000, 8
SHAPES = [  # Cin, Cout, H (input), k, s
    (64, 64, 8, 3, 1), (128, 128, 4, 3, 1), (256, 256, 2, 3, 1), (512, 512, 1, 3, 1), (256, 1024, 2, 1, 1),
    (1024, 256, 2, 1, 1), (64, 256, 8, 1, 1), (512, 2048, 1, 1, 1), (128, 128, 8, 3, 2), (256, 512, 8, 1, 2)]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


variants = [(0, 0), (13, 1), (13, 2), (13, 4), (15, 2), (15, 4)]
for cin, cout, H, k, s in SHAPES:
    p = k // 2
    Ho = (H + 2 * p - k) // s + 1
    x = torch.randn(N, cin, H, H, device=dev).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5).contiguous(memory_format=torch.channels_last)
    K = k * k * cin
    w3 = torch.empty((3, cout, K), dtype=torch.bfloat16, device=dev)
    wt3 = torch.empty((3, cin, k * k * cout), dtype=torch.bfloat16, device=dev)
    C.gpu_wsplit_multi([(w, w3, wt3, cout, k * k, cin, 0)])
    y = torch.empty(N, cout, Ho, Ho, device=dev).contiguous(memory_format=torch.channels_last)
    dx = torch.empty_like(x)
    fl = 2.0 * N * Ho * Ho * cout * K / 1e12
    line = f"{cin:5d}->{cout:5d} H{H} k{k} s{s} ({fl * 1e3:.1f} GF)"
    for pm, ks in variants:
        tf = timeit(lambda: C.gpu_conv_f32(x, w3, k, k, s, s, p, p, 1, 1, False, y, None, pm, ks))
        td = timeit(lambda: C.gpu_conv_f32(y, wt3, k, k, s, s, p, p, 1, 1, True, dx, None, pm, ks))
        line += f" | pm{pm}/ks{ks} f {tf:.3f} d {td:.3f}"
    rows = N * Ho * Ho // G
    for var in ((2,) if cin % 128 == 0 and cout % 128 == 0 else (3,)):
        for S in (1, 2, 4, 8, 16):
            part = torch.empty((S, G, cout, K), device=dev)
            tw = timeit(lambda: C.gpu_wgrad_f32(x, y, k, k, s, s, p, p, 1, 1, G, part, S, var))
            line += f" | wg v{var} S{S} {tw:.3f} ({fl / tw * 1e3:.0f})"
    print(line, flush=True)
