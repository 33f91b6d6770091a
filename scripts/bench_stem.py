"""Micro-benchmark of the ResNet stem (7x7/2, 3 -> 64) at the bench shape: stem_nhwc.hip
forward / per-worker weight gradient vs the generic im2col + hipBLASLt path.

    python scripts/bench_stem.py [--n 2000] [--groups 8] [--hw 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from garfield_amd import _native  # noqa: E402
from garfield_amd.ops.grouped import _wmat  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1000, 1)   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--hw", type=int, default=32)
    ap.add_argument("--wg", type=int, nargs="*", default=[256, 512, 1024, 2048])
    a = ap.parse_args()
    C = _native.native()
    dev = torch.device("cuda", 0)
    N, G, H = a.n, a.groups, a.hw
    x = torch.randn(N, 3, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device=dev) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 6 - 7) // 2 + 1
    y = torch.empty(N, 64, Ho, Ho, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    w160 = _wmat(w, 160).contiguous()
    res = {"stem_fwd_us": timed(lambda: C.gpu_stem_fwd(x, w160, y))}
    col = torch.empty(N * Ho * Ho, 152, dtype=torch.bfloat16, device=dev)
    w152 = _wmat(w, 152).contiguous()
    res["im2col_us"] = timed(lambda: C.gpu_im2col(x, 7, 7, 2, 2, 3, 3, 1, 1, col))
    res["gemm_fwd_us"] = timed(lambda: torch.mm(col, w152.t()))
    dy = torch.randn_like(y)
    per = N // G
    for wg in a.wg:
        S = max(1, min(per, -(-wg // G)))
        part = torch.empty(S, G, 64, 147, device=dev)
        res[f"stem_wgrad_S{S}_us"] = timed(lambda: C.gpu_stem_wgrad(x, dy, G, part))
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, 64)
    res["gemm_wgrad_us"] = timed(lambda: torch.bmm(dy2.view(G, -1, 64).transpose(1, 2), col.view(G, -1, 152)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
