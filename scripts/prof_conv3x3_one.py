"""One 3x3 convolution shape, launched a few times, for rocprofv3 --pmc passes (SHAPE = l1 | l2 | l3 | l4,
PM = gpu_iconv pm, WG = 1 runs the halo weight gradient instead)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402

SHAPES = {"l1": (32, 64, 64), "l2": (16, 128, 128), "l3": (8, 256, 256), "l4": (4, 512, 512)}


def main():
    C_ = _native.native()
    dev = torch.device("cuda")
    H, C, Co = SHAPES[os.environ.get("SHAPE", "l1")]
    N = int(os.environ.get("N", 2000))
    pm = int(os.environ.get("PM", 24))
    x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device=dev) / (9 * C) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.empty(N, Co, H, H, dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    if os.environ.get("WG", "0") == "1":
        S = int(os.environ.get("S", 16))
        part = torch.empty(S, 8, Co, 9 * C, device=dev)
        for _ in range(5):
            C_.gpu_iwgrad(x, y, 3, 3, 1, 1, 1, 1, 1, 1, 8, part, S)
    else:
        for _ in range(5):
            C_.gpu_iconv(x, w, 3, 3, 1, 1, 1, 1, 1, 1, y, None, pm)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
