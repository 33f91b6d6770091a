"""Debug: where the halo 3x3 weight gradient leaves non-finite / wrong entries."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd import _native  # noqa: E402


def run(G, B, C, Co, H, S):
    C_ = _native.native()
    cuda = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(G * B, C, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(G * B, Co, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    K = 9 * C
    ref = torch.stack([torch.nn.grad.conv2d_weight(x[g * B:(g + 1) * B].float(), (Co, C, 3, 3),
                                                   dy[g * B:(g + 1) * B].float(), 1, 1).permute(0, 2, 3, 1)
                       .reshape(Co, K) for g in range(G)])
    part = torch.full((S, G, Co, K), float("nan"), device=cuda)
    C_.gpu_iwgrad(x, dy, 3, 3, 1, 1, 1, 1, 1, 1, G, part, S)
    torch.cuda.synchronize()
    out = part.sum(0).view(G, Co, 9, C)
    r = ref.view(G, Co, 9, C)
    bad = ~torch.isfinite(out) | ((out - r).abs() > 0.05 * r.abs().amax().clamp_min(1e-3))
    print(f"G{G} B{B} C{C} Co{Co} H{H} S{S}: bad {int(bad.sum())} of {bad.numel()}", flush=True)
    if bad.any():
        idx = bad.nonzero()
        for name, col in (("g", 0), ("co", 1), ("tap", 2), ("ci", 3)):
            vals = torch.unique(idx[:, col]).tolist()
            print(f"   {name}: {len(vals)} distinct, first {vals[:24]}", flush=True)
        nonfin = (~torch.isfinite(out)).sum().item()
        print(f"   nonfinite {nonfin}", flush=True)


if __name__ == "__main__":
    for cfg in [(1, 8, 512, 512, 4, 1), (64, 1, 64, 64, 4, 1), (32, 2, 128, 128, 4, 1), (8, 8, 256, 256, 4, 1),
                (16, 8, 256, 256, 4, 1), (32, 8, 256, 256, 4, 1), (256, 1, 64, 64, 4, 1), (512, 1, 64, 64, 4, 1),
                (512, 1, 64, 64, 8, 1), (512, 1, 64, 64, 16, 1), (8, 8, 512, 512, 4, 1)]:
        run(*cfg)
