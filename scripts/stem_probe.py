"""The ImageNet-size stem kernels alone (for rocprofv3 --pmc): forward and weight gradient over 256 images."""
import torch

from garfield_amd import _native

C_ = _native.native()
dev = torch.device("cuda")
N, G = 256, 8
x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device=dev) / 12).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.empty(N, 64, 112, 112, dtype=torch.bfloat16, device=dev).contiguous(memory_format=torch.channels_last)
dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
part = torch.empty(N // G, G, 64, 147, device=dev)
for _ in range(3):
    C_.gpu_stem_fwd(x, w, y)
    C_.gpu_stem_wgrad(x, dy, G, part)
torch.cuda.synchronize()
print("ok")
