"""One fp32 convolution shape of the ResNet-50 CIFAR step (256 ch 3x3 at 4x4 px, 2000 images), forward
+ data gradient (pm 15) and the per-worker weight gradient, launched a few times: the target of the
rocprofv3 --pmc passes in scripts/gpu_pmc_f32.sh."""
import torch

from garfield_amd import _native

C = _native.native()
dev = torch.device("cuda", 0)
N, G, cin, cout, H, k = 2000, 8, 256, 256, 4, 3
x = torch.randn(N, cin, H, H, device=dev).contiguous(memory_format=torch.channels_last)
w = (torch.randn(cout, cin, k, k, device=dev) / 48).contiguous(memory_format=torch.channels_last)
K = k * k * cin
w3 = torch.empty((3, cout, K), dtype=torch.bfloat16, device=dev)
wt3 = torch.empty((3, cin, k * k * cout), dtype=torch.bfloat16, device=dev)
C.gpu_wsplit_multi([(w, w3, wt3, cout, k * k, cin, 0)])
y = torch.empty(N, cout, H, H, device=dev).contiguous(memory_format=torch.channels_last)
dx = torch.empty_like(x)
part = torch.empty((2, G, cout, K), device=dev)
for _ in range(3):
    C.gpu_conv_f32(x, w3, k, k, 1, 1, 1, 1, 1, 1, False, y, None, 15, 1)
    C.gpu_conv_f32(y, wt3, k, k, 1, 1, 1, 1, 1, 1, True, dx, None, 15, 1)
    C.gpu_wgrad_f32(x, y, k, k, 1, 1, 1, 1, 1, 1, G, part, 2)
torch.cuda.synchronize()
