"""One 1x1 GEMM shape through each gemm_nt variant (for rocprofv3 --pmc): hipBLASLt, the
K-loop kernel, the weight-stationary kernel plain and with fused BatchNorm statistics."""
import sys

import torch

from garfield_amd import _native

M, K, N = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (128000, 64, 256)))
cfgs = [int(c) for c in sys.argv[4].split(",")] if len(sys.argv) > 4 else [7, 10]
rg = M // 8
C_ = _native.native()
dev = torch.device("cuda")
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
for _ in range(3):
    torch.mm(x, w.t())
for cfg in cfgs:
    st = torch.empty(C_.gemm_nt_stats_geometry(cfg, M, N, K, rg)[2], device=dev)
    for _ in range(3):
        C_.gpu_gemm_nt(x, w, y, None, None, 0, cfg)
        C_.gpu_gemm_nt(x, w, y, None, st, rg, cfg)
torch.cuda.synchronize()
print("ok")
