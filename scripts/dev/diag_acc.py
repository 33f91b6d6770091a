"""Diagnostic: grouped vs per-worker bf16 gradient error against fp32 autograd (ResNet-50, k=4, B=16)."""
import sys
import torch

sys.path.insert(0, "tests")
import test_grouped_gpu as T  # noqa: E402

cuda = torch.device("cuda", 0)
for name in ("resnet18", "resnet50"):
    pw = T._rows_vs_fp32(cuda, name, 4, 16, False)
    gr = T._rows_vs_fp32(cuda, name, 4, 16, True)
    print(name, "per-worker", [round(x, 4) for x in pw], "grouped", [round(x, 4) for x in gr], flush=True)
