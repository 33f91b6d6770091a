"""Diagnostic: exchange-row differences between the small-image / stride-2 paths and flags."""
import sys
import torch

sys.path.insert(0, "tests")
import test_grouped_gpu as T  # noqa: E402
import garfield_amd.ops.grouped as grouped  # noqa: E402

cuda = torch.device("cuda", 0)
grouped.S2_FORCE = True
grouped.SC_DENSE_WGRAD = True
res = {}
for lazy in (False, True):
    for sc in (False, True):
        grouped.LAZY_RES = lazy
        grouped.SMALL_CONV = sc
        grouped._S2_CHOICE.clear()
        r = T._grouped_rows(cuda, "resnet50", 4, 16)
        e = T._rows_vs_fp32(cuda, "resnet50", 4, 16, True)
        res[(lazy, sc)] = r
        print(f"lazy={lazy} small_conv={sc} err_vs_fp32={[round(x, 4) for x in e]}", flush=True)
keys = list(res)
for i in range(len(keys)):
    for j in range(i + 1, len(keys)):
        a, b = res[keys[i]], res[keys[j]]
        print(keys[i], keys[j], [round(T.rel(b[k], a[k]), 4) for k in range(4)], flush=True)
