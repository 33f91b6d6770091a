"""Diagnostic: per-parameter relative error of the engine's per-worker gradient
rows (grouped and per-worker bf16 paths) against fp32 per-worker autograd."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def main(name="resnet18", k=4, B=16):
    cuda = torch.device("cuda")
    names = [n for n, _ in build_model(name, 10).named_parameters()]
    res = {}
    for wb in (False, True):
        torch.manual_seed(0)
        ref = build_model(name, 10).to(cuda)
        eng = RobustDataParallel(build_model(name, 10), F.cross_entropy, DistContext(device=cuda),
                                 EngineConfig(gar="average", f=0, workers_per_rank=k, exchange_dtype=torch.float32,
                                              lr=0.0, momentum=0.0, weight_decay=0.0, cuda_graph=False,
                                              worker_batching=wb))
        with torch.no_grad():
            for p, v in zip(ref.parameters(), eng.flat.params):
                p.copy_(v)
        b = synthetic_batches(k, B, (3, 32, 32), 10, cuda)
        eng.step(b)
        torch.cuda.synchronize()
        ref.train()
        x, y = b[0]
        ref.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        errs = [rel(v, p.grad) for v, p in zip(eng.flat.views(eng.X[0, 0]), ref.parameters())]
        res[wb] = errs
    for i, n in enumerate(names):
        print(f"{n:40s} per-worker {res[False][i]:.4f}  grouped {res[True][i]:.4f}")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["resnet18"]))
