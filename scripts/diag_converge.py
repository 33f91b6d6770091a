"""Loss curves of the headline path (grouped bf16, HIP graph) vs the per-worker fp32
engine on learnable synthetic data: ResNet-18, 8 workers, Krum f=2, one reverse
attacker; a sweep of learning rates (VERDICT r1 #4 diagnostics)."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402


def run(grouped, lr, steps, model="resnet18", batch=32, wd=5e-4, momentum=0.9):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    kw = dict(gar="krum", f=2, workers_per_rank=8, byzantine={7: "reverse"}, lr=lr, weight_decay=wd, momentum=momentum)
    if grouped:
        cfg = EngineConfig(cuda_graph=True, **kw)
    else:
        cfg = EngineConfig(autocast_dtype=None, exchange_dtype=torch.float32, worker_batching=False,
                           lp_weights=False, **kw)
    eng = RobustDataParallel(build_model(model), F.cross_entropy, DistContext(device=dev), cfg)
    pool = [synthetic_batches(8, batch, (3, 32, 32), 10, dev, seed=1000 + i) for i in range(8)]
    losses = [float(eng.step(pool[i % 8])) for i in range(steps)]
    return losses


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 150
    model = sys.argv[2] if len(sys.argv) > 2 else "resnet18"
    lrs = [float(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else (0.002, 0.005, 0.01, 0.02)
    for lr in lrs:
        for grouped in (True, False):
            ls = run(grouped, lr, steps, model=model)
            print(json.dumps({"model": model, "lr": lr, "grouped_bf16": grouped, "first": round(ls[0], 4),
                              "curve": [round(sum(ls[i:i + 10]) / 10, 3) for i in range(0, steps, 10)],
                              "last10": round(sum(ls[-10:]) / 10, 4)}), flush=True)
