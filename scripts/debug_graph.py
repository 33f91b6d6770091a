"""Diagnose graph-vs-eager differences of the robust engine on one GPU."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402

model_name = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 250
k = 8
amp = None if (len(sys.argv) > 3 and sys.argv[3] == "fp32") else torch.bfloat16
dev = torch.device("cuda", 0)
for graph in (False, True):
    torch.manual_seed(1234)
    eng = RobustDataParallel(build_model(model_name), F.cross_entropy, DistContext(device=dev),
                             EngineConfig(gar="krum", f=2, workers_per_rank=k, lr=0.01, cuda_graph=graph,
                                         autocast_dtype=amp))
    b = synthetic_batches(k, batch, (3, 32, 32), 10, dev, seed=1000)
    for s in range(5):
        loss = eng.step(b)
        torch.cuda.synchronize()
        rows_nan = (~torch.isfinite(eng.G.float())).sum(1).tolist()
        per = eng._static_loss.tolist() if (graph and eng._graph is not None) else None
        print(f"graph={graph} step={s} loss={float(loss):.4f} per_worker={per} nan_rows={rows_nan} "
              f"w={eng.last_weights.tolist() if eng.last_weights is not None else None} "
              f"pnan={bool(torch.isnan(eng.flat_model()).any())}", flush=True)
