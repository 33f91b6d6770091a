"""Diagnostic: grouped engine, eager vs HIP graph, finiteness of every step."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402

cuda = torch.device("cuda")
for graph in (False, True):
    torch.manual_seed(0)
    cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, cuda_graph=graph, byzantine={5: "reverse"}, lr=1e-3)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=cuda), cfg)
    b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda)
    for s in range(4):
        loss = float(eng.step(b))
        torch.cuda.synchronize()
        rows = eng.X[:, 0, : eng.d].float()
        fin_rows = torch.isfinite(rows).all(1).tolist()
        print(f"graph={graph} step={s} loss={loss:.4f} params_finite={bool(torch.isfinite(eng.flat.data).all())} "
              f"shadow_finite={bool(torch.isfinite(eng._shadow).all())} rows_finite={fin_rows} "
              f"w={[round(v, 3) for v in eng.last_weights.tolist()]}", flush=True)
        if not fin_rows[0]:
            bad = [(n, tuple(p.shape)) for n, p, v in zip([n for n, _ in eng.model.named_parameters()],
                                                          eng.flat.params, eng.flat.views(eng.X[0, 0]))
                   if not torch.isfinite(v).all()]
            print("non-finite params of row 0:", bad[:10], flush=True)
