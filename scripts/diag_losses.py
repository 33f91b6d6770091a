"""Diagnostic: loss trajectories of the bench configuration in the engine's modes
(per-worker graphs, grouped eager, grouped graph) from the same initialisation."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402

cuda = torch.device("cuda")
B = int(os.environ.get("B", 250))
steps = int(os.environ.get("STEPS", 15))
for name, wb, graph in (("per-worker graph", False, True), ("grouped eager", True, False),
                        ("grouped graph", True, True)):
    torch.manual_seed(1234)
    cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, lr=0.01, momentum=0.9, weight_decay=5e-4,
                       cuda_graph=graph, worker_batching=wb)
    eng = RobustDataParallel(build_model("resnet50", 10), F.cross_entropy, DistContext(device=cuda), cfg)
    b = synthetic_batches(8, B, (3, 32, 32), 10, cuda, seed=1000)
    losses = [round(float(eng.step(b)), 3) for _ in range(steps)]
    print(f"{name:18s} {losses}", flush=True)
