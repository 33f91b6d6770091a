"""Debug: which exchange-row parameters go non-finite in the graphed grouped ResNet-18 step (the
test_grouped_engine_graph_matches_eager_and_excludes_attacker configuration)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from garfield_amd.models import build_model  # noqa: E402
from garfield_amd.parallel.comm import DistContext  # noqa: E402
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches  # noqa: E402


def main():
    cuda = torch.device("cuda")
    for graph in (False, True):
        torch.manual_seed(0)
        cfg = EngineConfig(gar="krum", f=2, workers_per_rank=8, cuda_graph=graph, byzantine={5: "reverse"}, lr=1e-3)
        model = build_model("resnet18")
        eng = RobustDataParallel(model, F.cross_entropy, DistContext(device=cuda), cfg)
        b = synthetic_batches(8, 8, (3, 32, 32), 10, cuda)
        for s in range(4):
            loss = float(eng.step(b))
            torch.cuda.synchronize()
            G = eng.X.view(eng.n, eng.ld)[:, : eng.d].float()
            bad = ~torch.isfinite(G)
            names = [n for n, _ in model.named_parameters()]
            msg = []
            if bad.any():
                for name, size, off in zip(names, eng.flat.sizes, eng.flat.offsets):
                    numel = 1
                    for v in size:
                        numel *= v
                    nb = int(bad[:, off:off + numel].sum())
                    if nb:
                        msg.append(f"{name}{tuple(size)}:{nb}")
            p = eng.flat.reference_vector()
            print(f"graph={graph} step {s} loss {loss:.4f} nonfinite rows: {int(bad.any(1).sum())} params finite "
                  f"{bool(torch.isfinite(p).all())}", " ".join(msg[:12]), flush=True)


if __name__ == "__main__":
    main()
