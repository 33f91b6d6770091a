"""Diagnose the fp32 grouped step's gradient rows: ours vs fp32 GPU autograd vs fp64 CPU autograd,
per parameter tensor (worst first)."""
import sys

import torch
import torch.nn.functional as F

from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


name = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
B = int(sys.argv[3]) if len(sys.argv) > 3 else 4
dev = torch.device("cuda", 0)
torch.manual_seed(0)
ref = build_model(name, 10).to(dev)
eng = RobustDataParallel(build_model(name, 10), F.cross_entropy, DistContext(device=dev),
                         EngineConfig(gar="average", f=0, workers_per_rank=k, exchange_dtype=torch.float32,
                                      autocast_dtype=None, lp_weights=False, lr=0.0, momentum=0.0,
                                      weight_decay=0.0, cuda_graph=False, worker_batching=True))
with torch.no_grad():
    for p, v in zip(ref.parameters(), eng.flat.params):
        p.copy_(v)
ref64 = build_model(name, 10).double()
ref64.load_state_dict({kk: v.double().cpu() for kk, v in ref.state_dict().items()})
b = synthetic_batches(k, B, (3, 32, 32), 10, dev)
eng.step(b)
torch.cuda.synchronize()
names = [n for n, _ in ref.named_parameters()]
for j, (x, y) in enumerate(b):
    ref.zero_grad()
    ref64.zero_grad()
    F.cross_entropy(ref(x.float().contiguous()), y).backward()
    F.cross_entropy(ref64(x.double().cpu()), y.cpu()).backward()
    ours = [v for v in eng.flat.views(eng.X[j, 0])]
    g32 = [p.grad for p in ref.parameters()]
    g64 = [p.grad for p in ref64.parameters()]
    cat = lambda L: torch.cat([t.reshape(-1).double().cpu() for t in L])
    print(f"worker {j}: ours vs fp64 {rel(cat(ours), cat(g64)):.3e}  fp32-autograd vs fp64 {rel(cat(g32), cat(g64)):.3e}"
          f"  ours vs fp32 {rel(cat(ours), cat(g32)):.3e}")
    rows = sorted(((rel(o, r), rel(a, r), n) for o, a, r, n in zip(ours, g32, g64, names)), reverse=True)
    for e1, e2, n in rows[:6]:
        print(f"   {n:40s} ours {e1:.3e}   fp32 {e2:.3e}")

# Conditioning: how far do the fp64 gradients move under a 1e-7 relative perturbation of the
# weights (below fp32 rounding)? ReLU units whose pre-activation is within rounding of zero flip.
base = {kk: v.clone() for kk, v in ref64.state_dict().items()}
for j, (x, y) in enumerate(b):
    xs = x.double().cpu()
    ref64.load_state_dict(base)
    ref64.zero_grad()
    F.cross_entropy(ref64(xs), y.cpu()).backward()
    g0 = torch.cat([p.grad.reshape(-1).clone() for p in ref64.parameters()])
    moves = []
    for t in range(3):
        gen = torch.Generator().manual_seed(100 + t)
        ref64.load_state_dict({kk: (v * (1 + 1e-7 * torch.randn(v.shape, generator=gen, dtype=v.dtype))
                                    if v.is_floating_point() else v) for kk, v in base.items()})
        ref64.zero_grad()
        F.cross_entropy(ref64(xs), y.cpu()).backward()
        moves.append(rel(torch.cat([p.grad.reshape(-1) for p in ref64.parameters()]), g0))
    print(f"worker {j}: fp64 gradient moves under 1e-7 weight noise: " + " ".join(f"{m:.2e}" for m in moves))
