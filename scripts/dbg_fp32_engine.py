import torch, torch.nn.functional as F
from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches
dev = torch.device("cuda")
rows = []
for wb in (False, True):
    torch.manual_seed(0)
    cfg = EngineConfig(gar="average", f=0, workers_per_rank=4, lr=0.05, momentum=0.9, weight_decay=5e-4,
                       autocast_dtype=None, lp_weights=False, worker_batching=wb, cuda_graph=False,
                       exchange_dtype=torch.float32)
    eng = RobustDataParallel(build_model("resnet18"), F.cross_entropy, DistContext(device=dev), cfg)
    print("wb", wb, "gexec", type(eng._gexec).__name__, "X", tuple(eng.X.shape), eng.X.dtype)
    b = synthetic_batches(4, 8, (3, 32, 32), 10, dev, seed=40)
    loss = eng.step(b)
    torch.cuda.synchronize()
    print("loss", float(loss))
    rows.append(eng.G[:, : eng.d].float().clone())
d = rows[0].shape[1]
for j in range(rows[0].shape[0]):
    a, b = rows[0][j], rows[1][j]
    print(j, "rel", ((a - b).norm() / a.norm()).item(), a.norm().item(), b.norm().item())
names = [n for n, _ in eng.model.named_parameters()]
for n, p, off, num in zip(names, eng.work_params, eng.flat.offsets, eng.flat.numels):
    a, b = rows[0][0, off:off + num], rows[1][0, off:off + num]
    r = ((a - b).norm() / a.norm().clamp_min(1e-30)).item()
    if r > 1e-3:
        print(n, tuple(p.shape), p.is_contiguous(), p.is_contiguous(memory_format=torch.channels_last), "rel", r)
