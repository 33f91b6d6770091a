import copy, torch, torch.nn.functional as F
from garfield_amd.models import build_model
from garfield_amd.parallel.comm import DistContext
from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches
dev = torch.device("cuda")
torch.manual_seed(0)
model0 = build_model("resnet18")
b = synthetic_batches(4, 8, (3, 32, 32), 10, dev, seed=40)
# independent reference: worker 0's gradient in fp32, standard layout
ref = copy.deepcopy(model0).to(dev)
ref.train()
loss = F.cross_entropy(ref(b[0][0].float()), b[0][1])
w = dict(ref.named_parameters())["layer3.1.conv1.weight"]
gref = torch.autograd.grad(loss, [w])[0]
for wb in (False, True):
    torch.manual_seed(0)
    cfg = EngineConfig(gar="average", f=0, workers_per_rank=4, lr=0.05, momentum=0.9, weight_decay=5e-4,
                       autocast_dtype=None, lp_weights=False, worker_batching=wb, cuda_graph=False,
                       exchange_dtype=torch.float32)
    eng = RobustDataParallel(copy.deepcopy(model0), F.cross_entropy, DistContext(device=dev), cfg)
    eng.step(b)
    torch.cuda.synchronize()
    names = [n for n, _ in eng.model.named_parameters()]
    i = names.index("layer3.1.conv1.weight")
    off, num = eng.flat.offsets[i], eng.flat.numels[i]
    seg = eng.G[0, off:off + num].float()
    std = gref.reshape(-1)
    cl = gref.permute(0, 2, 3, 1).reshape(-1)
    print("wb", wb, "vs standard order", ((seg - std).norm() / std.norm()).item(),
          "vs channels_last order", ((seg - cl).norm() / cl.norm()).item())
