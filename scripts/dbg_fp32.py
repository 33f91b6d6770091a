import copy, torch, torch.nn.functional as F
from garfield_amd.models import build_model
from garfield_amd.ops.grouped import GradSink
from garfield_amd.parallel.grouped_fp32 import GroupedChannelResNet
dev = torch.device("cuda")
for dt in (torch.float32,):
    torch.manual_seed(0)
    G, B, hw = 3, 4, 32
    model = build_model("resnet18", num_classes=10).to(dev, dt)
    ref = copy.deepcopy(model)
    params = list(model.parameters())
    offsets, off = {}, 0
    for p in params:
        offsets[id(p)] = off; off += p.numel()
    d = off
    flat = torch.zeros(G * d, dtype=dt, device=dev)
    ex = GroupedChannelResNet(model, G, GradSink(flat, d, 0, offsets, G))
    x = torch.randn(G * B, 3, hw, hw, dtype=dt, device=dev); y = torch.randint(0, 10, (G * B,), device=dev)
    losses = ex.run(x, y)
    rparams = list(ref.parameters())
    names = [n for n, _ in ref.named_parameters()]
    for g in range(G):
        loss = F.cross_entropy(ref(x[g*B:(g+1)*B]), y[g*B:(g+1)*B])
        grads = torch.autograd.grad(loss, rparams)
        print(dt, g, float(loss), float(losses[g]))
        o = 0
        for n, gr in zip(names, grads):
            got = flat.view(G, d)[g, o:o+gr.numel()]
            e = ((got - gr.reshape(-1)).norm() / gr.norm().clamp_min(1e-30)).item()
            if e > 1e-3: print("  bad", n, e)
            o += gr.numel()
