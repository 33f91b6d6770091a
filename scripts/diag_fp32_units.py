"""fp32 kernels at the CIFAR ResNet-18 / ResNet-50 step's own shapes (N = k * B images): forward,
data gradient with and without the fused add (the residual join), weight gradient, BatchNorm --
each vs float64, worst relative error per op printed."""
import sys

import torch
import torch.nn.functional as F

from garfield_amd import _native


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


C = _native.native()
dev = torch.device("cuda", 0)
torch.manual_seed(0)
G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
N = G * B
shapes = [  # Cin, Cout, H, k, s, p
    (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (64, 128, 32, 1, 2, 0), (128, 128, 16, 3, 1, 1),
    (128, 256, 16, 3, 2, 1), (128, 256, 16, 1, 2, 0), (256, 256, 8, 3, 1, 1), (256, 512, 8, 3, 2, 1),
    (256, 512, 8, 1, 2, 0), (512, 512, 4, 3, 1, 1), (64, 256, 32, 1, 1, 0), (256, 64, 32, 1, 1, 0),
    (512, 1024, 8, 1, 2, 0), (1024, 2048, 4, 1, 2, 0), (128, 128, 32, 3, 2, 1)]
for cin, cout, H, k, s, p in shapes:
    x = cl(torch.randn(N, cin, H, H, device=dev))
    w = cl(torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5)
    K = k * k * cin
    w3 = torch.empty((3, cout, K), dtype=torch.bfloat16, device=dev)
    wt3 = torch.empty((3, cin, k * k * cout), dtype=torch.bfloat16, device=dev)
    C.gpu_wsplit_multi([(w, w3, wt3, cout, k * k, cin, 0)])
    ref = F.conv2d(x.double(), w.double(), None, s, p)
    y = cl(torch.full(ref.shape, float("nan"), device=dev))
    C.gpu_conv_f32(x, w3, k, k, s, s, p, p, 1, 1, False, y, None, 0)
    e_fwd = rel(y, ref)
    dy = cl(torch.randn(ref.shape, device=dev))
    dref = torch.nn.grad.conv2d_input(x.shape, w.double(), dy.double(), s, p)
    dx = cl(torch.full(x.shape, float("nan"), device=dev))
    C.gpu_conv_f32(dy, wt3, k, k, s, s, p, p, 1, 1, True, dx, None, 0)
    e_dg = rel(dx, dref)
    add = cl(torch.randn(x.shape, device=dev))
    dx2 = add.clone()
    C.gpu_conv_f32(dy, wt3, k, k, s, s, p, p, 1, 1, True, dx2, dx2, 0)
    e_dga = rel(dx2, dref + add.double())
    part = torch.full((1, G, cout, K), float("nan"), device=dev)
    rows = N * ref.shape[2] * ref.shape[3] // G
    S = 1
    while S < 16 and rows // (2 * S) >= 256:
        S *= 2
    part = torch.full((S, G, cout, K), float("nan"), device=dev)
    C.gpu_wgrad_f32(x, dy, k, k, s, s, p, p, 1, 1, G, part, S)
    e_wg = 0.0
    for g in range(G):
        sl = slice(g * B, (g + 1) * B)
        dw = torch.nn.grad.conv2d_weight(x[sl].double(), (cout, cin, k, k), dy[sl].double(), s, p)
        e_wg = max(e_wg, rel(part[:, g].sum(0), dw.permute(0, 2, 3, 1).reshape(cout, K)))
    print(f"conv {cin:5d}->{cout:5d} H{H:3d} k{k} s{s}: fwd {e_fwd:.2e} dgrad {e_dg:.2e} dgrad+add {e_dga:.2e} "
          f"wgrad(S={S}) {e_wg:.2e}", flush=True)

from garfield_amd.ops.grouped import BNState, GradSink, Workspace, grouped_bn  # noqa: E402

for Cc, H, relu, res in [(64, 32, True, False), (64, 32, True, True), (128, 16, True, True), (256, 8, False, False),
                         (512, 4, True, True), (2048, 4, True, True), (256, 32, False, False)]:
    bn = torch.nn.BatchNorm2d(Cc).to(dev)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    flat = torch.zeros(G * 4 * Cc, device=dev)
    sink = GradSink(flat, 4 * Cc, 0, {id(bn.weight): 0, id(bn.bias): Cc}, G)
    st = BNState(bn, relu, sink, G)
    x = cl(torch.randn(N, Cc, H, H, device=dev) * 3 + 1).requires_grad_(True)
    r = cl(torch.randn(N, Cc, H, H, device=dev)).requires_grad_(True) if res else None
    y = grouped_bn(x, st, Workspace(), r)
    dy = cl(torch.randn(y.shape, device=dev))
    y.backward(dy)
    sink.flush()
    worst = [0.0] * 4
    for g in range(G):
        sl = slice(g * B, (g + 1) * B)
        xg = x[sl].detach().double().requires_grad_(True)
        wv = bn.weight.detach().double().requires_grad_(True)
        bv = bn.bias.detach().double().requires_grad_(True)
        yr = F.batch_norm(xg, None, None, wv, bv, True, 0.0, bn.eps)
        if res:
            yr = yr + r[sl].detach().double()
        if relu:
            yr = yr.clamp_min(0)
        yr.backward(dy[sl].double())
        errs = [rel(y[sl], yr), rel(x.grad[sl], xg.grad), rel(flat[g * 4 * Cc: g * 4 * Cc + Cc], wv.grad),
                rel(flat[g * 4 * Cc + Cc: g * 4 * Cc + 2 * Cc], bv.grad)]
        worst = [max(a, b) for a, b in zip(worst, errs)]
    print(f"bn C{Cc} H{H} relu{int(relu)} res{int(res)}: y {worst[0]:.2e} dx {worst[1]:.2e} dg {worst[2]:.2e} "
          f"db {worst[3]:.2e}", flush=True)
