"""Worker-grouped fp32 execution: the k logical workers of a rank as ONE pass, for the
reference's fp32 precision (``pytorch_impl/applications/Garfield_CC/trainer.py:296-303``: no
autocast).

The bf16 grouped executor (``parallel/grouped.py``) relies on hand-written bf16 kernels; at fp32
the engine used to fall back to k per-worker forward/backward passes (~7.5k small kernels per
ResNet-50 step). MIOpen's grouped fp32 convolutions are no way out either: their weight-gradient
solvers for strided / 7x7 grouped layers are the naive reference kernels (25 ms of a 90 ms step,
profiles/r3/rocprof_fp32_miopen_grouped.txt) and their Winograd kernels are not HIP-graph replay
safe. Here every activation lives in a WORKER-MAJOR layout ``[k, C, B*H*W]`` (worker g's
channels, then its B images' pixels), and every layer is a batched GEMM over the k workers:

* a 1x1 stride-1 convolution is ``bmm(W_rep [k, Cout, Cin], x [k, Cin, B*H*W])`` with ``W_rep``
  the weight repeated k times: its weight gradient IS the k per-worker gradients;
* a k x k (or strided) convolution first gathers its patches ``[k, Cin*KH*KW, B*Ho*Wo]`` in one
  strided copy (``_Patches``), then the same batched GEMM; the data gradient adds each tap's
  slice back (the adjoint gather);
* BatchNorm is ``batch_norm`` of the ``[1, k*C, B*H*W]`` view: every (worker, channel) is
  normalised with that worker's own batch statistics, and dγ/dβ of length k*C are the per-worker
  gradients; the k sequential running-statistics updates of k independent workers are replayed
  from the per-worker batch statistics (``gpu_bn_running_update``);
* ReLU, pooling and the residual additions are elementwise / per plane;
* the classifier is one more batched GEMM and the loss each worker's mean cross-entropy.

All GEMMs are plain fp32 library GEMMs (hipBLASLt through ``torch.bmm``). Every per-worker
weight gradient lands in that worker's exchange row through the GradSink (one multi-tensor cast
kernel). Exact against k independent workers run one after the other (fp64 on the CPU,
tests/test_grouped_fp32_cpu.py).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from garfield_amd import _native
from garfield_amd.models.resnet import BasicBlock, Bottleneck, ResNet
from garfield_amd.ops.grouped import GradSink


def supports(model: nn.Module) -> bool:
    """The zoo's ResNets (BatchNorm with momentum and affine parameters, plain convolutions)."""
    if not isinstance(model, ResNet):
        return False
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d) and (m.momentum is None or not m.affine or not m.track_running_stats):
            return False
        if isinstance(m, nn.Conv2d) and (m.groups != 1 or m.bias is not None):
            return False
    for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
        for blk in layer:
            if not isinstance(blk, (BasicBlock, Bottleneck)):
                return False
    return isinstance(model.maxpool, (nn.MaxPool2d, nn.Identity))


class _Act:
    """A worker-major activation: t [k, C, B*H*W] and its image geometry."""

    __slots__ = ("t", "B", "H", "W")

    def __init__(self, t, B, H, W):
        self.t, self.B, self.H, self.W = t, B, H, W

    @property
    def C(self):
        return self.t.shape[1]


class _Patches(torch.autograd.Function):
    """[k, C, B, H, W] -> the patch matrix [k, C*KH*KW, B*Ho*Wo] (unfold's (ci, i, j) row order)
    as ONE strided copy (ATen's unfold launches one im2col kernel per image: 5000 launches per
    ResNet-50 step); the backward adds each tap's gradient slice back, KH*KW strided adds."""

    @staticmethod
    def forward(ctx, x5, k, d, p, s):
        G, C, B, H, W = x5.shape
        (kh, kw), (dh, dw), (ph, pw), (sh, sw) = k, d, p, s
        xp = F.pad(x5, (pw, pw, ph, ph)) if (ph or pw) else x5
        Hp, Wp = H + 2 * ph, W + 2 * pw
        Ho, Wo = (Hp - dh * (kh - 1) - 1) // sh + 1, (Wp - dw * (kw - 1) - 1) // sw + 1
        st = xp.stride()
        v = xp.as_strided((G, C, kh, kw, B, Ho, Wo), (st[0], st[1], dh * st[3], dw * st[4], st[2], sh * st[3], sw * st[4]))
        ctx.geom = (G, C, B, H, W, kh, kw, dh, dw, ph, pw, sh, sw, Ho, Wo)
        return v.reshape(G, C * kh * kw, B * Ho * Wo)

    @staticmethod
    def backward(ctx, gcol):
        G, C, B, H, W, kh, kw, dh, dw, ph, pw, sh, sw, Ho, Wo = ctx.geom
        g7 = gcol.reshape(G, C, kh, kw, B, Ho, Wo)
        gx = torch.zeros((G, C, B, H + 2 * ph, W + 2 * pw), dtype=gcol.dtype, device=gcol.device)
        for i in range(kh):
            for j in range(kw):
                gx[:, :, :, i * dh: i * dh + sh * (Ho - 1) + 1: sh, j * dw: j * dw + sw * (Wo - 1) + 1: sw] += g7[:, :, i, j]
        return gx[:, :, :, ph: ph + H, pw: pw + W], None, None, None, None


class GroupedChannelResNet:
    """``run(x, y)``: x [k*B, C, H, W] (worker g = rows [g*B, (g+1)*B)) and labels [k*B]; writes
    every worker's parameter gradient into its exchange row through ``sink`` and returns the
    per-worker mean losses. Interface of ``parallel.grouped.GroupedResNet``."""

    def __init__(self, model: ResNet, groups: int, sink: GradSink, loss_fn=F.cross_entropy, marks=(),
                 offsets: dict | None = None, signals: bool = True):
        if not supports(model):
            raise ValueError("GroupedChannelResNet supports the zoo's ResNet models only")
        if loss_fn is not F.cross_entropy:
            raise ValueError("GroupedChannelResNet computes the per-worker mean cross-entropy")
        self.model = model
        self.groups = int(groups)
        self.sink = sink
        self.marks = ()
        self.graph_safe = True
        self._offsets = offsets or {}
        self._leaves: list = []      # (parameter, repeated leaf [k, ...])
        self._run_jobs: list = []

    # interface of GroupedResNet (no bucket marks on this path)
    def bucket_offsets(self) -> list:
        return []

    def mark_events(self):
        return None

    def replayed(self) -> None:
        pass

    # ------------------------------------------------------------------ #

    def _rep(self, p: torch.Tensor, shape) -> torch.Tensor:
        """A leaf copy of p repeated k times (leading dim k): its gradient holds the k per-worker ones."""
        G = self.groups
        r = p.detach().reshape(1, *shape).expand(G, *shape).contiguous().requires_grad_(True)
        self._leaves.append((p, r))
        return r

    def _conv(self, a: _Act, conv: nn.Conv2d) -> _Act:
        kh, kw = conv.kernel_size
        cout, cin = conv.out_channels, conv.in_channels
        # weight [Cout, Cin, KH, KW] -> [Cout, Cin*KH*KW] in unfold's (ci, i, j) column order
        w = self._rep(conv.weight, (cout, cin * kh * kw))
        if (kh, kw) == (1, 1) and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (0, 0):
            return _Act(torch.bmm(w, a.t), a.B, a.H, a.W)
        G = self.groups
        Ho = (a.H + 2 * conv.padding[0] - conv.dilation[0] * (kh - 1) - 1) // conv.stride[0] + 1
        Wo = (a.W + 2 * conv.padding[1] - conv.dilation[1] * (kw - 1) - 1) // conv.stride[1] + 1
        col = _Patches.apply(a.t.reshape(G, cin, a.B, a.H, a.W), (kh, kw), tuple(conv.dilation),
                             tuple(conv.padding), tuple(conv.stride))
        return _Act(torch.bmm(w, col), a.B, Ho, Wo)

    def _bn(self, a: _Act, bn: nn.BatchNorm2d, relu: bool, res: "_Act | None" = None) -> _Act:
        G, C = self.groups, a.C
        gamma = self._rep(bn.weight, (C,)).view(G * C)
        beta = self._rep(bn.bias, (C,)).view(G * C)
        x3 = a.t.reshape(1, G * C, -1)
        y, mean, invstd = torch.ops.aten.native_batch_norm(x3, gamma, beta, None, None, True, 0.0, bn.eps)
        if bn.running_mean is not None:
            self._run_jobs.append((mean.detach(), invstd.detach(), bn, x3.shape[2]))
        y = y.view(G, C, -1)
        if res is not None:
            y = y + res.t
        return _Act(F.relu(y) if relu else y, a.B, a.H, a.W)

    def _block(self, blk, a: _Act) -> _Act:
        out = self._bn(self._conv(a, blk.conv1), blk.bn1, True)
        if isinstance(blk, Bottleneck):
            out = self._bn(self._conv(out, blk.conv2), blk.bn2, True)
            last_conv, last_bn = blk.conv3, blk.bn3
        else:
            last_conv, last_bn = blk.conv2, blk.bn2
        sc = a if blk.downsample is None else self._bn(self._conv(a, blk.downsample[0]), blk.downsample[1], False)
        return self._bn(self._conv(out, last_conv), last_bn, True, res=sc)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [k*B, C, H, W] -> logits [k, B, classes]."""
        m, G = self.model, self.groups
        B = x.shape[0] // G
        t = x.reshape(G, B, x.shape[1], -1).transpose(1, 2).reshape(G, x.shape[1], -1)
        a = self._bn(self._conv(_Act(t, B, x.shape[2], x.shape[3]), m.conv1), m.bn1, True)
        if isinstance(m.maxpool, nn.MaxPool2d):
            mp = m.maxpool
            img = a.t.reshape(1, G * a.C * a.B, a.H, a.W)     # pooling is per plane: no layout change
            y = F.max_pool2d(img, mp.kernel_size, mp.stride, mp.padding, mp.dilation, mp.ceil_mode)
            a = _Act(y.reshape(G, a.C, -1), a.B, y.shape[2], y.shape[3])
        for name in ("layer1", "layer2", "layer3", "layer4"):
            for blk in getattr(m, name):
                a = self._block(blk, a)
        pooled = a.t.reshape(G, a.C, a.B, a.H * a.W).mean(3)             # [k, F, B]
        fc = m.fc
        w = self._rep(fc.weight, tuple(fc.weight.shape))                 # [k, O, F]
        logits = torch.bmm(w, pooled)                                    # [k, O, B]
        if fc.bias is not None:
            logits = logits + self._rep(fc.bias, (fc.bias.shape[0],))[:, :, None]
        return logits.transpose(1, 2)                                    # [k, B, O]

    def _running_updates(self) -> None:
        """The k sequential running-statistics updates of k workers, per BatchNorm."""
        G = self.groups
        if not self._run_jobs:
            return
        m0 = self._run_jobs[0][0]
        if m0.is_cuda and m0.dtype == torch.float32 and all(j[2].running_mean.dtype == torch.float32
                                                             for j in self._run_jobs):
            C_ = _native.native()
            for i in range(0, len(self._run_jobs), 48):
                C_.gpu_bn_running_update([(mean, invstd, bn.running_mean, bn.running_var, rows, float(bn.eps),
                                           float(bn.momentum)) for mean, invstd, bn, rows in self._run_jobs[i:i + 48]])
        else:
            with torch.no_grad():
                for mean, invstd, bn, rows in self._run_jobs:
                    var = (1.0 / invstd.double() ** 2 - bn.eps).clamp_min(0).view(G, -1)
                    unb = var * rows / max(rows - 1, 1)
                    mu = mean.view(G, -1)
                    for g in range(G):
                        bn.running_mean.mul_(1 - bn.momentum).add_(mu[g].to(bn.running_mean.dtype), alpha=bn.momentum)
                        bn.running_var.mul_(1 - bn.momentum).add_(unb[g].to(bn.running_var.dtype), alpha=bn.momentum)
        self._run_jobs = []

    def run(self, x: torch.Tensor, y: torch.Tensor, loss_out: torch.Tensor | None = None) -> torch.Tensor:
        G = self.groups
        if x.shape[0] % G:
            raise ValueError(f"batch of {x.shape[0]} rows is not divisible into {G} workers")
        B = x.shape[0] // G
        self._leaves = []
        self._run_jobs = []
        logits = self.forward(x.contiguous())                            # [k, B, O]
        per = F.cross_entropy(logits.reshape(G * B, -1), y.view(G * B), reduction="none").view(G, B).mean(1)
        per.sum().backward()
        self._running_updates()
        for p, r in self._leaves:
            g = r.grad.view(G, *p.shape)
            if p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last):
                g = g.permute(0, 1, 3, 4, 2).contiguous()    # [k, Cout, KH, KW, Cin]: the weight's memory order
            self.sink.put_groups(p, g)
        self._leaves = []
        self.sink.flush()
        per = per.detach()
        if loss_out is not None:
            loss_out.copy_(per)
        return per
