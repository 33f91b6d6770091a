"""Worker-grouped fp32 execution: the k logical workers of a rank as ONE pass in a
GROUPED-CHANNEL layout, for the reference's fp32 precision.

The bf16 grouped executor (``parallel/grouped.py``) relies on hand-written bf16 kernels. At
the reference's fp32 precision (``pytorch_impl/applications/Garfield_CC/trainer.py:296-303``:
no autocast) the engine used to fall back to k per-worker forward/backward passes (MIOpen
graphs, ~7.5k small kernels per ResNet-50 step). Here the k workers' activations are laid out
as ONE tensor ``[B, k*C, H, W]`` (worker g owns channels ``[g*C, (g+1)*C)``), so that every
per-worker quantity is an ordinary per-CHANNEL quantity of a single ATen call:

* a convolution is ``conv2d(x, W_rep, groups=k)`` with ``W_rep = W`` repeated k times along
  the output channels: group g sees only worker g's channels, and the weight gradient of the
  grouped convolution IS the per-worker weight gradient ([k*Cout, Cin, kh, kw] = [k][Cout]...);
* BatchNorm over k*C channels normalises each (worker, channel) with that worker's batch
  statistics, and its dγ/dβ of length k*C are the per-worker gradients; the k sequential
  running-statistics updates of k independent workers are replayed from the per-worker
  batch statistics by one ``gpu_bn_running_update`` launch;
* ReLU, max/avg pooling and the residual additions are channel-wise, so unchanged;
* the classifier is a batched matmul against the repeated weight, and the loss the mean
  cross-entropy of every worker.

Every per-worker weight gradient lands in that worker's exchange row through the GradSink
(one multi-tensor cast kernel). Same math as k separate fp32 workers (checked on CPU against
k independent forward/backward passes, tests/test_grouped_fp32_cpu.py).
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
        self._offsets = offsets or {}
        self._leaves: list = []      # (parameter, repeated leaf, view shape of the per-worker gradient)
        self._run_jobs: list = []

    # interface of GroupedResNet (no bucket marks on this path)
    def bucket_offsets(self) -> list:
        return []

    def mark_events(self):
        return None

    def replayed(self) -> None:
        pass

    # ------------------------------------------------------------------ #

    def _rep(self, p: torch.Tensor, dim0_shape) -> torch.Tensor:
        """A leaf copy of p repeated k times along dim 0 (its gradient: the k per-worker ones)."""
        G = self.groups
        r = p.detach().unsqueeze(0).expand(G, *p.shape).reshape(*dim0_shape).requires_grad_(True)
        self._leaves.append((p, r))
        return r

    def _conv(self, x, conv: nn.Conv2d):
        G = self.groups
        w = self._rep(conv.weight, (G * conv.out_channels, *conv.weight.shape[1:]))
        return F.conv2d(x, w, None, conv.stride, conv.padding, conv.dilation, G)

    def _bn(self, x, bn: nn.BatchNorm2d, relu: bool, res=None):
        G = self.groups
        gamma = self._rep(bn.weight, (G * bn.num_features,))
        beta = self._rep(bn.bias, (G * bn.num_features,))
        y, mean, invstd = torch.ops.aten.native_batch_norm(x, gamma, beta, None, None, True, 0.0, bn.eps)
        if bn.running_mean is not None:
            rows = x.shape[0] * x.shape[2] * x.shape[3]          # rows per worker
            self._run_jobs.append((mean.detach(), invstd.detach(), bn, rows))
        if res is not None:
            y = y + res
        return F.relu(y) if relu else y

    def _block(self, blk, x):
        out = self._bn(self._conv(x, blk.conv1), blk.bn1, True)
        if isinstance(blk, Bottleneck):
            out = self._bn(self._conv(out, blk.conv2), blk.bn2, True)
            last_conv, last_bn = blk.conv3, blk.bn3
        else:
            last_conv, last_bn = blk.conv2, blk.bn2
        sc = x if blk.downsample is None else self._bn(self._conv(x, blk.downsample[0]), blk.downsample[1], False)
        return self._bn(self._conv(out, last_conv), last_bn, True, res=sc)

    def forward(self, xg: torch.Tensor) -> torch.Tensor:
        """xg: [B, k*C, H, W] -> logits [k, B, classes]."""
        m, G = self.model, self.groups
        x = self._bn(self._conv(xg, m.conv1), m.bn1, True)
        if isinstance(m.maxpool, nn.MaxPool2d):
            x = F.max_pool2d(x, m.maxpool.kernel_size, m.maxpool.stride, m.maxpool.padding, m.maxpool.dilation,
                             m.maxpool.ceil_mode)
        for name in ("layer1", "layer2", "layer3", "layer4"):
            for blk in getattr(m, name):
                x = self._block(blk, x)
        B = x.shape[0]
        pooled = x.mean((2, 3)).view(B, G, -1).transpose(0, 1)           # [k, B, F]
        fc = m.fc
        w = self._rep(fc.weight, (G, *fc.weight.shape))                  # [k, O, F]
        logits = torch.bmm(pooled, w.transpose(1, 2))
        if fc.bias is not None:
            logits = logits + self._rep(fc.bias, (G, fc.bias.shape[0]))[:, None, :]
        return logits

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
        xg = x.reshape(G, B, *x.shape[1:]).transpose(0, 1).reshape(B, G * x.shape[1], *x.shape[2:])
        logits = self.forward(xg.contiguous())                           # [k, B, O]
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
