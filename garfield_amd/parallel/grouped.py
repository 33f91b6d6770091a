"""Grouped execution of a rank's k logical workers (ResNet family).

The engine's per-worker loop (``engine.RobustDataParallel.compute_local``) runs k
independent forward/backward passes per step; for ResNet-50 on CIFAR-shape
micro-batches that is ~7.5k small kernels per step on one MI355X, and the step is
bound by kernel boundaries, not by the matrix cores. ``GroupedResNet`` runs the
same k workers as ONE NHWC batch with per-worker BatchNorm statistics and
per-worker parameter gradients (``garfield_amd.ops.grouped``), which is the same
math as k separate workers (tests/test_grouped_cpu.py checks it against k
sequential standard forward/backward passes, running statistics included).

Reference counterpart: one ``Worker.compute_gradients`` per worker process
(``pytorch_impl/libs/garfieldpp/worker.py:77-96``) on the reference's ResNet
models (``models/resnet.py``; torchvision ``resnet50`` for ``resnet50``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from garfield_amd.models.resnet import BasicBlock, Bottleneck, ResNet
from garfield_amd.parallel.signals import DeviceSignal
from garfield_amd.ops.grouped import (BNState, ConvSpec, GradJoin, GradSink, LinearSpec, ResLink, Workspace,
                                      bn_conv_ok, global_avgpool, grouped_bn, grouped_bn_conv, grouped_conv,
                                      grouped_cross_entropy, grouped_linear, grouped_maxpool, refresh_dgrad_weights,
                                      refresh_f32_weights, refresh_sc_weights)
import garfield_amd.ops.grouped as _gops


def supports(model: nn.Module) -> bool:
    """True for the zoo's ResNets with layers the grouped kernels handle."""
    if not isinstance(model, ResNet):
        return False
    for m in model.modules():
        if isinstance(m, nn.BatchNorm2d):
            if m.num_features % 8 or m.momentum is None or not m.affine:
                return False
        elif isinstance(m, nn.Conv2d):
            if m.groups != 1 or m.bias is not None:
                return False
    for layer in (model.layer1, model.layer2, model.layer3, model.layer4):
        for blk in layer:
            if not isinstance(blk, (BasicBlock, Bottleneck)):
                return False
    return isinstance(model.maxpool, (nn.MaxPool2d, nn.Identity))


INDEX_LIMIT = 2 ** 31 - 1   # the grouped kernels index activations with 32-bit element offsets
_CAPACITY: dict = {}


def largest_index(model: ResNet, rows: int, sample_shape) -> int:
    """The largest element count a grouped step of ``rows`` images of ``sample_shape`` must index:
    every convolution's input and output, every BatchNorm / pooling / ReLU output, the logits, and
    the column matrix (pixels x taps x Cin) of the strided k x k convolutions whose data gradient can
    take the dcol GEMM + col2im form (the stem runs on its own implicit kernels). Shapes come from a
    forward on meta tensors (no memory, no kernel); cached per (model, rows, shape)."""
    key = (id(model), int(rows), tuple(sample_shape))
    hit = _CAPACITY.get(key)
    if hit is not None:
        return hit
    sizes = [int(rows) * int(torch.Size(sample_shape).numel())]

    def hook(mod, inp, out):
        sizes.append(out.numel())
        if isinstance(mod, nn.Conv2d):
            sizes.append(inp[0].numel())
            kh, kw = mod.kernel_size
            if mod is not model.conv1 and kh * kw > 1 and tuple(mod.stride) != (1, 1):
                sizes.append(out.numel() // mod.out_channels * mod.in_channels * kh * kw)

    hooks = [m.register_forward_hook(hook) for m in model.modules()
             if isinstance(m, (nn.Conv2d, nn.BatchNorm2d, nn.MaxPool2d, nn.ReLU, nn.Linear, nn.AdaptiveAvgPool2d))]
    state = {n: torch.empty_like(t, device="meta") for n, t in [*model.named_parameters(), *model.named_buffers()]}
    try:
        with torch.no_grad():
            torch.func.functional_call(model, state, (torch.empty((rows, *sample_shape), device="meta"),))
    finally:
        for h in hooks:
            h.remove()
    _CAPACITY[key] = out = max(sizes)
    return out


def fits(model: ResNet, rows: int, sample_shape) -> bool:
    """Whether a grouped step of ``rows`` images stays within the kernels' 32-bit indexing."""
    return largest_index(model, rows, sample_shape) <= INDEX_LIMIT


class GroupedResNet:
    """Forward + backward of ``groups`` workers' micro-batches in one pass.

    ``run(x, y)`` takes the concatenated inputs (worker g = rows [g*B, (g+1)*B),
    channels_last) and labels, writes every worker's parameter gradient into its
    exchange row through ``sink`` and returns the per-worker mean losses."""

    def __init__(self, model: ResNet, groups: int, sink: GradSink, loss_fn=F.cross_entropy, marks=(),
                 offsets: dict | None = None, signals: bool = True):
        if not supports(model):
            raise ValueError("GroupedResNet supports the zoo's ResNet models only")
        self.model = model
        self.groups = int(groups)
        self.sink = sink
        self.loss_fn = loss_fn
        self.ws = Workspace()
        self.conv = {m: ConvSpec(m, sink, self.groups) for m in model.modules() if isinstance(m, nn.Conv2d)}
        self.fc = LinearSpec(model.fc, sink, self.groups)
        self.bn: dict = {}
        self._seed = None
        self.join_residuals = True
        # bucket marks: the backward records a device signal when it has produced every
        # gradient of the named layer and the layers after it (the exchange of that
        # bucket can start), and one more at the very end (the last bucket). Inside the
        # captured HIP graph each is a 1-lane counter kernel that fires on every replay
        # (parallel/signals.py: no HIP event, so no cross-stream dependency on the main
        # stream).
        self.marks = tuple(marks)
        self._offsets = offsets or {}
        self._events = None
        self._end = None
        if signals and self.marks and next(model.parameters()).is_cuda:   # else the marks only cut buckets
            dev = next(model.parameters()).device
            self._events = {name: DeviceSignal(dev) for name in self.marks}
            self._end = DeviceSignal(dev)

    def bucket_offsets(self) -> list:
        """Flat offset where each marked layer's parameters start (bucket boundaries)."""
        out = []
        for name in self.marks:
            layer = getattr(self.model, name)
            offs = [self._offsets[id(p)] for p in layer.parameters() if id(p) in self._offsets]
            if offs:
                out.append(min(offs))
        return out

    def mark_events(self):
        """Signals in the order the backward records them (the marks' order, then the end of
        the backward), or None."""
        if self._events is None:
            return None
        return [self._events[name] for name in self.marks] + [self._end]

    def replayed(self) -> None:
        """One replay of a captured run(): every signal fired once more."""
        for sgn in self.mark_events() or ():
            sgn.replayed()

    # ------------------------------------------------------------------ #

    def _state(self, bn: nn.BatchNorm2d, relu: bool) -> BNState:
        st = self.bn.get(bn)
        if st is None:
            st = self.bn[bn] = BNState(bn, relu, self.sink, self.groups)
        return st

    def _bn(self, x, bn: nn.BatchNorm2d, relu: bool, res=None, res_join=None, res_link=None, out_link=None):
        return grouped_bn(x, self._state(bn, relu), self.ws, res, res_join, res_link, out_link)

    def _conv(self, x, conv: nn.Conv2d, join=None):
        return grouped_conv(x, self.conv[conv], join)

    def _conv_bn(self, x, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool, join=None, res=None, res_join=None,
                 res_link=None, out_link=None, res_st=None):
        """conv -> BatchNorm; the convolution may hand the BatchNorm its statistics (gemm_nt.hip)."""
        st = self._state(bn, relu)
        y = self._conv_stats(x, conv, st, join)
        return grouped_bn(y, st, self.ws, res, res_join, res_link, out_link, res_st)

    def _conv_stats(self, x, conv: nn.Conv2d, st, join=None):
        """The convolution, handing the BatchNorm ``st`` its statistics when its kernel can."""
        spec = self.conv[conv]
        spec.bn_next = st
        try:
            return grouped_conv(x, spec, join)
        finally:
            spec.bn_next = None

    def _shortcut(self, blk, x, join):
        """A projection block's shortcut: (pre-BatchNorm output, its BatchNorm state) when that BatchNorm
        is folded into the block's last one (GPU), else (its normalised output, None) and the ResLink."""
        conv, bn = blk.downsample[0], blk.downsample[1]
        if _gops.FOLD_SHORTCUT_BN and x.is_cuda and isinstance(bn, nn.BatchNorm2d):
            st = self._state(bn, False)
            return self._conv_stats(x, conv, st, join), st, None
        link = ResLink()   # the shortcut BatchNorm receives the residual gradient as dy + ReLU bits
        return self._conv_bn(x, conv, bn, False, join, out_link=link), None, link

    def _block(self, blk, x):
        # x's two gradient branches (conv1 and the shortcut) are summed inside the
        # second branch's backward kernel instead of by an autograd add
        join = GradJoin() if self.join_residuals else None
        out = self._conv_bn(x, blk.conv1, blk.bn1, True, join)
        if isinstance(blk, Bottleneck):
            st2 = self._state(blk.bn2, True)
            spec2 = self.conv[blk.conv2]
            spec2.bn_next = st2
            try:
                x2 = grouped_conv(out, spec2)            # pre-bn2 (with bn2's statistics when the conv has them)
            finally:
                spec2.bn_next = None
            spec3 = self.conv[blk.conv3]
            if bn_conv_ok(x2, st2, spec3):
                # bn2 + ReLU applied by conv3's kernels: the normalised activation is never written
                st3 = self._state(blk.bn3, True)
                spec3.bn_next = st3
                try:
                    y3 = grouped_bn_conv(x2, st2, self.ws, spec3)
                finally:
                    spec3.bn_next = None
                if blk.downsample is None:
                    return grouped_bn(y3, st3, self.ws, x, join)
                sc, sst, link = self._shortcut(blk, x, join)
                return grouped_bn(y3, st3, self.ws, sc, res_link=link, res_st=sst)
            out = grouped_bn(x2, st2, self.ws)
            last_conv, last_bn = blk.conv3, blk.bn3
        else:
            last_conv, last_bn = blk.conv2, blk.bn2
        if blk.downsample is None:
            return self._conv_bn(out, last_conv, last_bn, True, res=x, res_join=join)
        sc, sst, link = self._shortcut(blk, x, join)
        return self._conv_bn(out, last_conv, last_bn, True, res=sc, res_link=link, res_st=sst)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = []
        for _ in self._forward_stages(x, out):
            pass
        return out[0]

    def _forward_stages(self, x: torch.Tensor, out: list):
        """The forward, yielding before each marked layer (a bucket boundary): the stage
        that follows reads that bucket's weights first. The logits land in ``out``."""
        m = self.model
        # small layers' running statistics: one batched launch after the last BatchNorm
        self.ws.defer_running = x.is_cuda
        self.ws.running_jobs = []
        x = self._conv_bn(x, m.conv1, m.bn1, True)
        if isinstance(m.maxpool, nn.MaxPool2d):
            x = grouped_maxpool(x, m.maxpool)
        for name in ("layer1", "layer2", "layer3", "layer4"):
            if self._events is not None and name in self._events:
                x = _BucketMark.apply(x, self._events[name], self.sink)
            if name in self.marks:
                yield name
            if x.is_cuda and x.dtype != torch.float32:
                # this layer's small-image convolutions (2x2 / 1x1 inputs): expanded weights, one launch, after
                # the stage boundary (the staged step updates this bucket's weights up to its event)
                refresh_sc_weights([self.conv[c] for c in getattr(m, name).modules() if isinstance(c, nn.Conv2d)])
            for blk in getattr(m, name):
                x = self._block(blk, x)
        self.ws.flush_running()
        out.append(grouped_linear(global_avgpool(x), self.fc))

    def stage_ends(self, ld: int) -> list:
        """Flat offset where the parameters each stage of ``run_stages`` reads end: the
        stages cut at the marked layers, in forward order; the last one (the rest of the
        forward and the whole backward, which writes every gradient row) ends at ``ld``."""
        offs = []
        for name in ("layer1", "layer2", "layer3", "layer4"):
            if name in self.marks:
                layer = getattr(self.model, name)
                o = [self._offsets[id(p)] for p in layer.parameters() if id(p) in self._offsets]
                if o:
                    offs.append(min(o))
        return [*offs, ld]

    def stageable(self, x: torch.Tensor) -> bool:
        """Whether ``run_stages``' stages read only their own bucket's weights: the bf16 step
        (its backward's transposed 1x1 weights are refreshed after the forward); the fp32
        step splits every weight into bf16 pieces before the forward."""
        return bool(self.marks) and x.is_cuda and x.dtype != torch.float32

    def losses(self, logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        G = self.groups
        if self.loss_fn is F.cross_entropy:
            return grouped_cross_entropy(logits, y, G)
        if logits.dtype != torch.float64:
            logits = logits.float()
        lg = logits.view(G, -1, logits.shape[-1])
        yg = y.view(G, -1, *y.shape[1:])
        return torch.stack([self.loss_fn(lg[g], yg[g]) for g in range(G)])

    def run(self, x: torch.Tensor, y: torch.Tensor, loss_out: torch.Tensor | None = None) -> torch.Tensor:
        for _ in self.run_stages(x, y, loss_out):
            pass
        return self._per

    def run_stages(self, x: torch.Tensor, y: torch.Tensor, loss_out: torch.Tensor | None = None):
        """``run`` cut into stages at the marked layers (a generator: it yields between stages).
        The engine captures each stage as its own HIP graph, so the next step's stem-to-layer2
        forward can start while the later buckets' updates and weight all-gathers still run
        on the comm stream (each later stage waits for its bucket's event)."""
        if x.shape[0] % self.groups:
            raise ValueError(f"batch of {x.shape[0]} rows is not divisible into {self.groups} workers")
        if x.is_cuda and x.dtype == torch.float32:
            refresh_f32_weights(self.conv.values())     # the fp32 step's split weights: one launch
        out = []
        yield from self._forward_stages(x, out)
        if x.is_cuda and x.dtype != torch.float32:
            refresh_dgrad_weights(self.conv.values())   # the backward's Wᵀ of every 1x1 layer: one launch
        per = self.losses(out[0], y)
        # d(Σ_g loss_g)/d loss_g = 1: seeded directly (no sum / fill / expand kernels)
        if self._seed is None or self._seed.shape != per.shape or self._seed.device != per.device \
                or self._seed.dtype != per.dtype:
            self._seed = torch.ones_like(per)
        per.backward(self._seed)
        self.sink.flush()
        if self._end is not None:
            self._end.record(torch.cuda.current_stream(x.device))
        per = per.detach()
        if loss_out is not None:
            loss_out.copy_(per)
        self._per = per


class _BucketMark(torch.autograd.Function):
    """Identity whose backward records ``event`` (a DeviceSignal) on the current stream:
    by then the backward has produced every gradient of the layers after this point
    (the split-K weight-gradient sums queued so far are flushed first, so the
    bucket's rows are complete when the event fires)."""

    @staticmethod
    def forward(ctx, x, event, sink):
        ctx.event, ctx.sink = event, sink
        return x.view_as(x)

    @staticmethod
    def backward(ctx, dy):
        if ctx.sink is not None:
            ctx.sink.flush_splits()
        ctx.event.record(torch.cuda.current_stream(dy.device))
        return dy, None, None
