"""Worker-grouped layers: the k logical workers of a rank as ONE batched pass.

The reference computes each worker's gradient in its own process, one batch at a
time (``pytorch_impl/libs/garfieldpp/worker.py:77-96``). Its robust rules need
every worker's gradient *separately*, so a naive port runs k small forward/
backward passes per GPU: ResNet-50 on CIFAR-shape batches of 250 is ~960 small
kernels per worker, and on MI355X the step becomes kernel-boundary bound (1.5-2 µs
per dependent launch, tiny grids on 256 CUs).

Here the k workers' micro-batches are concatenated into one NHWC batch. Only two
things couple samples, and both are kept per worker:

* **BatchNorm statistics**: ``grouped_bn`` normalises each worker's rows with
  that worker's own mean/variance (hand-written HIP kernels ``bn_nhwc.hip``, with
  the ReLU and the residual add fused) and replays the k sequential running-stat
  updates;
* **parameter gradients**: the weight gradient of every layer is produced per
  worker (the implicit-GEMM MFMA kernel ``iconv_nhwc.hip:k_iwgrad`` for the
  k x k layers, one strided-batched GEMM for 1x1 convolutions and the classifier,
  an NHWC im2col gather + batched GEMM for the rest, e.g. the 3-channel stem) and
  lands in that worker's row of the exchange buffer (written in place through
  ``GradSink.rows_view``, or queued for one multi-tensor cast kernel);
  BatchNorm's dγ/dβ are written there directly by the finalize kernel.

Activation gradients (dgrad) and forward convolutions run once on the whole
batch: implicit-GEMM MFMA convolutions (``k_iconv_lds``, no im2col matrix) for the
k x k layers with enough workgroups (the halo-staged conv3x3_nhwc.hip kernels for 3x3 stride-1),
the hand-written MFMA GEMMs of gemm_nt.hip on the NHWC rows for 1x1 stride-1 layers, im2col +
gemm_nt (+ col2im) otherwise. Library GEMMs remain only as fallbacks for shapes no kernel takes
(e.g. channel counts that are not multiples of 64) and for a 1000-class ImageNet classifier. The two gradient branches of
a residual block's input are summed inside the second branch's kernel
(``GradJoin``). The custom autograd functions take the real
parameters as inputs (so the graph reaches them) but return ``None`` for them:
nothing is accumulated into ``.grad``.

CPU tensors take plain PyTorch implementations of the same math (used by the CPU
test suite); on the GPU the native extension is mandatory.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from garfield_amd import _native
from garfield_amd.ops import tuning
from garfield_amd.utils.flat import is_dense

# Kernel choices of the grouped step. Each was measured against the path it replaced (the
# profiles cited at each switch's use); they stay module flags so tests can compare the two.
# Implicit-GEMM MFMA convolutions (iconv_nhwc.hip) for the k x k layers whose channel counts fit its
# tiles (C % 64, Cout % 64): forward, and the stride-1 data gradient as a convolution with the flipped
# weight; else im2col + GEMM.
ICONV = True
# Their per-worker weight gradients by the implicit MFMA kernel (no im2col matrix) ...
IWGRAD = True
# ... and for the 1x1 stride-1 convolutions too: 6.77-6.83 vs 6.82-6.88 ms/step for the split-K batched
# GEMM (profiles/r2/ab_iwgrad_1x1.log)
IWGRAD_1X1 = True
# The ResNet stem (7x7/2, 3 -> 64 channels) on its own implicit MFMA kernels (stem_nhwc.hip): no im2col
# patch matrix in the forward or the weight gradient.
STEM = True
_STEM_WG = 1024   # stem weight-gradient workgroups to aim for
XENT = True       # fused per-worker cross-entropy kernel (loss_xent.hip)
# 1x1 stride-1 convolutions (forward and data gradient) on the hand-written MFMA GEMMs of gemm_nt.hip
# instead of hipBLASLt: the weight-stationary persistent kernel for K <= 256, the K-loop kernel
# otherwise. The forward also emits the next (large-layer) BatchNorm's per-worker statistics from its
# registers, so that BatchNorm runs no partial-sum pass (profiles/r3/bench_gemm_nt.json.log).
GEMM_NT = True
GEMM_NT_DGRAD = True
# 3x3 / stride-1 / pad-1 convolutions on the halo-staged kernel (conv3x3_nhwc.hip) wherever its tiles fit:
# the forward through gpu_iconv's automatic choice, the data gradient on the flipped transposed weight
# (refresh_dgrad_weights) (profiles/r3/conv3x3/).
CONV3X3 = True
# A bottleneck's bn2 + ReLU applied inside its 1x1 conv3 (GEMM prologue, weight-gradient prologue, ReLU test
# recomputed in the BatchNorm backward): the normalised activation is never written (_GroupedBNConv).
# Measured slower on the CIFAR and ImageNet steps (profiles/r5/bn_prologue/): off; tests exercise it.
BN_PROLOGUE = False
# Data gradients of the stride-2 convolutions (3x3 downsampling, 1x1 projection shortcut) on the parity-class
# MFMA kernel (iconv_nhwc.hip S2) instead of a dcol GEMM + col2im, per layer where the first (eager) step
# measured it faster (ResNet-18 CIFAR: 15.20 -> 14.93 ms/step; ResNet-50 CIFAR / ImageNet layers keep the
# GEMM: profiles/r5/s2_dgrad/).
S2_DGRAD = True
_S2_CHOICE: dict = tuning.register("s2", {})   # (dy shape, w shape, dx shape, kernel, padding) -> use the parity-class kernel
S2_FORCE = False        # tests: take the parity-class kernel wherever it fits, unmeasured
# 3x3 / stride-1 / pad-1 convolutions on images of at most 2x2 pixels (ResNet-50 CIFAR layer3 / layer4) as
# dense GEMMs over [N, P * C] rows with the per-step expanded weight (sconv_nhwc.hip): no out-of-image
# taps computed (2.25x / 9x of the useful MFMA work on the implicit-GEMM / im2col paths).
SMALL_CONV = True
# An identity block's residual gradient (dres = dy masked by the last BatchNorm's ReLU) is not written by
# that BatchNorm's backward when the block's conv1 is a 1x1 GEMM: conv1's data-gradient epilogue adds
# dy where the forward's ReLU bit is set (gpu_gemm_nt add_mask), saving dres's write and re-read (MaskedGrad).
LAZY_RES = True
# A projection block's shortcut BatchNorm folded into the block's last BatchNorm (statistics pass only,
# its scale / shift applied to the pre-BatchNorm shortcut inside the last BatchNorm's apply pass, its
# backward run there too): the shortcut's normalised activation is never written (_GroupedBN res_st).
FOLD_SHORTCUT_BN = True
# ... and its backward shares one statistics pass and one apply pass with the last BatchNorm's (a ReLU-bit
# mask or none; tests set False to run the two-call form, which a saved ReLU output still takes)
BN_DUAL = True


def rows2d(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last tensor -> its [N*H*W, C] row view (no copy)."""
    if t.dim() == 2:
        return t
    if not t.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("grouped layers need channels_last activations")
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def from_rows(t2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    """[N*H*W, C] rows -> [N, C, H, W] channels_last view."""
    return t2.view(n, h, w, t2.shape[1]).permute(0, 3, 1, 2)


def _cl(t: torch.Tensor) -> torch.Tensor:
    return t.contiguous(memory_format=torch.channels_last) if t.dim() == 4 else t.contiguous()


# --------------------------------------------------------------------------- #
# Gradient sink: per-worker parameter gradients -> exchange-buffer rows


class GradSink:
    """Routes per-worker parameter gradients into the exchange buffer.

    ``flat`` is the whole exchange buffer (1-D); worker g's row starts at
    ``base + g * row_stride``; parameter p occupies ``[offset(p), offset(p) + numel)``
    of a row, in the parameter's MEMORY order (the flat-parameter layout).
    Dense per-worker gradient tensors are queued with ``put`` and written by one
    multi-tensor cast kernel in ``flush``."""

    def __init__(self, flat: torch.Tensor, row_stride: int, base: int, offsets: dict, groups: int):
        self.flat = flat
        self.row_stride = int(row_stride)
        self.base = int(base)
        self.offsets = offsets        # id(param) -> element offset inside a row
        self.groups = int(groups)
        self._srcs: list = []
        self._offs: list = []
        self._split_parts: list = []   # deferred split-K sums (part [S, G, ...] fp32, out [G, ...] rows)
        self._split_outs: list = []
        self.defer_splits = True

    def offset(self, p: torch.Tensor) -> int:
        return self.offsets[id(p)]

    def row_offset(self, g: int, p: torch.Tensor) -> int:
        return self.base + g * self.row_stride + self.offsets[id(p)]

    def put(self, p: torch.Tensor, g: int, grad: torch.Tensor) -> None:
        if grad.numel() != p.numel():
            raise ValueError(f"gradient of {grad.numel()} elements for a parameter of {p.numel()}")
        self._srcs.append(grad)
        self._offs.append(self.row_offset(g, p))

    def rows_view(self, p: torch.Tensor, shape: tuple, dtype: torch.dtype) -> torch.Tensor | None:
        """[groups, *shape] view of parameter p's slots in every worker row (``shape``:
        p's memory-order shape, last dim contiguous), for GEMMs / reductions that write
        the per-worker gradients in place; None when the exchange dtype is not
        ``dtype`` (the caller then queues a ``put``)."""
        if self.flat.dtype != dtype:
            return None
        strides, acc = [], 1
        for d in reversed(shape):
            strides.append(acc)
            acc *= int(d)
        if acc != p.numel():
            raise ValueError(f"rows_view of {acc} elements for a parameter of {p.numel()}")
        return self.flat.as_strided((self.groups, *shape), (self.row_stride, *reversed(strides)),
                                    self.base + self.offsets[id(p)])

    def queue_split(self, part: torch.Tensor, out: torch.Tensor) -> None:
        """Σ_s part[s] -> out, deferred to ``flush`` where every queued layer's split-K sum runs
        in ONE launch (the exchange rows are read only after the backward)."""
        if self.defer_splits and part.is_cuda:
            self._split_parts.append(part)
            self._split_outs.append(out)
        else:
            _native.native().gpu_split_reduce(part, out)

    def put_groups(self, p: torch.Tensor, grads) -> None:
        """``grads``: [groups, ...] tensor or a list of per-group tensors."""
        for g in range(self.groups):
            self.put(p, g, grads[g])

    def flush_splits(self) -> None:
        """Run the queued split-K sums now (one launch), e.g. before a bucket mark."""
        if self._split_parts:
            _native.native().gpu_split_reduce_multi(self._split_parts, self._split_outs)
            self._split_parts.clear()
            self._split_outs.clear()

    def flush(self) -> None:
        self.flush_splits()
        if not self._srcs:
            return
        if self.flat.is_cuda:
            srcs = [s if is_dense(s) else s.contiguous() for s in self._srcs]
            _native.native().gpu_flatten_cast_at(srcs, self._offs, self.flat)
        else:
            with torch.no_grad():
                for s, o in zip(self._srcs, self._offs):
                    v = _memory_order(s)
                    self.flat[o:o + v.numel()].copy_(v)
        self._srcs.clear()
        self._offs.clear()


def _memory_order(t: torch.Tensor) -> torch.Tensor:
    if t.is_contiguous():
        return t.reshape(-1)
    perm = sorted(range(t.dim()), key=lambda i: -t.stride(i))
    return t.permute(perm).reshape(-1)


class GradJoin:
    """Sums the two gradient branches of one activation inside a backward kernel.

    A residual block's input x is read by two branches (conv1 and the shortcut:
    the identity, through the last BatchNorm's residual input, or the downsample
    convolution). Autograd would produce both gradients and add them with a
    separate elementwise kernel. Instead, the branch whose backward runs FIRST
    parks its gradient here and returns None for x; the second one folds it into
    its own output (``addmm_`` for a 1x1 GEMM dgrad, an accumulating col2im for a
    k x k one) and returns the sum. A fresh join is made per forward."""

    __slots__ = ("pending", "lazy")

    def __init__(self):
        self.pending = None
        self.lazy = False     # the other branch folds a MaskedGrad into its GEMM epilogue (set by its forward)

    def take(self):
        prev, self.pending = self.pending, None
        return prev

    def park(self, g: torch.Tensor) -> None:
        if self.pending is not None:
            raise RuntimeError("GradJoin: both branches parked a gradient")
        self.pending = g


class MaskedGrad:
    """dres = dy where the forward ReLU bit is set, else 0, not materialised: dy [N, C, H, W]
    channels_last and the BatchNorm's bit mask (one byte per 8 elements in dy's memory order)."""

    __slots__ = ("dy", "mask")

    def __init__(self, dy: torch.Tensor, mask: torch.Tensor):
        self.dy, self.mask = dy, mask

    def materialize(self) -> torch.Tensor:
        bits = (self.mask.unsqueeze(1) >> torch.arange(8, dtype=torch.uint8, device=self.mask.device)) & 1
        d2 = rows2d(self.dy)
        out = torch.where(bits.view(d2.shape).bool(), d2, torch.zeros((), dtype=d2.dtype, device=d2.device))
        n, _, h, w = self.dy.shape
        return from_rows(out, n, h, w)


class ResLink:
    """A projection-shortcut block's residual gradient, handed from the block's last BatchNorm (whose
    residual input is the shortcut BatchNorm's output) to the shortcut BatchNorm's backward as dy + the
    ReLU bits (MaskedGrad) instead of a written dres: autograd passes None along that edge, and the
    shortcut BatchNorm (no ReLU of its own) applies the bits as its ReLU mask."""

    __slots__ = ("pending", "ok")

    def __init__(self):
        self.pending = None
        self.ok = False          # set by the shortcut BatchNorm's forward: it can take a MaskedGrad


# --------------------------------------------------------------------------- #
# Grouped BatchNorm (+ residual) (+ ReLU)


class BNState:
    """Per-layer buffers of a grouped BatchNorm (allocated once, reused: capture-safe)."""

    def __init__(self, bn: torch.nn.BatchNorm2d, relu: bool, sink: GradSink | None, groups: int):
        if bn.momentum is None:
            raise ValueError("grouped BatchNorm needs a momentum (cumulative averaging is not supported)")
        self.bn = bn
        self.relu = relu
        self.sink = sink
        self.groups = groups
        self.C = bn.num_features
        self.mean = self.istd = self.scale = self.shift = None
        self.tile = None          # (stats, H, E): statistics of the next input, from the producing GEMM

    def ensure(self, device, dtype=torch.float32) -> None:
        if self.mean is None or self.mean.device != device or self.mean.dtype != dtype:
            shape = (self.groups, self.C)
            self.mean = torch.empty(shape, dtype=dtype, device=device)
            self.istd = torch.empty_like(self.mean)
            self.scale = torch.empty_like(self.mean)
            self.shift = torch.empty_like(self.mean)


class Workspace:
    """Shared scratch (BatchNorm partial sums / backward coefficients), and the
    running-statistics updates deferred by single-kernel (small) BatchNorm layers
    when ``defer_running`` is set: ``flush_running`` replays them in one launch."""

    def __init__(self):
        self.t = {}
        self.defer_running = False
        self.running_jobs: list = []

    def flush_running(self) -> None:
        if self.running_jobs:
            _native.native().gpu_bn_running_update(self.running_jobs)
            self.running_jobs = []

    def get(self, name: str, numel: int, device) -> torch.Tensor:
        t = self.t.get(name)
        if t is None or t.numel() < numel or t.device != device:
            t = torch.empty(max(int(numel), 1), dtype=torch.float32, device=device)
            self.t[name] = t
        return t


def _acc(t: torch.Tensor) -> torch.Tensor:
    """Accumulation dtype of the CPU reference path: fp64 stays fp64, the rest fp32."""
    return t if t.dtype == torch.float64 else t.float()


def _affine(bn, like):
    gamma = bn.weight.detach().to(like.dtype) if bn.weight is not None else torch.ones_like(like)
    beta = bn.bias.detach().to(like.dtype) if bn.bias is not None else torch.zeros_like(like)
    return gamma, beta


def _bn_fwd_ref(x2, r2, st: BNState):
    """fp32 PyTorch reference of the grouped forward (CPU path)."""
    bn, G = st.bn, st.groups
    xg = _acc(x2).view(G, -1, st.C)
    M = xg.shape[1]
    mean = xg.mean(1)
    var = xg.var(1, unbiased=False)
    istd = torch.rsqrt(var + bn.eps)
    gamma, beta = _affine(bn, mean[0])
    scale = istd * gamma
    shift = beta - mean * scale
    y = xg * scale[:, None] + shift[:, None]
    if r2 is not None:
        y = y + _acc(r2).view(G, -1, st.C)
    if st.relu:
        y = y.clamp_min(0)
    st.mean.copy_(mean)
    st.istd.copy_(istd)
    st.scale.copy_(scale)
    st.shift.copy_(shift)
    if bn.track_running_stats and bn.running_mean is not None:
        m = bn.momentum
        unb = var * M / max(M - 1, 1)
        with torch.no_grad():
            for g in range(G):
                bn.running_mean.mul_(1 - m).add_(mean[g], alpha=m)
                bn.running_var.mul_(1 - m).add_(unb[g], alpha=m)
    return y.view(-1, st.C).to(x2.dtype)


def _bn_bwd_ref(x2, dy2, y2, st: BNState, need_res: bool):
    bn, G = st.bn, st.groups
    xg = _acc(x2).view(G, -1, st.C)
    dz = _acc(dy2).view(G, -1, st.C)
    if st.relu:
        dz = torch.where(y2.view(G, -1, st.C) > 0, dz, torch.zeros_like(dz))
    M = xg.shape[1]
    mean, istd = st.mean.to(xg.dtype), st.istd.to(xg.dtype)
    xm = xg - mean[:, None]
    A = dz.sum(1)
    B = (dz * xm).sum(1)
    dgamma = B * istd
    dbeta = A
    gamma, _ = _affine(bn, A[0])
    dx = (gamma * istd)[:, None] * (dz - (A / M)[:, None] - xm * (istd * dgamma / M)[:, None])
    if st.sink is not None:
        with torch.no_grad():
            for g in range(G):
                if bn.weight is not None:
                    o = st.sink.row_offset(g, bn.weight)
                    st.sink.flat[o:o + st.C].copy_(dgamma[g])
                if bn.bias is not None:
                    o = st.sink.row_offset(g, bn.bias)
                    st.sink.flat[o:o + st.C].copy_(dbeta[g])
    dres = dz.reshape(-1, st.C).to(x2.dtype) if need_res else None
    return dx.reshape(-1, st.C).to(x2.dtype), dres


def _bn_forward_gpu(x2: torch.Tensor, r2, st: BNState, ws: Workspace, y2, relu_state, res_st: "BNState | None" = None):
    """One grouped BatchNorm forward on the HIP kernels; y2 None: statistics only (scale / shift for a
    consumer that applies them itself); ``res_st``: r2 is the pre-BatchNorm input of that (shortcut)
    BatchNorm, whose scale / shift the apply pass applies to it."""
    bn = st.bn
    C = x2.shape[1]
    rg = x2.shape[0] // st.groups
    C_ = _native.native()
    part = ws.get("bn_part", C_.bn_part_floats(rg, st.groups, C), x2.device)
    track = bn.track_running_stats and bn.running_mean is not None
    tile, st.tile = st.tile, None
    defer = bool(track and ws.defer_running and C_.bn_small(rg) and tile is None)
    C_.gpu_bn_forward(x2, r2, st.groups, bn.weight, bn.bias, float(bn.eps), float(bn.momentum),
                      bn.running_mean if track else None, bn.running_var if track else None,
                      part, st.mean, st.istd, st.scale, st.shift, y2, st.relu and y2 is not None, relu_state, defer,
                      tile_stats=tile[0] if tile is not None else None,
                      tile_m=tile[1] if tile is not None else 0, tile_e=tile[2] if tile is not None else 1,
                      res_scale=res_st.scale if res_st is not None else None,
                      res_shift=res_st.shift if res_st is not None else None)
    if defer:
        ws.running_jobs.append((st.mean, st.istd, bn.running_mean, bn.running_var, rg, float(bn.eps),
                                float(bn.momentum)))


class _GroupedBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, st: BNState, ws: Workspace, join: GradJoin | None = None,
                res_link: ResLink | None = None, out_link: ResLink | None = None, res_st: BNState | None = None):
        n, C, h, w = x.shape
        x2 = rows2d(x)
        r2 = rows2d(res) if res is not None else None
        st.ensure(x.device, torch.float64 if x.dtype == torch.float64 else torch.float32)
        if x.is_cuda:
            if x.dtype not in (torch.bfloat16, torch.float32):
                raise TypeError("grouped BatchNorm on the GPU takes bf16 or fp32 activations")
            y = torch.empty_like(x, memory_format=torch.channels_last)
            # the backward's ReLU test reads one bit per element instead of y
            relu_state = torch.empty((x2.numel() // 8,), dtype=torch.uint8, device=x.device) if st.relu else None
            if res_st is not None:   # the shortcut BatchNorm: statistics only, applied inside this apply pass
                if res is None or res_st.relu:
                    raise ValueError("res_st: a pre-BatchNorm residual without a ReLU of its own")
                res_st.ensure(x.device, torch.float32)
                _bn_forward_gpu(r2, None, res_st, ws, None, None)
            _bn_forward_gpu(x2, r2, st, ws, rows2d(y), relu_state, res_st)
        else:
            if res_st is not None:
                raise ValueError("res_st (a folded shortcut BatchNorm) is a GPU path")
            y = from_rows(_bn_fwd_ref(x2, r2, st), n, h, w)
            relu_state = y if st.relu else None
        ctx.st, ctx.ws, ctx.has_res, ctx.join = st, ws, res is not None, join
        ctx.res_link, ctx.out_link, ctx.res_st = res_link, out_link, res_st
        if out_link is not None and x.is_cuda and not st.relu and LAZY_RES:
            ctx.set_materialize_grads(False)     # the output's gradient may arrive through out_link only
            out_link.ok = True
        ctx.save_for_backward(x, relu_state, res if res_st is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, xs = ctx.saved_tensors            # y: the ReLU state (bit mask on the GPU, y on the CPU) or None
        st, ws = ctx.st, ctx.ws
        n, C, h, w = x.shape
        y2 = (y if y.dim() == 1 else rows2d(y)) if y is not None else None
        if dy is None:                          # a shortcut BatchNorm: dy + ReLU bits through out_link
            m, ctx.out_link.pending = ctx.out_link.pending, None
            if m is None:
                return (None,) * 10
            dy, y2 = m.dy, m.mask               # no ReLU of its own: the bits are its only mask
        dy = _cl(dy)
        x2, dy2 = rows2d(x), rows2d(dy)
        lazy = None
        if x.is_cuda:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            if (ctx.has_res and LAZY_RES and y2 is not None and y2.dim() == 1 and
                    ((ctx.join is not None and ctx.join.lazy) or (ctx.res_link is not None and ctx.res_link.ok))):
                lazy = MaskedGrad(dy, y2)        # the consumer applies the ReLU bits itself
            dres = torch.empty_like(x, memory_format=torch.channels_last) \
                if (ctx.has_res and lazy is None and ctx.res_st is None) else None
            rg = x2.shape[0] // st.groups
            C_ = _native.native()
            part = ws.get("bn_part", C_.bn_part_floats(rg, st.groups, C), x.device)
            coef = ws.get("bn_coef", 3 * st.groups * C, x.device)
            sink, bn = st.sink, st.bn
            grow, stride, og, ob = None, 0, -1, -1
            if sink is not None:
                grow, stride = sink.flat, sink.row_stride
                og = sink.base + sink.offset(bn.weight) if bn.weight is not None else -1
                ob = sink.base + sink.offset(bn.bias) if bn.bias is not None else -1
            dual = False
            if ctx.res_st is not None:           # the folded shortcut BatchNorm: dy + this one's ReLU bits
                rs_, rbn = ctx.res_st, ctx.res_st.bn
                dres = torch.empty_like(xs, memory_format=torch.channels_last)
                ogs = sink.base + sink.offset(rbn.weight) if (sink is not None and rbn.weight is not None) else -1
                obs = sink.base + sink.offset(rbn.bias) if (sink is not None and rbn.bias is not None) else -1
                xs2 = rows2d(xs)
                if BN_DUAL and (y2 is None or y2.dim() == 1):  # one statistics / apply pass for both
                    part_b = ws.get("bn_part2", C_.bn_part_floats(rg, st.groups, C), x.device)
                    coef_b = ws.get("bn_coef2", 3 * st.groups * C, x.device)
                    dual = True
                    C_.gpu_bn_backward_dual(x2, xs2, dy2, y2, st.groups, bn.weight, rbn.weight, st.mean,
                                                   st.istd, rs_.mean, rs_.istd, part, part_b, coef, coef_b,
                                                   rows2d(dx), rows2d(dres), grow, stride, og, ob, ogs, obs)
            if not dual:   # (the two backward calls run in stream order on the same workspaces)
                C_.gpu_bn_backward(x2, dy2, y2, st.groups, bn.weight, st.mean, st.istd, part, coef, rows2d(dx),
                                   rows2d(dres) if (dres is not None and ctx.res_st is None) else None, grow, stride,
                                   og, ob)
                if ctx.res_st is not None:
                    C_.gpu_bn_backward(xs2, dy2, y2, rs_.groups, rbn.weight, rs_.mean, rs_.istd, part, coef,
                                       rows2d(dres), None, grow, stride, ogs, obs)
        else:
            dx2, dr2 = _bn_bwd_ref(x2, dy2, y2, st, ctx.has_res)
            dx = from_rows(dx2, n, h, w)
            dres = from_rows(dr2, n, h, w) if dr2 is not None else None
        if lazy is not None:
            if ctx.join is not None:
                ctx.join.park(lazy)
            else:
                ctx.res_link.pending = lazy     # autograd passes None to the shortcut BatchNorm
        elif dres is not None and ctx.join is not None:
            ctx.join.park(dres)
            dres = None
        return dx, None, None, dres, None, None, None, None, None, None


def grouped_bn(x, st: BNState, ws: Workspace, res=None, res_join: GradJoin | None = None,
               res_link: ResLink | None = None, out_link: ResLink | None = None, res_st: BNState | None = None):
    """y = [relu](BN_per_worker(x) [+ res]); x/res channels_last. With ``res_join``
    the residual's gradient is handed to the join instead of autograd; ``res_link`` / ``out_link``:
    the block's last BatchNorm / its shortcut BatchNorm of one ResLink (see there). ``res_st`` (GPU):
    res is the shortcut convolution's output BEFORE its BatchNorm, which this call folds in (statistics
    pass, then res * scale + shift inside this apply pass; its backward here too): the shortcut's
    normalised activation is never written."""
    return _GroupedBN.apply(_cl(x), st.bn.weight, st.bn.bias, _cl(res) if res is not None else None, st, ws,
                            res_join, res_link, out_link, res_st)


# --------------------------------------------------------------------------- #
# Grouped convolution (per-worker weight gradients)


class ConvSpec:
    def __init__(self, conv: torch.nn.Conv2d, sink: GradSink | None, groups: int):
        if conv.groups != 1 or conv.bias is not None:
            raise ValueError("grouped convolution supports groups=1 convolutions without bias")
        self.conv = conv
        self.sink = sink
        self.groups = groups
        self.kernel = tuple(conv.kernel_size)
        self.stride = tuple(conv.stride)
        self.padding = tuple(conv.padding)
        self.dilation = tuple(conv.dilation)
        self.gemm = (self.kernel == (1, 1) and self.stride == (1, 1) and self.padding == (0, 0)
                     and self.dilation == (1, 1))
        self.bn_next = None       # BNState of the BatchNorm that consumes this convolution's output
        self.wpad = None          # persistent zero-padded [Cout, Kp] weight matrix (im2col + GEMM layers)
        self.wt = None            # [K, Cout] transposed weight matrix of the data-gradient GEMM (refresh_dgrad_weights)
        self.dcol = False         # its data gradient runs dcol = dy · Wmat + col2im (Wmatᵀ refreshed per step)
        self.wd = None            # flipped transposed weight [Cin, Cout, 3, 3] of the halo-kernel data gradient
        self.flip = False         # its data gradient runs on the halo kernel (wd refreshed per step)
        # fp32 step: the weight split into three bf16 pieces [3, Cout, K] and the channel-transposed
        # pieces [3, Cin, KH, KW, Cout] of the data gradient (refresh_f32_weights, once per step)
        self.w3 = self.wt3 = None
        # small-image dense form (SMALL_CONV): (H, W) of its input once chosen, and the per-step expanded
        # weight Wbig [P*Cout, P*Cin] and its transpose (refresh_sc_weights)
        self.sc = None
        self.wbig = self.wbigT = None


def _gemm_nt_ok(a2: torch.Tensor, b2: torch.Tensor) -> bool:
    M, K = a2.shape
    N = b2.shape[0]
    return (a2.is_cuda and a2.dtype == torch.bfloat16 and b2.dtype == torch.bfloat16 and K % 64 == 0
            and N % 64 == 0 and b2.shape[1] == K and a2.is_contiguous() and b2.is_contiguous()
            and M * max(K, N) < 2 ** 31)


# Configuration of each gemm_nt problem, measured once: key (M, N, K, rg or 0, add) -> cfg. The
# step's first (eager) run times every valid tile configuration on the real operands (scratch
# outputs, 3 calls each after a warm call) and keeps the fastest; graph captures and replays
# reuse it (during a capture the static choice of gemm_nt_pick stands in).
_GEMM_CFG: dict = tuning.register("gemm", {})   # (ops/tuning.py: agreed over ranks, checkpointed)


def _gemm_cfg(a2: torch.Tensor, b2: torch.Tensor, rg: int, add: torch.Tensor | None, pro=None) -> int:
    """``pro``: (scale, shift, groups) of a BatchNorm prologue on a2 (only configurations with a
    prologue form are candidates)."""
    C_ = _native.native()
    M, K = a2.shape
    N = b2.shape[0]
    key = (M, N, K, rg, add is not None, pro is not None)
    cfg = _GEMM_CFG.get(key)
    if cfg is not None:
        return cfg

    def pro_ok(c):
        return pro is None or C_.gemm_nt_pro_ok(c, K, M // pro[2], pro[2])

    cands = [c for c in range(C_.gemm_nt_num_cfg())
             if C_.gemm_nt_valid(c, N, K) and (rg == 0 or C_.gemm_nt_stats_rows(c) <= rg) and pro_ok(c)]
    cfg = C_.gemm_nt_pick(M, N, K, rg)
    if cfg >= 0 and not pro_ok(cfg):
        cfg = cands[0] if cands else -1
    if cfg < 0 or torch.cuda.is_current_stream_capturing():
        return cfg
    if not tuning.measuring():   # GARFIELD_TUNING=fixed: the static pick, identical everywhere
        _GEMM_CFG[key] = cfg
        return cfg
    out = torch.empty((M, N), dtype=a2.dtype, device=a2.device)
    addc = add.clone() if add is not None else None
    pkw = {} if pro is None else {"pro_scale": pro[0], "pro_shift": pro[1], "pro_groups": pro[2]}
    # two rounds over the candidates, each candidate's best of its rounds (5 calls after a warm one):
    # a single short sample let clock / cache noise flip near-tied choices from run to run
    times = {}
    for _ in range(2):
        for c in cands:
            st = torch.empty(C_.gemm_nt_stats_geometry(c, M, N, K, rg)[2], device=a2.device) if rg else None
            C_.gpu_gemm_nt(a2, b2, addc if addc is not None else out, addc, st, rg, c, **pkw)   # warm
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(5):
                C_.gpu_gemm_nt(a2, b2, addc if addc is not None else out, addc, st, rg, c, **pkw)
            t1.record()
            t1.synchronize()
            times[c] = min(times.get(c, float("inf")), t0.elapsed_time(t1))
    best = min(cands, key=lambda c: (times[c], c)) if cands else cfg
    _GEMM_CFG[key] = best
    return best


def _gemm_nt_forward(x2: torch.Tensor, w2: torch.Tensor, spec: ConvSpec, pro=None):
    """y = x2 · w2ᵀ on gemm_nt.hip; with ``spec.bn_next`` (the BatchNorm that consumes y, a
    large-layer one) the kernel also writes that BatchNorm's per-worker tile statistics. ``pro``
    ((scale, shift, groups)): x2 is a pre-BatchNorm activation, normalised + ReLU'd by the kernel as
    it stages it. None: use hipBLASLt (never with ``pro``)."""
    if not (GEMM_NT and _gemm_nt_ok(x2, w2)):
        return None
    C_ = _native.native()
    M, K = x2.shape
    N = w2.shape[0]
    st = spec.bn_next
    rg = M // spec.groups
    stats_rg = rg if (st is not None and M % spec.groups == 0 and not C_.bn_small(rg)) else 0
    cfg = _gemm_cfg(x2, w2, stats_rg, None, pro) if stats_rg else -1
    if cfg < 0:
        stats_rg = 0
        cfg = _gemm_cfg(x2, w2, 0, None, pro)
    if cfg < 0:
        return None
    y2 = torch.empty((M, N), dtype=x2.dtype, device=x2.device)
    stats = None
    if stats_rg:
        geo = C_.gemm_nt_stats_geometry(cfg, M, N, K, stats_rg)
        stats = torch.empty(geo[2], dtype=torch.float32, device=x2.device)
    pkw = {} if pro is None else {"pro_scale": pro[0], "pro_shift": pro[1], "pro_groups": pro[2]}
    C_.gpu_gemm_nt(x2, w2, y2, None, stats, stats_rg, cfg, **pkw)
    if stats is not None:
        st.tile = (stats, geo[0], geo[1])
    return y2


def _mm_nt(a2: torch.Tensor, b2: torch.Tensor) -> torch.Tensor:
    """a2 · b2ᵀ: gemm_nt.hip when the shapes fit it, else hipBLASLt."""
    if GEMM_NT and _gemm_nt_ok(a2, b2):
        cfg = _gemm_cfg(a2, b2, 0, None)
        if cfg >= 0:
            out = torch.empty((a2.shape[0], b2.shape[0]), dtype=a2.dtype, device=a2.device)
            _native.native().gpu_gemm_nt(a2, b2, out, None, None, 0, cfg)
            return out
    return torch.mm(a2, b2.t())


def _dcol(dy2: torch.Tensor, w: torch.Tensor, kp: int, spec: "ConvSpec") -> torch.Tensor:
    """dcol = dy2 · Wmat ([rows, Cout] x [Cout, Kp]) for col2im: gemm_nt.hip with the step's Wmatᵀ
    (refresh_dgrad_weights, flagged on first use) when Kp is the unpadded K, else hipBLASLt."""
    K = w.numel() // w.shape[0]
    if GEMM_NT and GEMM_NT_DGRAD and dy2.is_cuda and kp == K and K % 64 == 0 and w.shape[0] % 64 == 0:
        spec.dcol = True
        wt = spec.wt
        if wt is None or wt.shape != (K, w.shape[0]):
            wt = _wmat(w, kp).t().contiguous()
        if _gemm_nt_ok(dy2, wt):
            cfg = _gemm_cfg(dy2, wt, 0, None)
            if cfg >= 0:
                out = torch.empty((dy2.shape[0], K), dtype=dy2.dtype, device=dy2.device)
                _native.native().gpu_gemm_nt(dy2, wt, out, None, None, 0, cfg)
                return out
    return torch.mm(dy2, _wmat(w, kp, spec))


def refresh_dgrad_weights(specs) -> None:
    """Transposed copies Wᵀ [Cin, Cout] of every 1x1 stride-1 convolution weight, for the
    data-gradient GEMMs of this step: ONE launch for the whole network (the weights change
    once per step, in the update kernel), and the flipped transposed weights of the 3x3 layers whose
    data gradient runs on the halo kernel (``spec.flip``), in the same launch."""
    srcs, dsts = [], []
    for spec in specs:
        w = spec.conv.weight
        if spec.flip:
            srcs.append(w.detach())
            dsts.append(_flip_weight_buf(spec))
            continue
        if not (GEMM_NT and GEMM_NT_DGRAD):
            continue
        if not ((spec.gemm or spec.dcol) and w.is_cuda and w.dtype == torch.bfloat16 and w.shape[0] % 64 == 0
                and (w.numel() // w.shape[0]) % 64 == 0 and _channels_last_weight(w)):
            continue
        w2 = w.detach().permute(0, 2, 3, 1).reshape(w.shape[0], -1)   # [Cout, (kh, kw, ci)]: a view
        if not w2.is_contiguous():
            continue
        if spec.wt is None or spec.wt.shape != (w2.shape[1], w2.shape[0]) or spec.wt.device != w2.device:
            spec.wt = torch.empty((w2.shape[1], w2.shape[0]), dtype=w2.dtype, device=w2.device)
        srcs.append(w2)
        dsts.append(spec.wt)
    if srcs:
        _native.native().gpu_transpose_multi(srcs, dsts)


def _flip_weight_buf(spec: "ConvSpec") -> torch.Tensor:
    """The persistent [Cin, Cout, KH, KW] channels_last buffer of spec's flipped transposed weight."""
    w = spec.conv.weight
    shape = (w.shape[1], w.shape[0], w.shape[2], w.shape[3])
    if spec.wd is None or tuple(spec.wd.shape) != shape or spec.wd.device != w.device or spec.wd.dtype != w.dtype:
        spec.wd = torch.empty(shape, dtype=w.dtype, device=w.device).contiguous(memory_format=torch.channels_last)
    return spec.wd


def _halo_dgrad_ok(dy: torch.Tensor, w: torch.Tensor, spec: "ConvSpec") -> bool:
    """The 3x3 / stride-1 / pad-1 data gradient on the halo-staged kernel (conv3x3_nhwc.hip): a forward
    convolution of dy with the flipped transposed weight (refreshed once per step)."""
    return (CONV3X3 and dy.is_cuda and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and spec.kernel == (3, 3) and spec.stride == (1, 1) and spec.padding == (1, 1) and spec.dilation == (1, 1)
            and _channels_last_weight(w)
            and _native.native().conv3x3_pick(dy.shape[0], dy.shape[2], dy.shape[3], w.shape[0], w.shape[1]) > 0)


def _halo_dgrad(dy: torch.Tensor, w: torch.Tensor, spec: "ConvSpec", add: torch.Tensor | None,
                add_mask: torch.Tensor | None = None) -> torch.Tensor | None:
    if not spec.flip or spec.wd is None:       # first use (eager): make the flipped weight now
        spec.flip = True
        _native.native().gpu_transpose_multi([w.detach()], [_flip_weight_buf(spec)])
    return _iconv(dy, spec.wd, (3, 3, 1, 1, 1, 1, 1, 1), (dy.shape[2], dy.shape[3]), add, add_mask=add_mask)


def _gemm_nt_dgrad(dy2: torch.Tensor, w2: torch.Tensor, add: torch.Tensor | None, spec: "ConvSpec | None" = None,
                   add_mask: torch.Tensor | None = None):
    """dx = dy2 · w2 (+ add, in place of add) on gemm_nt.hip with the transposed weight (the step's
    ``spec.wt`` when refreshed, else transposed here); None: use hipBLASLt. ``add_mask``: add is a
    MaskedGrad's dy, counted where its bit is set, and dx is a new tensor."""
    if not (GEMM_NT and GEMM_NT_DGRAD and dy2.is_cuda and w2.shape[1] % 64 == 0):
        return None
    wt = spec.wt if (spec is not None and spec.wt is not None) else w2.t().contiguous()
    if not _gemm_nt_ok(dy2, wt) or (add is not None and not add.is_contiguous()):
        return None
    if add_mask is not None and (add is None or add.shape != (dy2.shape[0], wt.shape[0])):
        return None
    C_ = _native.native()
    cfg = _gemm_cfg(dy2, wt, 0, add)
    if cfg < 0:
        return None
    if add_mask is not None:
        out = torch.empty_like(add)
        C_.gpu_gemm_nt(dy2, wt, out, add, None, 0, cfg, add_mask=add_mask)
        return out
    out = add if add is not None else torch.empty((dy2.shape[0], wt.shape[0]), dtype=dy2.dtype, device=dy2.device)
    C_.gpu_gemm_nt(dy2, wt, out, add, None, 0, cfg)
    return out


def _dcol_dx(dy2: torch.Tensor, w: torch.Tensor, kp: int, spec: "ConvSpec", xshape, add: torch.Tensor | None):
    """dx (+ add, in place of add) = col2im(dy2 · Wmat): the k x k data gradient of any stride."""
    dcol = _dcol(dy2, w, kp, spec)
    if add is not None:
        _native.native().gpu_col2im(dcol, *_geom(spec), add, True)
        return add
    dx = torch.empty(xshape, dtype=dy2.dtype, device=dy2.device, memory_format=torch.channels_last)
    _native.native().gpu_col2im(dcol, *_geom(spec), dx)
    return dx


def _timed(fn, reps: int = 5, rounds: int = 2) -> float:
    """Best of ``rounds`` timings of ``reps`` calls (after a warm call)."""
    fn()
    best = float("inf")
    for _ in range(rounds):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(reps):
            fn()
        t1.record()
        t1.synchronize()
        best = min(best, t0.elapsed_time(t1))
    return best


def _s2_dgrad(dy: torch.Tensor, w: torch.Tensor, spec: "ConvSpec", xshape, add: torch.Tensor | None, kp: int):
    """dx (+ add, in place of add) of a stride-2 convolution on ``gpu_dgrad_s2``: dx's four parity
    classes, each a stride-1 correlation of dy with its taps of the forward weight. None when the
    kernel does not take the geometry, or when the first (eager) call of this shape measured the
    dcol GEMM + col2im faster (then that path runs)."""
    if not (S2_DGRAD and dy.is_cuda and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and spec.stride == (2, 2) and spec.dilation == (1, 1) and _channels_last_weight(w)
            and xshape[2] % 2 == 0 and xshape[3] % 2 == 0 and dy.shape[1] % 64 == 0 and xshape[1] % 64 == 0):
        return None
    C_ = _native.native()
    key = (tuple(dy.shape), tuple(w.shape), tuple(xshape), spec.kernel, spec.padding)
    use = _S2_CHOICE.get(key)
    if use is None:
        probe = torch.empty(xshape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        use = bool(C_.dgrad_s2_ok(dy, probe, *spec.kernel, *spec.padding))
        if use and not S2_FORCE and not torch.cuda.is_current_stream_capturing() and tuning.measuring():
            dflag = spec.dcol
            t_s2 = _timed(lambda: C_.gpu_dgrad_s2(dy, w, *spec.kernel, *spec.padding, probe))
            t_col = _timed(lambda: _dcol_dx(rows2d(dy), w, kp, spec, xshape, None))
            use = t_s2 < t_col
            spec.dcol = dflag or not use
        _S2_CHOICE[key] = use
    if not use:
        return None
    dx = add if add is not None else torch.empty(xshape, dtype=dy.dtype, device=dy.device,
                                                 memory_format=torch.channels_last)
    C_.gpu_dgrad_s2(dy, w, *spec.kernel, *spec.padding, dx, add)
    return dx


def _sc_ok(x: torch.Tensor, w: torch.Tensor, spec: "ConvSpec") -> bool:
    return (SMALL_CONV and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and spec.kernel == (3, 3) and spec.stride == (1, 1) and spec.padding == (1, 1) and spec.dilation == (1, 1)
            and x.shape[2] <= 2 and x.shape[3] <= 2 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and _channels_last_weight(w) and GEMM_NT)


def _sc_buffers(spec: "ConvSpec", h: int, wd: int) -> None:
    w = spec.conv.weight
    P = h * wd
    shape = (P * w.shape[0], P * w.shape[1])
    if spec.wbig is None or tuple(spec.wbig.shape) != shape or spec.wbig.device != w.device:
        spec.wbig = torch.empty(shape, dtype=w.dtype, device=w.device)
        spec.wbigT = torch.empty((shape[1], shape[0]), dtype=w.dtype, device=w.device)
    spec.sc = (h, wd)


def refresh_sc_weights(specs) -> None:
    """Wbig and Wbigᵀ of every small-image layer (``spec.sc``) from this step's weights: ONE launch."""
    ws, hs, wds, bigs, bigTs = [], [], [], [], []
    for spec in specs:
        if spec.sc is None:
            continue
        ws.append(spec.conv.weight.detach())
        hs.append(spec.sc[0])
        wds.append(spec.sc[1])
        bigs.append(spec.wbig)
        bigTs.append(spec.wbigT)
    if ws:
        _native.native().gpu_sc_expand(ws, hs, wds, bigs, bigTs)


def _sc_rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> its [N, H*W*C] row matrix (a view)."""
    return t.permute(0, 2, 3, 1).reshape(t.shape[0], -1)


def _sc_gemm(a2: torch.Tensor, b2: torch.Tensor, add: torch.Tensor | None) -> torch.Tensor:
    C_ = _native.native()
    cfg = _gemm_cfg(a2, b2, 0, add)
    if cfg < 0:
        raise RuntimeError(f"gemm_nt has no configuration for the small-image GEMM {tuple(a2.shape)} x {tuple(b2.shape)}")
    out = add if add is not None else torch.empty((a2.shape[0], b2.shape[0]), dtype=a2.dtype, device=a2.device)
    C_.gpu_gemm_nt(a2, b2, out, add, None, 0, cfg)
    return out


_SC_WG_CHOICE: dict = tuning.register("scwg", {})   # (x shape, dy shape, G) -> the dense form (else the implicit 3x3 kernel)
SC_DENSE_WGRAD = None      # tests: True / False force the dense / implicit form (None: measured)


def _sc_wgrad(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int) -> None:
    """Per-worker weight gradient of a small-image layer: the dense dWbig (1x1 implicit kernel over the
    [N, P*C] rows, folded onto the taps) or the implicit 3x3 kernel, whichever the first eager call of the
    shape measured faster (the dense form writes P^2 blocks of fp32 slabs; the implicit one computes the
    out-of-image taps)."""
    key = (tuple(x.shape), tuple(dy.shape), G)
    dense = _SC_WG_CHOICE.get(key) if SC_DENSE_WGRAD is None else SC_DENSE_WGRAD
    if dense is None:
        dense = True
        if not torch.cuda.is_current_stream_capturing() and tuning.measuring() and _iwgrad_ok(x, dy):
            sink = spec.sink
            spec.sink = _NullSink(sink, G)
            try:
                t_dense = _timed(lambda: _sc_wgrad_dense(x, dy, spec, G))
                t_imp = _timed(lambda: _iwgrad(x, dy, spec, G, 9 * x.shape[1]))
            finally:
                spec.sink = sink
            dense = t_dense <= t_imp
        _SC_WG_CHOICE[key] = dense
    if dense:
        _sc_wgrad_dense(x, dy, spec, G)
    else:
        _iwgrad(x, dy, spec, G, 9 * x.shape[1])


class _NullSink:
    """A GradSink stand-in for timing runs: rows views and queued sums land in scratch tensors."""

    def __init__(self, sink, groups: int):
        self.flat = sink.flat
        self.groups = groups

    def rows_view(self, p, shape, dtype):
        return torch.empty((self.groups, *shape), dtype=dtype, device=p.device)

    def queue_split(self, part, out):
        _native.native().gpu_split_reduce(part, out)

    def put_groups(self, p, grads):
        pass


def _sc_wgrad_dense(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int) -> None:
    n, cin, h, wd = x.shape
    cout = dy.shape[1]
    P = h * wd
    xv = _sc_rows(x).view(n, 1, 1, P * cin).permute(0, 3, 1, 2)
    dv = _sc_rows(dy).view(n, 1, 1, P * cout).permute(0, 3, 1, 2)
    C_ = _native.native()
    S = _iwgrad_splits(n // G, (P * cin // 64) * (P * cout // 64) * G // C_.iwgrad_taps_per_block(1, 1, P * cin, P * cout))
    slab = torch.empty((S, G, P * cout, P * cin), dtype=torch.float32, device=dy.device)
    C_.gpu_iwgrad(xv, dv, 1, 1, 1, 1, 0, 0, 1, 1, G, slab, S)
    out = spec.sink.rows_view(spec.conv.weight, (cout, 9 * cin), spec.sink.flat.dtype)
    if out is not None and spec.sink.flat.dtype in (torch.bfloat16, torch.float32):
        C_.gpu_sc_fold(slab, h, wd, out)
        return
    tmp = torch.empty((G, cout, 9 * cin), dtype=torch.float32, device=dy.device)
    C_.gpu_sc_fold(slab, h, wd, tmp)
    spec.sink.put_groups(spec.conv.weight, tmp)


def _conv_bwd(dy, x, w, spec: ConvSpec, mask):
    return torch.ops.aten.convolution_backward(dy, x, w, None, list(spec.stride), list(spec.padding),
                                               list(spec.dilation), False, [0, 0], 1, mask)


def _out_hw(spec: ConvSpec, h: int, w: int):
    (kh, kw), (sh, sw), (ph, pw), (dh, dw) = spec.kernel, spec.stride, spec.padding, spec.dilation
    return (h + 2 * ph - dh * (kh - 1) - 1) // sh + 1, (w + 2 * pw - dw * (kw - 1) - 1) // sw + 1


def _geom(spec: ConvSpec):
    return (*spec.kernel, *spec.stride, *spec.padding, *spec.dilation)


def _im2col(x: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    """[N*Ho*Wo, Kp] bf16 col (Kp = KH*KW*C rounded up to 8, pad columns zero)."""
    n, c, h, w = x.shape
    ho, wo = _out_hw(spec, h, w)
    K = spec.kernel[0] * spec.kernel[1] * c
    col = torch.empty((n * ho * wo, (K + 7) // 8 * 8), dtype=x.dtype, device=x.device)
    _native.native().gpu_im2col(x, *_geom(spec), col)
    return col


def _wmat(w: torch.Tensor, kp: int, spec: "ConvSpec | None" = None) -> torch.Tensor:
    """channels_last weight [Cout, Cin, KH, KW] -> [Cout, Kp] in (kh, kw, ci) column order. With
    ``spec``, zero padding columns live in a persistent buffer and only the weight is copied
    (one kernel instead of a fill + a copy per call)."""
    w2 = w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)
    if kp == w2.shape[1]:
        return w2
    if spec is None:
        return F.pad(w2, (0, kp - w2.shape[1]))
    buf = spec.wpad
    if buf is None or buf.shape != (w2.shape[0], kp) or buf.dtype != w2.dtype or buf.device != w2.device:
        buf = spec.wpad = torch.zeros((w2.shape[0], kp), dtype=w2.dtype, device=w2.device)
    buf[:, :w2.shape[1]].copy_(w2)
    return buf


def _iconv_ok(x: torch.Tensor, w: torch.Tensor, rows: int) -> bool:
    """Use the implicit-GEMM MFMA kernel (its LDS-staged form: C % 64, Cout % 64) when
    it has enough workgroups to fill the chip. Measured on the step's 3x3 shapes
    (scripts/bench_iconv.py, profiles/bench_iconv_r1.log): layer1 23.9 vs 73.8 µs for
    im2col + hipBLASLt, layer2 24.4 vs 42.3, layer3 30.5 vs 41.2; layer4 (2000 output
    pixels, 256 workgroups over a 4608-deep reduction) stays on im2col + GEMM, 48 vs 33."""
    return (ICONV and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and -(-rows // 64) * (w.shape[0] // 64) >= _ICONV_MINWG)


_ICONV_MINWG = 400   # workgroups (profiles/bench_iconv_r1.log)


def _iconv(x: torch.Tensor, w: torch.Tensor, geom, out_hw, add: torch.Tensor | None = None,
           transpose_w: bool = False, add_mask: torch.Tensor | None = None) -> torch.Tensor | None:
    """y = conv(x, w) (+ add, written in place of add when given) on the MFMA kernel;
    ``transpose_w``: w is a forward weight and its flipped transpose is applied (dgrad). ``add_mask``
    (a MaskedGrad's ReLU bits): add counts where its bit is set and y is a new tensor; None when the
    halo-staged kernel (the only one with the masked epilogue) does not take the shape."""
    n = x.shape[0]
    cout = w.shape[1] if transpose_w else w.shape[0]
    if add is not None and add_mask is None:
        y = add
    else:
        y = torch.empty((n, cout, *out_hw), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    if add_mask is not None:
        return y if _native.native().gpu_iconv(x, w, *geom, y, add, 0, transpose_w, add_mask=add_mask) else None
    _native.native().gpu_iconv(x, w, *geom, y, add, 0, transpose_w)
    return y


def _iwgrad_ok(x: torch.Tensor, dy: torch.Tensor) -> bool:
    return (IWGRAD and x.is_cuda and x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16
            and x.shape[1] % 64 == 0 and dy.shape[1] % 64 == 0)


def _iwgrad_splits(rows_per_worker: int, tiles: int) -> int:
    """Pixel splits of the implicit weight gradient: about ``_IWGRAD_WG`` workgroups to fill the
    chip, each split at least ``_IWGRAD_MINPIX`` pixels."""
    S = 1
    while S < _IWGRAD_MAXS and tiles * S < _IWGRAD_WG and rows_per_worker // (2 * S) >= _IWGRAD_MINPIX:
        S *= 2
    return S


def _wgrad3x3_splits(rows_per_worker: int, blocks: int) -> int:
    """Pixel splits of the halo-staged 3x3 weight gradient (one workgroup per (64 co, 64 ci) block,
    worker and split, all nine taps): about one workgroup per CU, each split at least ``_WGRAD3_MINTILES`` 128-pixel tiles."""
    tiles = -(-rows_per_worker // 128)
    S = 1
    while S < 64 and blocks * S < _WGRAD3_WG and tiles // (2 * S) >= _WGRAD3_MINTILES:
        S *= 2
    return S


# at least three 128-pixel tiles per split: on ResNet-50's small 3x3 layers (8x8 and 4x4, 125 and
# 32 tiles per worker) the slab traffic (each split writes a [G, cout, K] fp32 slab, read back by
# the deferred sum) weighs more than the extra workgroups; ResNet-18's larger layers keep their
# splits (profiles/r4/splits/: ResNet-50 6.17-6.20 -> 6.11-6.13 ms/step together with
# _IWGRAD_MINPIX 256 -> 512; ResNet-18 unchanged, while a 256-workgroup target costs it 0.8 ms)
_WGRAD3_WG = 512
_WGRAD3_MINTILES = 3


# profiles/iwgrad_split_sweep_r1.log; 512 since the 1x1 layers joined the implicit kernel
# (profiles/r2/iwgrad_wg_nt_sweep.log)
_IWGRAD_WG = 512
_IWGRAD_MINPIX = 512
_IWGRAD_MAXS = 64   # ImageNet-size rows: more than 16 splits fill the chip (profiles/r4/splits/in_*: 177.8 -> 177.1 ms)


def _iwgrad(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int, K: int, pro=None) -> None:
    """Per-worker weight gradients of an iconv-mode convolution without an im2col matrix
    (``gpu_iwgrad``): written straight into the exchange rows when one pass covers every
    worker's pixels, else as fp32 split slabs summed into the sink. ``pro`` ((scale, shift), 1x1
    only): x is a pre-BatchNorm activation normalised + ReLU'd in the kernel."""
    pkw = {} if pro is None else {"pro_scale": pro[0], "pro_shift": pro[1]}
    cout = dy.shape[1]
    rows = dy.shape[0] * dy.shape[2] * dy.shape[3] // G
    C_ = _native.native()
    if (CONV3X3 and spec.kernel == (3, 3) and spec.stride == (1, 1) and spec.padding == (1, 1)
            and spec.dilation == (1, 1) and C_.wgrad3x3_fits(x.shape[0], x.shape[2], x.shape[3], x.shape[1], cout, G)):
        S = _wgrad3x3_splits(rows, (x.shape[1] // 64) * (cout // 64) * G)
    else:
        S = _iwgrad_splits(rows, (K // 64) * (cout // 64) * G //
                          C_.iwgrad_taps_per_block(spec.kernel[1], spec.kernel[0], x.shape[1], cout))
    out = spec.sink.rows_view(spec.conv.weight, (cout, K), dy.dtype) if S == 1 else None
    if out is not None:
        C_.gpu_iwgrad(x, dy, *_geom(spec), G, out, 1, **pkw)
        return
    part = torch.empty((S, G, cout, K), dtype=torch.float32, device=dy.device)
    C_.gpu_iwgrad(x, dy, *_geom(spec), G, part, S, **pkw)
    rows = spec.sink.rows_view(spec.conv.weight, (cout, K), spec.sink.flat.dtype)
    if rows is not None:     # the S slabs summed straight into the exchange rows (deferred, batched)
        spec.sink.queue_split(part, rows)
    else:
        spec.sink.put_groups(spec.conv.weight, part.sum(0) if S > 1 else part[0])


def _stem_kind(w: torch.Tensor, spec: "ConvSpec") -> int | None:
    """stem_nhwc.hip's geometry of a 3 -> 64-channel first layer: 0 the 7x7/2/pad-3 ResNet stem, 1 the
    CIFAR ResNet-18 3x3/1/pad-1 one; None for anything else."""
    if spec.dilation != (1, 1):
        return None
    if tuple(w.shape) == (64, 3, 7, 7) and spec.stride == (2, 2) and spec.padding == (3, 3):
        return 0
    if tuple(w.shape) == (64, 3, 3, 3) and spec.stride == (1, 1) and spec.padding == (1, 1):
        return 1
    return None


def _stem_ok(x: torch.Tensor, w: torch.Tensor, spec: "ConvSpec") -> bool:
    """A 3-channel stem into 64 channels (``_stem_kind``), bf16 channels_last, on sizes whose staged
    input rows fit the kernels' LDS (every CIFAR/ImageNet-crop size)."""
    kind = _stem_kind(w, spec)
    return (STEM and kind is not None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and _channels_last_weight(w) and x.is_contiguous(memory_format=torch.channels_last)
            and _native.native().stem_supported(x.shape[2], x.shape[3], kind))


def _stem_wgrad(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int) -> None:
    """Per-worker stem weight gradients (``gpu_stem_wgrad``): fp32 slabs of image slices,
    summed into the exchange rows by the deferred split-K reduction."""
    per = x.shape[0] // G
    # large images (ImageNet crops: 12544 output pixels each) take twice the workgroups: one image
    # per slice still amortises the band staging (profiles/r4/splits/inst_*: 179.6 -> 178.7 ms),
    # while CIFAR-size images keep ~2 images per slice (splits/stc_*: 2048 costs 0.03 ms there)
    wg = _STEM_WG * (2 if dy.shape[2] * dy.shape[3] > 4096 else 1)
    S = max(1, min(per, -(-wg // G)))
    C_ = _native.native()
    kind = _stem_kind(spec.conv.weight, spec) or 0
    K = C_.stem_k(kind)
    part = torch.empty((S, G, 64, K), dtype=torch.float32, device=dy.device)
    C_.gpu_stem_wgrad(x, dy, G, part, kind)
    rows = spec.sink.rows_view(spec.conv.weight, (64, K), spec.sink.flat.dtype)
    if rows is not None:
        spec.sink.queue_split(part, rows)
    else:
        spec.sink.put_groups(spec.conv.weight, part.sum(0))


def _dgrad_weight_shape(w: torch.Tensor) -> torch.Tensor:
    """A meta tensor shaped like ``_dgrad_weight(w)`` (for the kernel-choice test)."""
    return torch.empty((w.shape[1], w.shape[0], w.shape[2], w.shape[3]), dtype=w.dtype, device="meta")


def _dgrad_weight(w: torch.Tensor) -> torch.Tensor:
    """W'[ci, i', j', co] = W[co, KH-1-i', KW-1-j', ci] as a channels_last [Cin, Cout, KH, KW] tensor: the
    data gradient of a stride-1 convolution is the convolution of dy with W'."""
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


def _channels_last_weight(w: torch.Tensor) -> bool:
    return w.dim() == 4 and w.is_contiguous(memory_format=torch.channels_last)


def _match_layout(g: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    """A dense copy/view of gradient g with the same memory order as parameter p."""
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
        return g.contiguous(memory_format=torch.channels_last)
    return g.contiguous()


def _wgrad(dy2: torch.Tensor, a2: torch.Tensor, G: int, out: torch.Tensor | None = None,
           sink: "GradSink | None" = None) -> torch.Tensor:
    """Per-worker weight gradients ``dW_g = dy_gᵀ · a_g`` for all G workers: [G, Cout, K].

    One strided-batched GEMM; when each worker has many rows (the CIFAR stem and
    layer1: 16k-64k rows against 64 output channels) the row dimension is split S
    ways into a (G*S)-batch GEMM and the S partials are summed in fp32: the
    reduction is too long and the output too small for one GEMM to fill 256 CUs
    (measured 1.6-3.7x faster on those layers, scripts/bench_wgrad_gemm.py).
    ``out`` ([G, Cout, K], e.g. ``GradSink.rows_view``) receives the result in place:
    the GEMM (or the fp32-accumulated split-K sum) writes the exchange rows directly."""
    cout, K = dy2.shape[1], a2.shape[1]
    M = dy2.shape[0] // G
    S = 1
    # layer2-size reductions (4000 rows) still gain from S=4: 21.6 vs 28.3 µs for 128>512
    # (scripts/bench_wgrad_1x1.py, profiles/bench_wgrad_1x1_r1.log); 1000 rows lose
    while S < 16 and M % (2 * S) == 0 and (M // (2 * S) >= 4000 or (S < 4 and M // (2 * S) >= 1000)):
        S *= 2
    Ko = out.shape[-1] if out is not None else K          # out may drop padding columns (K >= Ko)
    if S == 1 and Ko == K:
        if out is not None:
            return torch.bmm(dy2.view(G, M, cout).transpose(1, 2), a2.view(G, M, K), out=out)
        return torch.bmm(dy2.view(G, M, cout).transpose(1, 2), a2.view(G, M, K))
    if dy2.is_cuda and out is not None and dy2.dtype in (torch.bfloat16, torch.float16):
        # fp32 partials (no per-split rounding), summed (and cropped to Ko columns) into the
        # exchange rows by one launch
        part = torch.bmm(dy2.view(G * S, M // S, cout).transpose(1, 2), a2.view(G * S, M // S, K),
                         out_dtype=torch.float32)
        red = part.view(G, S, cout, K).transpose(0, 1)[..., :Ko]
        if sink is not None:
            sink.queue_split(red, out)
        else:
            _native.native().gpu_split_reduce(red, out)
        return out
    part = torch.bmm(dy2.view(G * S, M // S, cout).transpose(1, 2), a2.view(G * S, M // S, K))
    if out is not None:
        return torch.sum(part.view(G, S, cout, K)[..., :Ko], 1, out=out)   # fp32 accumulation, one rounding
    return part.view(G, S, cout, K).float().sum(1)


# --------------------------------------------------------------------------- #
# fp32 (reference-precision) convolutions: conv_f32.hip / stem_nhwc.hip on split-bf16 MFMA


def _stem_shape(w: torch.Tensor, spec: "ConvSpec") -> bool:
    return (tuple(w.shape) == (64, 3, 7, 7) and spec.stride == (2, 2) and spec.padding == (3, 3)
            and spec.dilation == (1, 1))


def _f32_conv_ok(x: torch.Tensor, w: torch.Tensor, spec: "ConvSpec") -> bool:
    """The fp32 step's own kernels take this convolution (raises on a GPU shape they cannot:
    the fp32 grouped step never falls back to a library convolution)."""
    if not (x.is_cuda and x.dtype == torch.float32):
        return False
    if _stem_shape(w, spec) and _native.native().stem_supported(x.shape[2], x.shape[3]):
        return True
    if w.shape[0] % 64 or (w.shape[1] % 64 and w.shape[1] % 32 == 0):
        raise ValueError(f"fp32 grouped convolution: no kernel for {tuple(w.shape)} (Cout % 64; Cin % 64 or a "
                         f"gathered Cin % 32 != 0)")
    return True


def _gathered(w: torch.Tensor) -> bool:
    """Input channels the fp32 kernels gather one element at a time (e.g. a 3-channel first layer):
    the split weight rows are the flattened (tap, channel) index padded to a multiple of 32."""
    return w.shape[1] % 32 != 0


def refresh_f32_weights(specs) -> None:
    """The fp32 step's per-step weight split, ONE launch for the whole network: every convolution
    weight W (fp32, channels_last) -> its bf16 pieces W0 = bf16(W), W1 = bf16(W - W0), W2 =
    bf16(W - W0 - W1) [3, Cout, K] and the channel-transposed pieces [3, Cin, KH, KW, Cout] its data
    gradient multiplies by; the stem's pieces are zero-padded [64, 160] matrices (stem_nhwc.hip)."""
    jobs = []
    for spec in specs:
        w = spec.conv.weight
        if not (w.is_cuda and w.dtype == torch.float32):
            continue
        if not _channels_last_weight(w):
            raise ValueError("fp32 grouped convolution: the weight must be channels_last")
        cout, cin, kh, kw = w.shape
        wd = w.detach()
        if _stem_shape(w, spec):
            if spec.w3 is None or spec.w3.device != w.device:
                spec.w3 = torch.zeros((3, 64, 160), dtype=torch.bfloat16, device=w.device)
            jobs.append((wd, spec.w3, None, 64, 1, 147, 160))
            continue
        K = kh * kw * cin
        if _gathered(w):   # a first layer (its data gradient is never taken): padded rows, no transposed pieces
            kp = (K + 31) // 32 * 32
            if spec.w3 is None or spec.w3.shape != (3, cout, kp) or spec.w3.device != w.device:
                spec.w3 = torch.zeros((3, cout, kp), dtype=torch.bfloat16, device=w.device)
            jobs.append((wd, spec.w3, None, cout, 1, K, kp))
            continue
        if spec.w3 is None or spec.w3.shape != (3, cout, K) or spec.w3.device != w.device:
            spec.w3 = torch.empty((3, cout, K), dtype=torch.bfloat16, device=w.device)
            spec.wt3 = torch.empty((3, cin, kh * kw * cout), dtype=torch.bfloat16, device=w.device)
        jobs.append((wd, spec.w3, spec.wt3, cout, kh * kw, cin, 0))
    if jobs:
        _native.native().gpu_wsplit_multi(jobs)


# Kernel form of each fp32 convolution (forward or data gradient), measured once like the gemm_nt tiles:
# key (dgrad, src shape, out shape, geometry, add) -> (pm, ksplit) of gpu_conv_f32 (pm 11..15: pixel
# fragments per wave 1 / 2 / 2 / 4 / 4 with a 3 / 3 / 2 / 2 / 3-deep ring; ksplit > 1: split-K slabs
# summed by a second pass). The static choice (pm 0: 2 fragments, 2-deep ring, split-K below 400 tiles)
# is one of the candidates, so measuring never picks a slower form than it, up to the timing noise.
_F32_CONV_CFG: dict = tuning.register("f32conv", {})
_F32_CONV_CANDS = [(pm, 1) for pm in (11, 12, 13, 14, 15)] + [(pm, S) for S in (2, 4, 8) for pm in (13, 14, 15)]


def _f32_conv_cfg(src: torch.Tensor, w3: torch.Tensor, spec: "ConvSpec", dgrad: bool, out: torch.Tensor,
                  add: torch.Tensor | None) -> tuple:
    key = (bool(dgrad), tuple(src.shape), tuple(out.shape), _geom(spec), add is not None)
    cfg = _F32_CONV_CFG.get(key)
    if cfg is not None:
        return tuple(cfg)
    if torch.cuda.is_current_stream_capturing():
        return (0, 0)
    if not tuning.measuring():
        _F32_CONV_CFG[key] = (0, 0)
        return (0, 0)
    C_ = _native.native()
    scratch = torch.empty_like(out)
    addc = add.clone() if add is not None else None
    best, best_t = (0, 0), _timed(lambda: C_.gpu_conv_f32(src, w3, *_geom(spec), dgrad, scratch, addc))
    for pm, S in _F32_CONV_CANDS:
        t = _timed(lambda: C_.gpu_conv_f32(src, w3, *_geom(spec), dgrad, scratch, addc, pm, S))
        if t < best_t:
            best, best_t = (pm, S), t
    _F32_CONV_CFG[key] = best
    return best


def _f32_forward(x: torch.Tensor, w: torch.Tensor, spec: "ConvSpec") -> torch.Tensor:
    if spec.w3 is None:
        refresh_f32_weights([spec])
    n, _, h, wd = x.shape
    ho, wo = _out_hw(spec, h, wd)
    y = torch.empty((n, w.shape[0], ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
    if _stem_shape(w, spec):
        _native.native().gpu_stem_fwd(x, spec.w3, y)
    else:
        pm, S = _f32_conv_cfg(x, spec.w3, spec, False, y, None)
        _native.native().gpu_conv_f32(x, spec.w3, *_geom(spec), False, y, None, pm, S)
    return y


def _f32_dgrad(dy: torch.Tensor, w: torch.Tensor, spec: "ConvSpec", xshape, add: torch.Tensor | None):
    """dx (+ add, written in place of add) of an fp32 convolution, any stride."""
    dx = add if add is not None else torch.empty(xshape, dtype=dy.dtype, device=dy.device,
                                                 memory_format=torch.channels_last)
    pm, S = _f32_conv_cfg(dy, spec.wt3, spec, True, dx, add)
    _native.native().gpu_conv_f32(dy, spec.wt3, *_geom(spec), True, dx, add, pm, S)
    return dx


# pixel splits of the fp32 weight gradients: up to ~1024 workgroups (two per CU), each split
# >= 250 pixels: the measured optimum on the ResNet-50 CIFAR shapes (scripts/bench_conv_f32.py,
# profiles/r4/bench_conv_f32.log)
_F32_WGRAD_WG = 1024
_F32_WGRAD_MINPIX = 250


# (pixel splits, kernel form) of each fp32 weight gradient, measured once (ops/tuning.py): key (x shape, dy
# shape, geometry, groups) -> (S, variant: 2 the 128 x 128 tile, 3 the 64 x 64 one). A split's cost counts
# its share of the deferred slab sum (S slabs read, one row written, at the split-K sum's ~4.5 TB/s);
# the static choice (up to ~1024 workgroups, >= 250 pixels per split) is a candidate.
_F32_WGRAD_CFG: dict = tuning.register("f32wgrad", {})


def _f32_wgrad_static(x: torch.Tensor, dy: torch.Tensor, G: int, cout: int, K: int) -> int:
    rows = dy.shape[0] * dy.shape[2] * dy.shape[3] // G
    tile = 128 if (x.shape[1] % 128 == 0 and cout % 128 == 0) else 64   # conv_f32.hip: the wide form
    tiles = -(-K // tile) * (cout // tile) * G
    S = 1
    while S < 16 and tiles * S < _F32_WGRAD_WG and rows // (2 * S) >= _F32_WGRAD_MINPIX:
        S *= 2
    return S


def _f32_wgrad_cfg(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int, cout: int, K: int) -> tuple:
    key = (tuple(x.shape), tuple(dy.shape), _geom(spec), G)
    cfg = _F32_WGRAD_CFG.get(key)
    if cfg is not None:
        return tuple(cfg)
    static = (_f32_wgrad_static(x, dy, G, cout, K), 0)
    if torch.cuda.is_current_stream_capturing():
        return static
    if not tuning.measuring():
        _F32_WGRAD_CFG[key] = static
        return static
    C_ = _native.native()
    rows = dy.shape[0] * dy.shape[2] * dy.shape[3] // G
    wide = x.shape[1] % 128 == 0 and cout % 128 == 0
    variants = (2, 3) if wide else (3,)
    cands = [(S, v) for S in (1, 2, 4, 8, 16) if S == 1 or rows // S >= 64 for v in variants]
    slab = G * cout * K * 4
    best, best_t = None, float("inf")
    for S, v in cands:
        part = torch.empty((S, G, cout, K), dtype=torch.float32, device=dy.device)
        t = _timed(lambda: C_.gpu_wgrad_f32(x, dy, *_geom(spec), G, part, S, v)) / 5.0
        if S > 1:
            t += (S + 1) * slab / 4.5e9   # ms: the deferred sum of the S slabs into the row
        if t < best_t:
            best, best_t = (S, v), t
        del part
    _F32_WGRAD_CFG[key] = best
    return best


def _f32_wgrad(x: torch.Tensor, dy: torch.Tensor, spec: "ConvSpec", G: int) -> None:
    """Per-worker fp32 weight gradients straight into the (fp32) exchange rows, or as split
    slabs summed there by the deferred split-K reduction."""
    C_ = _native.native()
    w = spec.conv.weight
    if _stem_shape(w, spec):
        _stem_wgrad(x, dy, spec, G)
        return
    cout = dy.shape[1]
    K = w.numel() // cout
    S, var = _f32_wgrad_cfg(x, dy, spec, G, cout, K)
    out = spec.sink.rows_view(w, (cout, K), torch.float32) if S == 1 else None
    if out is not None:
        C_.gpu_wgrad_f32(x, dy, *_geom(spec), G, out, 1, var)
        return
    part = torch.empty((S, G, cout, K), dtype=torch.float32, device=dy.device)
    C_.gpu_wgrad_f32(x, dy, *_geom(spec), G, part, S, var)
    rows_v = spec.sink.rows_view(w, (cout, K), spec.sink.flat.dtype)
    if rows_v is not None:
        spec.sink.queue_split(part, rows_v)
    else:
        spec.sink.put_groups(w, part.sum(0))


class _GroupedConv(torch.autograd.Function):
    """Convolution over the grouped batch with per-worker weight gradients.

    GPU, k x k kernels: implicit-GEMM / halo-staged MFMA kernels, or im2col -> GEMMs ->
    col2im (im2col_nhwc.hip); the forward's col is kept for the weight gradient.
    1x1 stride-1 kernels are plain GEMMs on the NHWC rows. CPU (and
    shapes no kernel takes): ATen convolutions, per-worker weight gradients. fp32 activations take
    the fp32 kernels (conv_f32.hip)."""

    @staticmethod
    def forward(ctx, x, w, spec: ConvSpec, join: GradJoin | None = None):
        ctx.spec = spec
        ctx.join = join
        ctx.xshape = tuple(x.shape)
        n, _, h, wd = x.shape
        if _f32_conv_ok(x, w, spec):
            ctx.mode = "f32"
            ctx.save_for_backward(x, w)
            return _f32_forward(x, w, spec)
        if spec.gemm:
            ctx.mode = "rows"
            ctx.save_for_backward(x, w)
            if join is not None and x.is_cuda:
                join.lazy = True                 # the backward's GEMM takes the other branch's MaskedGrad
            y2 = _gemm_nt_forward(rows2d(x), w.reshape(w.shape[0], -1), spec)
            if y2 is None:
                y2 = torch.mm(rows2d(x), w.reshape(w.shape[0], -1).t())
            return from_rows(y2, n, h, wd)
        if _sc_ok(x, w, spec):
            ctx.mode = "sc"
            ctx.save_for_backward(x, w)
            if spec.sc != (h, wd) or spec.wbig is None:   # first use (eager): expand now; later steps refresh
                _sc_buffers(spec, h, wd)
                refresh_sc_weights([spec])
            y2 = _sc_gemm(_sc_rows(x), spec.wbig, None)
            return y2.view(n, h, wd, -1).permute(0, 3, 1, 2)
        if _stem_ok(x, w, spec):
            ctx.mode = "stem"
            ctx.save_for_backward(x, w)
            ho, wo = _out_hw(spec, h, wd)
            y = torch.empty((n, 64, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            C_ = _native.native()
            kind = _stem_kind(w, spec)
            # the consuming BatchNorm's statistics from the kernel's epilogue (whole-image tiles): no partial pass
            st, stats = spec.bn_next, None
            if st is not None and kind == 0 and n % spec.groups == 0 and not C_.bn_small(n // spec.groups * ho * wo):
                tiles = C_.stem_fwd_stat_tiles(n, h, wd, 0)
                if tiles:
                    stats = torch.empty(tiles * 2 * 3 * 64, dtype=torch.float32, device=x.device)
            C_.gpu_stem_fwd(x, w, y, kind, stats)   # the weight is padded while staged
            if stats is not None:
                st.tile = (stats, 256, 1)
            return y
        if _channels_last_weight(w) and _iconv_ok(x, w, n * math.prod(_out_hw(spec, h, wd))):
            ctx.mode = "iconv"
            ctx.save_for_backward(x, w)
            y = _iconv(x, w, _geom(spec), _out_hw(spec, h, wd))
            if join is not None and _halo_dgrad_ok(y, w, spec):
                join.lazy = True                 # the halo-staged dgrad takes the other branch's MaskedGrad
            return y
        if x.is_cuda and _channels_last_weight(w):
            ctx.mode = "col"
            col = _im2col(x, spec)
            ho, wo = _out_hw(spec, h, wd)
            y = from_rows(_mm_nt(col, _wmat(w, col.shape[1], spec)), n, ho, wo)
            ctx.save_for_backward(col, w)
            ctx.x = x if (spec.sink is not None and _iwgrad_ok(x, y)) else None   # implicit weight gradient
            return y
        ctx.mode = "aten"
        ctx.save_for_backward(x, w)
        return _cl(F.conv2d(x, w, None, spec.stride, spec.padding, spec.dilation))

    @staticmethod
    def backward(ctx, dy):
        a, w = ctx.saved_tensors
        spec, mode = ctx.spec, ctx.mode
        dy = _cl(dy)
        G = spec.groups
        cout = dy.shape[1]
        dy2 = rows2d(dy)
        n, cin, h, wd = ctx.xshape
        dx = None
        need_dx = ctx.needs_input_grad[0]
        prev = ctx.join.take() if (need_dx and ctx.join is not None) else None
        first = need_dx and ctx.join is not None and prev is None   # park dx for the other branch
        if isinstance(prev, MaskedGrad) and mode not in ("rows", "iconv"):
            prev = prev.materialize()
        if mode == "f32":                        # a = x
            if need_dx:
                if _stem_shape(w, spec) or _gathered(w):   # a first layer: dx of the input, never wanted in training
                    dx = _cl(_conv_bwd(dy, a, w, spec, [True, False, False])[0])
                else:
                    dx = _f32_dgrad(dy, w, spec, ctx.xshape, _cl(prev) if prev is not None else None)
                    prev = None
            if spec.sink is not None:
                _f32_wgrad(a, dy, spec, G)
        elif mode == "rows":                     # a = x
            if need_dx:
                w2 = w.reshape(cout, -1)
                if isinstance(prev, MaskedGrad):   # dres from dy + the ReLU bits, inside the GEMM epilogue
                    d2 = _gemm_nt_dgrad(dy2, w2, rows2d(prev.dy), spec, prev.mask)
                    if d2 is None:
                        d2 = rows2d(prev.materialize()).addmm_(dy2, w2)
                    dx = from_rows(d2, n, h, wd)
                    prev = None
                elif prev is not None:           # the other branch's gradient, folded into the GEMM
                    p2 = rows2d(_cl(prev))
                    d2 = _gemm_nt_dgrad(dy2, w2, p2, spec)
                    dx = from_rows(d2 if d2 is not None else p2.addmm_(dy2, w2), n, h, wd)
                    prev = None
                else:
                    d2 = _gemm_nt_dgrad(dy2, w2, None, spec)
                    dx = from_rows(d2 if d2 is not None else torch.mm(dy2, w2), n, h, wd)
            if spec.sink is not None:
                K = w.numel() // cout
                if IWGRAD_1X1 and _iwgrad_ok(a, dy):
                    _iwgrad(a, dy, spec, G, K)
                else:
                    out = spec.sink.rows_view(spec.conv.weight, (cout, K), dy2.dtype)
                    dW = _wgrad(dy2, rows2d(a), G, out, spec.sink)
                    if out is None:
                        spec.sink.put_groups(spec.conv.weight, dW)
        elif mode == "iconv":                    # a = x
            (kh, kw), (sh, sw), (ph, pw), (dh, dw) = spec.kernel, spec.stride, spec.padding, spec.dilation
            K = w.numel() // cout
            use_iw = spec.sink is not None and IWGRAD
            col = None if use_iw else _im2col(a, spec)
            kp = col.shape[1] if col is not None else K
            if need_dx:
                if isinstance(prev, MaskedGrad):   # dres from dy + the ReLU bits, in the halo kernel's epilogue
                    if _halo_dgrad_ok(dy, w, spec):
                        dx = _halo_dgrad(dy, w, spec, prev.dy, prev.mask)
                    if dx is None:
                        prev = prev.materialize()
                    else:
                        prev = None
                if dx is not None:
                    pass
                elif _halo_dgrad_ok(dy, w, spec):
                    dx = _halo_dgrad(dy, w, spec, _cl(prev) if prev is not None else None)
                elif ((sh, sw, dh, dw) == (1, 1, 1, 1) and ph <= kh - 1 and pw <= kw - 1
                        and _iconv_ok(dy, _dgrad_weight_shape(w), dy2.shape[0])):
                    dx = _iconv(dy, w, (kh, kw, 1, 1, kh - 1 - ph, kw - 1 - pw, 1, 1), (h, wd),
                                _cl(prev) if prev is not None else None, transpose_w=True)
                elif (d_s2 := _s2_dgrad(dy, w, spec, ctx.xshape, _cl(prev) if prev is not None else None,
                                        kp)) is not None:
                    dx = d_s2
                else:
                    dx = _dcol_dx(dy2, w, kp, spec, ctx.xshape, _cl(prev) if prev is not None else None)
                prev = None
            if use_iw:
                _iwgrad(a, dy, spec, G, K)
            elif spec.sink is not None:
                out = spec.sink.rows_view(spec.conv.weight, (cout, K), dy2.dtype) if (kp == K or dy2.is_cuda) \
                    else None
                dW = _wgrad(dy2, col, G, out, spec.sink)
                if out is None:
                    if kp != K:
                        dW = dW[:, :, :K].contiguous()
                    spec.sink.put_groups(spec.conv.weight, dW)
        elif mode == "sc":                       # a = x, H, W <= 2: dense GEMMs on the expanded weight
            if need_dx:
                add = _sc_rows(_cl(prev)) if prev is not None else None
                dx = _sc_gemm(_sc_rows(dy), spec.wbigT, add).view(n, h, wd, cin).permute(0, 3, 1, 2)
                prev = None
            if spec.sink is not None:
                _sc_wgrad(a, dy, spec, G)
        elif mode == "stem":                     # a = x (the network input: dx is rarely wanted)
            if need_dx:
                dx = _cl(_conv_bwd(dy, a, w, spec, [True, False, False])[0])
            if spec.sink is not None:
                _stem_wgrad(a, dy, spec, G)
        elif mode == "col":                      # a = col [N*Ho*Wo, Kp]
            kp = a.shape[1]
            if need_dx:
                add = _cl(prev) if prev is not None else None
                dx = _s2_dgrad(dy, w, spec, ctx.xshape, add, kp)
                if dx is None:
                    dx = _dcol_dx(dy2, w, kp, spec, ctx.xshape, add)
                prev = None
            if spec.sink is not None and getattr(ctx, "x", None) is not None:
                _iwgrad(ctx.x, dy, spec, G, w.numel() // cout)    # no patch matrix, no batched GEMM
                ctx.x = None
            elif spec.sink is not None:
                # dW_g[co, (i, j, ci)] = Σ_rows dy_g[row, co] · col_g[row, (i, j, ci)]: the
                # weight's channels_last memory order, one batched GEMM for all workers
                K = w.numel() // cout
                out = spec.sink.rows_view(spec.conv.weight, (cout, K), dy2.dtype) if (kp == K or dy2.is_cuda) \
                    else None
                dW = _wgrad(dy2, a, G, out, spec.sink)
                if out is None:
                    if kp != K:
                        dW = dW[:, :, :K].contiguous()
                    spec.sink.put_groups(spec.conv.weight, dW)
        else:                                    # a = x
            if need_dx:
                dx = _cl(_conv_bwd(dy, a, w, spec, [True, False, False])[0])
            if spec.sink is not None:
                B = a.shape[0] // G
                for g in range(G):
                    sl = slice(g * B, (g + 1) * B)
                    dw = _conv_bwd(dy[sl], a[sl], w, spec, [False, True, False])[1]
                    spec.sink.put(spec.conv.weight, g, _match_layout(dw, w))
        if prev is not None:                     # aten mode: not folded above
            dx = dx + prev
        if first:
            ctx.join.park(dx)
            dx = None
        return dx, None, None, None


def grouped_conv(x, spec: ConvSpec, join: GradJoin | None = None):
    """Convolution with per-worker weight gradients; ``join``: x's other gradient
    branch (see ``GradJoin``)."""
    return _GroupedConv.apply(_cl(x), spec.conv.weight, spec, join)


# --------------------------------------------------------------------------- #
# BatchNorm + ReLU fused into the following 1x1 convolution (the bottleneck's bn2 -> conv3)


class _GroupedBNConv(torch.autograd.Function):
    """conv(relu(BN_per_worker(x))) for a 1x1 stride-1 convolution, without ever writing the
    normalised activation.

    Forward: the BatchNorm's statistics and per-worker scale / shift only (no apply pass); the
    convolution's GEMM applies bf16(max(x * scale + shift, 0)) to each A chunk as it lands in LDS
    (gemm_nt.hip's prologue). Backward: the data gradient is the plain GEMM (it never reads the
    input); the weight gradient applies the same prologue to its input fragments (iconv_nhwc.hip);
    the BatchNorm backward recomputes its ReLU test from x, scale and shift (no mask). Saves the
    apply pass's read + write and the mask of every such BatchNorm, and the next layer reads the
    pre-BatchNorm tensor it would have read anyway."""

    @staticmethod
    def forward(ctx, x, gamma, beta, w, st: BNState, ws: Workspace, spec: ConvSpec):
        n, C, h, wd = x.shape
        x2 = rows2d(x)
        st.ensure(x.device)
        bn, G = st.bn, st.groups
        rg = x2.shape[0] // G
        C_ = _native.native()
        part = ws.get("bn_part", C_.bn_part_floats(rg, G, C), x.device)
        track = bn.track_running_stats and bn.running_mean is not None
        tile, st.tile = st.tile, None
        defer = bool(track and ws.defer_running)
        C_.gpu_bn_forward(x2, None, G, bn.weight, bn.bias, float(bn.eps), float(bn.momentum),
                          bn.running_mean if track else None, bn.running_var if track else None,
                          part, st.mean, st.istd, st.scale, st.shift, None, True, None, defer,
                          tile_stats=tile[0] if tile is not None else None,
                          tile_m=tile[1] if tile is not None else 0, tile_e=tile[2] if tile is not None else 1)
        if defer:
            ws.running_jobs.append((st.mean, st.istd, bn.running_mean, bn.running_var, rg, float(bn.eps),
                                    float(bn.momentum)))
        y2 = _gemm_nt_forward(x2, w.reshape(w.shape[0], -1), spec, pro=(st.scale, st.shift, G))
        if y2 is None:
            raise RuntimeError("fused BatchNorm -> 1x1 convolution: no gemm_nt configuration (bn_conv_ok)")
        ctx.st, ctx.ws, ctx.spec = st, ws, spec
        ctx.save_for_backward(x, w)
        return from_rows(y2, n, h, wd)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        st, ws, spec = ctx.st, ctx.ws, ctx.spec
        dy = _cl(dy)
        dy2 = rows2d(dy)
        G = spec.groups
        cout = dy.shape[1]
        n, C, h, wd = x.shape
        w2 = w.reshape(cout, -1)
        da2 = _gemm_nt_dgrad(dy2, w2, None, spec)          # d(normalised input): never reads x
        if da2 is None:
            da2 = torch.mm(dy2, w2)
        if spec.sink is not None:
            _iwgrad(x, dy, spec, G, C, pro=(st.scale, st.shift))
        x2 = rows2d(x)
        rg = x2.shape[0] // G
        C_ = _native.native()
        bn, sink = st.bn, st.sink
        part = ws.get("bn_part", C_.bn_part_floats(rg, G, C), x.device)
        coef = ws.get("bn_coef", 3 * G * C, x.device)
        grow, stride, og, ob = None, 0, -1, -1
        if sink is not None:
            grow, stride = sink.flat, sink.row_stride
            og = sink.base + sink.offset(bn.weight) if bn.weight is not None else -1
            ob = sink.base + sink.offset(bn.bias) if bn.bias is not None else -1
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        C_.gpu_bn_backward(x2, da2, None, G, bn.weight, st.mean, st.istd, part, coef, rows2d(dx), None, grow, stride,
                           og, ob, relu_scale=st.scale, relu_shift=st.shift)
        return dx, None, None, None, None, None, None


def bn_conv_ok(x: torch.Tensor, st: BNState, spec: ConvSpec) -> bool:
    """Whether BatchNorm st (with ReLU) fuses into the 1x1 convolution spec that consumes it: bf16
    on the GPU, a 1x1 stride-1 GEMM with its weight gradient on the implicit kernels, channel
    counts the MFMA tiles take, and a gemm_nt configuration with a prologue form."""
    if not (BN_PROLOGUE and GEMM_NT and IWGRAD_1X1 and IWGRAD and x.is_cuda and x.dtype == torch.bfloat16
            and spec.gemm and st.relu and spec.sink is not None):
        return False
    w = spec.conv.weight
    if w.dtype != torch.bfloat16 or w.shape[1] % 64 or w.shape[0] % 64 or x.shape[1] % 64:
        return False
    M = x.shape[0] * x.shape[2] * x.shape[3]
    if M % spec.groups:
        return False
    C_ = _native.native()
    K, N, prg = x.shape[1], w.shape[0], M // spec.groups
    return any(C_.gemm_nt_valid(c, N, K) and C_.gemm_nt_pro_ok(c, K, prg, spec.groups)
               for c in range(C_.gemm_nt_num_cfg()))


def grouped_bn_conv(x, st: BNState, ws: Workspace, spec: ConvSpec):
    """conv(relu(BN(x))) with the BatchNorm folded into the convolution (see _GroupedBNConv); the
    caller checks ``bn_conv_ok``."""
    return _GroupedBNConv.apply(_cl(x), st.bn.weight, st.bn.bias, spec.conv.weight, st, ws, spec)


# --------------------------------------------------------------------------- #
# Max pooling (the stem's 3x3/2): no per-worker state, only a faster kernel


def _pool_args(mp: torch.nn.MaxPool2d):
    def one(v):
        if isinstance(v, (tuple, list)):
            return v[0] if len(set(v)) == 1 else None
        return v
    return one(mp.kernel_size), one(mp.stride if mp.stride is not None else mp.kernel_size), one(mp.padding), \
        one(mp.dilation)


class _MaxPool(torch.autograd.Function):
    """NHWC max pooling keeping a one-byte argmax per output element; the backward
    is a gather over the covering windows (ATen's NHWC backward scatters into a
    zero-filled gradient: 102 + 10 µs vs ~15 µs for the stem of the grouped
    ResNet-50 step)."""

    @staticmethod
    def forward(ctx, x, k: int, s: int, p: int):
        n, c, h, w = x.shape
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        y = torch.empty((n, c, ho, wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((n * ho * wo * c,), dtype=torch.uint8, device=x.device)
        _native.native().gpu_maxpool_fwd(x, k, s, p, y, idx)
        ctx.geom = (k, s, p)
        ctx.xshape = tuple(x.shape)
        ctx.save_for_backward(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        k, s, p = ctx.geom
        dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _native.native().gpu_maxpool_bwd(_cl(dy), idx, k, s, p, dx)
        return dx, None, None, None


def grouped_maxpool(x: torch.Tensor, mp: torch.nn.MaxPool2d) -> torch.Tensor:
    k, s, p, d = _pool_args(mp)
    if (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.shape[1] % 8 == 0 and d == 1 and not mp.ceil_mode
            and None not in (k, s, p) and 2 * p <= k and k * k <= 256):
        return _MaxPool.apply(_cl(x), int(k), int(s), int(p))
    y = F.max_pool2d(x, mp.kernel_size, mp.stride, mp.padding, mp.dilation, mp.ceil_mode)
    return y.contiguous(memory_format=torch.channels_last)


# --------------------------------------------------------------------------- #
# Grouped linear (classifier)


class LinearSpec:
    def __init__(self, lin: torch.nn.Linear, sink: GradSink | None, groups: int):
        self.lin = lin
        self.sink = sink
        self.groups = groups
        self.wp = None    # wide bf16 head: the step's zero-padded weight [Op, F] and its transpose [F, Op]
        self.wpt = None


# outputs up to which the bf16 classifier runs on its own streaming kernels (conv_f32.hip: the CIFAR
# 10-class head is an 8 MB HBM stream, not a GEMM); a wider head (ImageNet's 1000 classes: 8 GFLOP
# per pass) is a GEMM and runs on gemm_nt.hip / the 1x1 weight-gradient kernel with its outputs
# padded to a multiple of 64 (``_wide_head_*``)
_LINEAR_BF16_MAX_O = 16


def _native_linear(x: torch.Tensor, w: torch.Tensor) -> str | None:
    """The classifier's own kernels (conv_f32.hip: fp32 accumulation, one rounding): "f32" / "bf16"
    for matching GPU operands, None for the CPU path (and the wide bf16 head, see above)."""
    if not x.is_cuda:
        return None
    if x.dtype == torch.float32 and w.dtype == torch.float32:
        return "f32"
    if x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        if w.shape[0] <= _LINEAR_BF16_MAX_O:
            return "bf16" if x.shape[1] % 8 == 0 else None
        return "wide" if x.shape[1] % 64 == 0 and w.shape[0] % 8 == 0 else None
    raise TypeError(f"grouped linear on the GPU: fp32 or bf16 operands, got {x.dtype} x {w.dtype}")


class _GroupedLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, spec: LinearSpec):
        ctx.spec = spec
        ctx.save_for_backward(x, w)
        kind = _native_linear(x, w)
        if kind == "wide":
            return _wide_head_forward(x, w, b, spec)
        if kind is not None:   # no library GEMM: the classifier's own kernel
            y = torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
            bb = b.detach().to(x.dtype).contiguous() if b is not None else None
            fwd = _native.native().gpu_linear_f32_fwd if kind == "f32" else _native.native().gpu_linear_bf16_fwd
            fwd(x.contiguous(), w.contiguous(), bb, y)
            return y
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        spec = ctx.spec
        G = spec.groups
        dy = dy.contiguous()
        kind = _native_linear(x, w) if dy.is_cuda else None
        if kind == "f32":
            return _linear_f32_backward(ctx, x, w, dy, spec, G)
        if kind == "bf16":
            return _linear_bf16_backward(ctx, x, w, dy.to(torch.bfloat16), spec, G)
        if kind == "wide":
            return _wide_head_backward(ctx, x, w, dy.to(torch.bfloat16), spec, G)
        dx = torch.mm(dy, w) if ctx.needs_input_grad[0] else None
        if spec.sink is not None:
            out, fin = dy.shape[1], x.shape[1]
            dy3 = dy.view(G, -1, out)
            x3 = x.contiguous().view(G, -1, fin)
            wv = spec.sink.rows_view(spec.lin.weight, (out, fin), dy.dtype)
            if wv is not None:
                torch.bmm(dy3.transpose(1, 2), x3, out=wv)
            else:
                spec.sink.put_groups(spec.lin.weight, torch.bmm(dy3.transpose(1, 2), x3))
            if spec.lin.bias is not None:
                sink = spec.sink
                if (dy.is_cuda and dy.dtype in (torch.bfloat16, torch.float32) and sink.flat.is_cuda
                        and sink.flat.dtype in (torch.float32, torch.bfloat16, torch.float16)):
                    # fp32 sums straight into the exchange rows (no ATen reduction)
                    _native.native().gpu_linear_bias_grad(dy, G, sink.flat, sink.row_stride,
                                                          sink.base + sink.offset(spec.lin.bias))
                else:
                    bv = sink.rows_view(spec.lin.bias, (out,), dy.dtype)
                    if bv is not None:       # reduced in fp32, written in the exchange dtype
                        torch.sum(dy3, 1, out=bv)
                    else:
                        sink.put_groups(spec.lin.bias, _acc(dy3).sum(1))
        return dx, None, None, None


def _wide_head_forward(x: torch.Tensor, w: torch.Tensor, b, spec: LinearSpec) -> torch.Tensor:
    """y = x·wᵀ + b for a wide bf16 head: the step's padded weights (one launch, refreshed here since the
    weights change once per step), the GEMM on gemm_nt.hip into [R, Op] rows, then one pass that crops
    them to [R, O] adding the bias (fp32 add, so the logits are rounded twice: GEMM, bias)."""
    C_ = _native.native()
    O, F = w.shape
    Op = -(-O // 64) * 64
    if spec.wp is None or spec.wp.shape != (Op, F) or spec.wp.device != w.device:
        spec.wp = torch.empty((Op, F), dtype=w.dtype, device=w.device)
        spec.wpt = torch.empty((F, Op), dtype=w.dtype, device=w.device)
    C_.gpu_head_weights(w.detach().contiguous(), spec.wp, spec.wpt)
    x = x.contiguous()
    yp = torch.empty((x.shape[0], Op), dtype=x.dtype, device=x.device)
    cfg = _gemm_cfg(x, spec.wp, 0, None)
    if cfg < 0:
        raise RuntimeError(f"wide head: no gemm_nt configuration for [{x.shape[0]}, {F}] x [{Op}, {F}]")
    C_.gpu_gemm_nt(x, spec.wp, yp, None, None, 0, cfg)
    y = torch.empty((x.shape[0], O), dtype=x.dtype, device=x.device)
    bb = b.detach().to(x.dtype).contiguous() if b is not None else None
    C_.gpu_repitch(yp, y, bb)
    return y


def _wide_head_backward(ctx, x, w, dy, spec: LinearSpec, G: int):
    """Wide bf16 head backward without a library GEMM: dy padded to [R, Op] (zero columns), dx = dyp·wpᵀᵀ
    on gemm_nt.hip with the step's wpt, every worker's dW on the 1x1 weight-gradient kernel as fp32 split
    slabs of [Op, F] whose first O rows are summed into the exchange rows (deferred, batched with the
    convolutions' slabs), db from dy straight into the rows."""
    C_ = _native.native()
    O, F = w.shape
    R = x.shape[0]
    Op = spec.wpt.shape[1]
    dyp = torch.empty((R, Op), dtype=dy.dtype, device=dy.device)
    C_.gpu_repitch(dy, dyp, None)
    dx = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty((R, F), dtype=x.dtype, device=x.device)
        cfg = _gemm_cfg(dyp, spec.wpt, 0, None)
        if cfg < 0:
            raise RuntimeError(f"wide head: no gemm_nt configuration for [{R}, {Op}] x [{F}, {Op}]")
        C_.gpu_gemm_nt(dyp, spec.wpt, dx, None, None, 0, cfg)
    sink = spec.sink
    if sink is not None:
        lin = spec.lin
        x4 = x.contiguous().view(R, F, 1, 1)     # a 1x1 convolution over R one-pixel images
        dy4 = dyp.view(R, Op, 1, 1)
        S = _iwgrad_splits(R // G, (F // 64) * (Op // 64) * G // C_.iwgrad_taps_per_block(1, 1, F, Op))
        part = torch.empty((S, G, Op, F), dtype=torch.float32, device=x.device)
        C_.gpu_iwgrad(x4, dy4, 1, 1, 1, 1, 0, 0, 1, 1, G, part, S)
        rows = sink.rows_view(lin.weight, (O, F), sink.flat.dtype)
        if rows is not None:
            sink.queue_split(part[:, :, :O], rows)
        else:
            sink.put_groups(lin.weight, part.sum(0)[:, :O])
        if lin.bias is not None:
            if sink.flat.is_cuda and sink.flat.dtype in (torch.float32, torch.bfloat16, torch.float16):
                C_.gpu_linear_bias_grad(dy, G, sink.flat, sink.row_stride, sink.base + sink.offset(lin.bias))
            else:
                sink.put_groups(lin.bias, dy.view(G, -1, O).float().sum(1))
    return dx, None, None, None


def _linear_f32_backward(ctx, x, w, dy, spec: LinearSpec, G: int):
    """fp32 classifier backward on the native kernels: dx = dy·W, and every worker's dW / db
    written straight into its fp32 exchange row (or queued for the flatten kernel)."""
    C_ = _native.native()
    dx = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty_like(x)
        C_.gpu_linear_f32_dgrad(dy, w.contiguous(), dx)
    sink = spec.sink
    if sink is not None:
        lin = spec.lin
        if sink.flat.dtype == torch.float32 and sink.flat.is_cuda:
            ob = sink.base + sink.offset(lin.bias) if lin.bias is not None else -1
            C_.gpu_linear_f32_wgrad(x.contiguous(), dy, G, sink.flat, sink.row_stride, sink.base + sink.offset(lin.weight),
                                    ob)
        else:
            x3 = x.contiguous().view(G, -1, x.shape[1])
            dy3 = dy.view(G, -1, dy.shape[1])
            sink.put_groups(lin.weight, torch.bmm(dy3.transpose(1, 2), x3))
            if lin.bias is not None:
                sink.put_groups(lin.bias, dy3.sum(1))
    return dx, None, None, None


def _linear_bf16_backward(ctx, x, w, dy, spec: LinearSpec, G: int):
    """bf16 classifier backward on the native kernels: dx = dy·W, and every worker's dW / db (fp32
    sums, one rounding) written straight into its exchange row (any exchange dtype)."""
    C_ = _native.native()
    dx = None
    if ctx.needs_input_grad[0]:
        dx = torch.empty_like(x)
        C_.gpu_linear_bf16_dgrad(dy, w.contiguous(), dx)
    sink = spec.sink
    if sink is not None:
        lin = spec.lin
        if sink.flat.is_cuda and sink.flat.dtype in (torch.float32, torch.bfloat16, torch.float16):
            ob = sink.base + sink.offset(lin.bias) if lin.bias is not None else -1
            C_.gpu_linear_bf16_wgrad(x.contiguous(), dy, G, sink.flat, sink.row_stride,
                                     sink.base + sink.offset(lin.weight), ob)
        else:
            x3 = x.contiguous().view(G, -1, x.shape[1]).float()
            dy3 = dy.view(G, -1, dy.shape[1]).float()
            sink.put_groups(lin.weight, torch.bmm(dy3.transpose(1, 2), x3))
            if lin.bias is not None:
                sink.put_groups(lin.bias, dy3.sum(1))
    return dx, None, None, None


class _AvgPoolF32(torch.autograd.Function):
    """Global average pool of an fp32 or bf16 NHWC activation on the native kernel (no ATen
    reduction)."""

    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        y = torch.empty((n, c), dtype=x.dtype, device=x.device)
        _native.native().gpu_avgpool_f32(x, y, False)
        ctx.xshape = tuple(x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _native.native().gpu_avgpool_f32(dy.contiguous(), dx, True)
        return dx


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> [N, C] mean over H, W (a view when H = W = 1)."""
    n, c, h, w = x.shape
    if h * w == 1:
        return x.reshape(n, c)
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous(memory_format=torch.channels_last):
        return _AvgPoolF32.apply(x)
    return x.mean((2, 3))


def grouped_linear(x, spec: LinearSpec):
    return _GroupedLinear.apply(x, spec.lin.weight, spec.lin.bias, spec)


class _GroupedXent(torch.autograd.Function):
    """Per-worker mean cross-entropy on the fused HIP kernel (loss_xent.hip): the
    forward writes each worker's loss and d(loss_g)/d(logits); the backward scales
    that by the upstream per-worker gradient."""

    @staticmethod
    def forward(ctx, logits, labels, groups: int):
        loss = torch.empty(groups, dtype=torch.float32, device=logits.device)
        dl = torch.empty_like(logits)
        _native.native().gpu_xent_forward(logits, labels, groups, loss, dl)
        ctx.save_for_backward(dl)
        ctx.groups = groups
        return loss

    @staticmethod
    def backward(ctx, go):
        (dl,) = ctx.saved_tensors
        dx = torch.empty_like(dl)
        _native.native().gpu_xent_backward(dl, go.float().contiguous(), ctx.groups, dx)
        return dx, None, None


def grouped_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, groups: int) -> torch.Tensor:
    """[groups] per-worker mean cross-entropy of ``logits`` [groups*rows, classes];
    the fused kernels on GPU (bf16/fp32 logits, int64 labels: one thread per row up to 64 classes,
    one wave per row beyond), else ATen."""
    if (XENT and logits.is_cuda and logits.dim() == 2
            and logits.dtype in (torch.bfloat16, torch.float32) and labels.dtype == torch.int64):
        return _GroupedXent.apply(logits.contiguous(), labels.contiguous(), groups)
    lg = logits if logits.dtype == torch.float64 else logits.float()
    return F.cross_entropy(lg, labels, reduction="none").view(groups, -1).mean(1)
