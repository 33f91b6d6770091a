"""Device-dispatching front-end of the robust gradient aggregation rules (GARs).

Every rule accepts the gradient set either as an ``[n, d]`` tensor (rows may be
views of a padded exchange buffer) or as a list of ``n`` 1-D tensors (the
reference's ``gradients=[...]`` calling convention, ``PT/libs/aggregators/
__init__.py:15-31``), and returns a NEW 1-D tensor of the input dtype.

GPU path (``garfield_amd._C``, gfx950 HIP), all launches asynchronous on the
current stream, nothing copied to the host:

* Krum / Multi-Krum: split-K MFMA Gram -> one-workgroup selection -> combine;
* Bulyan: Gram -> on-device selection loop -> W[t, n] -> fused W·G averaged-median;
* Brute: Gram -> device-wide subset search (atomicMin on (diameter, rank)) -> combine;
* Median / Trimmed-Mean / Averaged-Median / Average-NaN / Condense: register
  sorting-network kernels;
* Aksel: median kernel -> squared distance to it -> selection -> combine.

CPU path: the C++ thread-pool implementations in the same extension.

More than ``MAX_ROWS`` (128) gradients (the reference's gar_bench sweeps n to 512): on
the GPU, up to ``LARGE_ROWS`` (1024) rows run on ``gar_large.hip`` as one [n, d] matrix
(combine with fp32 accumulation; median / trimmed-mean / averaged-median and the Bulyan
tail by LDS radix select; the Krum/Bulyan Gram as a split-K MFMA kernel with fp32 output and
Bulyan's W·X on fp32 MFMA);
everything else, and the CPU, uses a vectorised PyTorch implementation.
"""
from __future__ import annotations

import math
import threading
from dataclasses import dataclass, field

import torch

from garfield_amd import _native
from garfield_amd.ops import reference as ref

MAX_ROWS = 128
LARGE_ROWS = 1024
_LARGE_MODE = {"median": 0, "trimmed-mean": 1, "averaged-median": 2}

_MODE = {"median": 0, "trimmed-mean": 1, "averaged-median": 2, "average-nan": 3, "condense": 4, "bulyan-tail": 5}


# --------------------------------------------------------------------------- #
# Input normalisation


@dataclass
class Rows:
    """A gradient set ready for the native layer."""

    obj: object  # [n, d] tensor or list of 1-D tensors
    n: int
    d: int
    dtype: torch.dtype
    device: torch.device
    out_dtype: torch.dtype  # dtype of the returned aggregate

    def stacked(self) -> torch.Tensor:
        if isinstance(self.obj, torch.Tensor):
            return self.obj
        return torch.stack(list(self.obj))


_SUPPORTED_GPU = (torch.float32, torch.bfloat16, torch.float16)


def _aligned(t: torch.Tensor) -> bool:
    return t.data_ptr() % 16 == 0


def prepare(gradients) -> Rows:
    """Validate and normalise a gradient set (list of tensors or [n, d] tensor)."""
    if isinstance(gradients, torch.Tensor):
        if gradients.dim() == 1:
            gradients = gradients.unsqueeze(0)
        if gradients.dim() != 2:
            raise ValueError(f"expected an [n, d] gradient tensor, got shape {tuple(gradients.shape)}")
        G = gradients
        out_dtype = G.dtype
        if G.device.type == "cpu":
            if G.dtype not in (torch.float32, torch.float64):
                G = G.float()
            if G.stride(1) != 1:
                G = G.contiguous()
        else:
            if G.dtype not in _SUPPORTED_GPU:
                G = G.float()
            esz = G.element_size()
            if G.stride(1) != 1 or (G.stride(0) * esz) % 16 != 0 or not _aligned(G):
                G = _padded_copy(G)
        return Rows(G, G.shape[0], G.shape[1], G.dtype, G.device, out_dtype)
    if not isinstance(gradients, (list, tuple)) or len(gradients) == 0:
        raise ValueError("expected a non-empty list of gradients")
    first = gradients[0]
    dev, dt = first.device, first.dtype
    d = first.numel()
    rows = []
    for g in gradients:
        if g.device != dev:
            raise ValueError("all gradients must be on the same device")
        if g.numel() != d:
            raise ValueError(f"all gradients must have the same size ({g.numel()} != {d})")
        rows.append(g.reshape(-1))
    out_dtype = dt
    if dev.type == "cpu":
        if dt not in (torch.float32, torch.float64):
            rows = [r.float() for r in rows]
        rows = [r if r.is_contiguous() else r.contiguous() for r in rows]
        if any(r.dtype != rows[0].dtype for r in rows):
            rows = [r.float() for r in rows]
    else:
        if dt not in _SUPPORTED_GPU or any(r.dtype != dt for r in rows):
            rows = [r.float() for r in rows]
        rows = [r if (r.is_contiguous() and _aligned(r)) else r.clone(memory_format=torch.contiguous_format)
                for r in rows]
        rows = [r if _aligned(r) else _aligned_clone(r) for r in rows]
    return Rows(rows, len(rows), d, rows[0].dtype, dev, out_dtype)


def _aligned_clone(t: torch.Tensor) -> torch.Tensor:
    buf = torch.empty(t.numel() + 16, dtype=t.dtype, device=t.device)
    off = (-(buf.data_ptr() % 16) // t.element_size()) % (16 // t.element_size())
    v = buf[off:off + t.numel()]
    v.copy_(t)
    return v


def _padded_copy(G: torch.Tensor) -> torch.Tensor:
    n, d = G.shape
    esz = G.element_size()
    align = 16 // esz
    ld = ((d + align - 1) // align) * align
    buf = torch.empty((n, ld), dtype=G.dtype, device=G.device)
    buf[:, :d].copy_(G)
    return buf[:, :d]


# --------------------------------------------------------------------------- #
# Device workspaces (allocated once per shape/stream, reused: capture-safe)


@dataclass
class Workspace:
    n: int
    d: int
    device: torch.device
    tensors: dict = field(default_factory=dict)

    def get(self, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
        t = self.tensors.get(name)
        if t is None or t.numel() < numel or t.dtype != dtype:
            t = torch.empty(max(numel, 1), dtype=dtype, device=self.device)
            self.tensors[name] = t
        return t[:numel]


_WS: dict = {}
_WS_LOCK = threading.Lock()


def workspace(rows: Rows) -> Workspace:
    stream = torch.cuda.current_stream(rows.device).cuda_stream if rows.device.type == "cuda" else 0
    key = (str(rows.device), rows.n, rows.d, stream)
    with _WS_LOCK:
        ws = _WS.get(key)
        if ws is None:
            if len(_WS) > 64:
                _WS.clear()
            ws = Workspace(rows.n, rows.d, rows.device)
            _WS[key] = ws
    return ws


def _C_for(rows: Rows):
    return _native.require_for(rows.device)


def _finish(out: torch.Tensor, rows: Rows) -> torch.Tensor:
    return out if out.dtype == rows.out_dtype else out.to(rows.out_dtype)


# --------------------------------------------------------------------------- #
# Building blocks


def gram(gradients) -> torch.Tensor:
    """G·Gᵀ (fp32 [n, n]) on the GPU; fp64 pairwise squared distances are in pairwise_distances."""
    rows = prepare(gradients)
    if rows.device.type != "cuda":
        X = rows.stacked().double()
        return X @ X.T
    if rows.n > MAX_ROWS:
        return _large_gram(rows)
    C = _C_for(rows)
    ws = workspace(rows)
    g = _gram_into(C, rows, ws)
    np_ = C.gram_padded(rows.n)
    return g.view(np_, np_)[: rows.n, : rows.n].clone()


def _gram_into(C, rows: Rows, ws: Workspace) -> torch.Tensor:
    grid = C.gram_grid(rows.d, _dtype_probe(rows), rows.n)
    slabs = ws.get("slabs", (grid + C.GRAM_REDUCE_GROUPS) * C.gram_slab_floats(rows.n))
    np_ = C.gram_padded(rows.n)
    g = ws.get("gram", np_ * np_)
    C.gpu_gram(rows.obj, slabs, g)
    return g


_PROBES: dict = {}


def _dtype_probe(rows: Rows) -> torch.Tensor:
    p = _PROBES.get(rows.dtype)
    if p is None:
        p = torch.empty(0, dtype=rows.dtype)
        _PROBES[rows.dtype] = p
    return p


def pairwise_distances(gradients) -> torch.Tensor:
    """Squared L2 distance matrix [n, n] (+inf on the diagonal and for non-finite pairs)."""
    rows = prepare(gradients)
    if rows.device.type == "cuda":
        g = gram(rows.obj).double()
        dg = torch.diagonal(g)
        D = dg[:, None] + dg[None, :] - 2 * g
        D = torch.where(torch.isfinite(D), D.clamp(min=0), torch.full_like(D, math.inf))
        D.fill_diagonal_(math.inf)
        return D.cpu()
    C = _C_for(rows)
    if C is None:
        return ref.pairwise_sqdist(rows.stacked())
    return C.cpu_pairwise(rows.obj)


def combine(gradients, weights: torch.Tensor) -> torch.Tensor:
    rows = prepare(gradients)
    if _large(rows):
        return _large_combine(rows, weights)
    if rows.n > MAX_ROWS:
        return _finish((weights.to(rows.device, torch.float32)[:, None] * rows.stacked().float()).sum(0), rows)
    C = _C_for(rows)
    if rows.device.type == "cuda":
        out = torch.empty(rows.d, dtype=rows.dtype, device=rows.device)
        C.gpu_combine(rows.obj, weights.to(rows.device, torch.float32).contiguous(), out)
        return _finish(out, rows)
    if C is None:
        return ref.combine(rows.stacked(), weights.double()).to(rows.out_dtype)
    return _finish(C.cpu_combine(rows.obj, weights.float().cpu()), rows)


def combine_into(gradients, weights: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32, [d]) = Σ_j w_j g_j in fp32 (the GPU combine kernel's arithmetic, no rounding to
    the gradients' dtype): the layer-wise loop's per-segment combine."""
    rows = prepare(gradients)
    if rows.device.type == "cuda" and rows.n <= MAX_ROWS:
        dst = out if (out.is_contiguous() and _aligned(out)) else torch.empty_like(out)
        _C_for(rows).gpu_combine(rows.obj, weights.to(rows.device, torch.float32).contiguous(), dst)
        if dst is not out:
            out.copy_(dst)
        return
    X = rows.stacked().double() if rows.dtype == torch.float64 else rows.stacked().float()
    out.copy_((weights.to(X.device, X.dtype)[:, None] * X).sum(0))


def _large(rows: Rows) -> bool:
    """GPU set of MAX_ROWS < n <= LARGE_ROWS gradients: the gar_large.hip kernels."""
    return rows.device.type == "cuda" and MAX_ROWS < rows.n <= LARGE_ROWS


def _matrix(rows: Rows) -> torch.Tensor:
    X = rows.stacked()
    return X if X.stride(1) == 1 else X.contiguous()


def _large_combine(rows: Rows, w: torch.Tensor) -> torch.Tensor:
    X = _matrix(rows)
    out = torch.empty(rows.d, dtype=X.dtype, device=X.device)
    _native.native().gpu_large_combine(X, w.to(X.device, torch.float32).contiguous(), out)
    return _finish(out, rows)


# --------------------------------------------------------------------------- #
# Rules


def average(gradients, **_) -> torch.Tensor:
    rows = prepare(gradients)
    if rows.device.type == "cuda" and rows.n <= MAX_ROWS:
        C = _C_for(rows)
        ws = workspace(rows)
        w = ws.tensors.get("avg_w")
        if w is None:
            w = torch.full((rows.n,), 1.0 / rows.n, dtype=torch.float32, device=rows.device)
            ws.tensors["avg_w"] = w
        out = torch.empty(rows.d, dtype=rows.dtype, device=rows.device)
        C.gpu_combine(rows.obj, w, out)
        return _finish(out, rows)
    if _large(rows):
        return _large_combine(rows, torch.full((rows.n,), 1.0 / rows.n, dtype=torch.float32, device=rows.device))
    return _finish(rows.stacked().float().mean(0) if rows.dtype != torch.float64 else rows.stacked().mean(0), rows)


def krum_weights(gradients, f: int, m: int | None = None) -> torch.Tensor:
    """Selection weights of Multi-Krum ([n] fp32 on the gradients' device)."""
    rows = prepare(gradients)
    m = rows.n - f - 2 if m is None else m
    return _krum_weights(rows, f, m)


def _krum_weights(rows: Rows, f: int, m: int) -> torch.Tensor:
    if rows.n > MAX_ROWS:
        return _large_krum_weights(rows, f, m)
    C = _C_for(rows)
    if rows.device.type == "cuda":
        ws = workspace(rows)
        g = _gram_into(C, rows, ws)
        w = ws.get("weights", rows.n)
        order = ws.get("order", rows.n, torch.int32)
        scores = ws.get("scores", rows.n)
        C.gpu_krum_select(g, rows.n, f, m, w, order, scores)
        return w
    if C is None:
        return ref.krum_weights(ref.pairwise_sqdist(rows.stacked()), f, m).float()
    w, _ = C.cpu_krum_weights(C.cpu_pairwise(rows.obj), f, m)
    return w


def krum(gradients, f: int, m: int | None = None, **_) -> torch.Tensor:
    rows = prepare(gradients)
    m = rows.n - f - 2 if m is None else m
    w = _krum_weights(rows, f, m)
    return _combine_rows(rows, w)


def _combine_rows(rows: Rows, w: torch.Tensor) -> torch.Tensor:
    if _large(rows):
        return _large_combine(rows, w)
    if rows.n > MAX_ROWS:
        return _finish((w.to(rows.device)[:, None] * rows.stacked().float()).sum(0), rows)
    C = _C_for(rows)
    if rows.device.type == "cuda":
        out = torch.empty(rows.d, dtype=rows.dtype, device=rows.device)
        C.gpu_combine(rows.obj, w, out)
        return _finish(out, rows)
    if C is None:
        return ref.combine(rows.stacked(), w.double()).to(rows.out_dtype)
    return _finish(C.cpu_combine(rows.obj, w), rows)


def bulyan_weights(gradients, f: int, m: int | None = None) -> torch.Tensor:
    rows = prepare(gradients)
    m = rows.n - f - 2 if m is None else m
    return _bulyan_W(rows, f, m)


def _bulyan_W(rows: Rows, f: int, m: int) -> torch.Tensor:
    t = rows.n - 2 * f - 2
    C = _C_for(rows)
    if rows.device.type == "cuda" and rows.n <= MAX_ROWS:
        ws = workspace(rows)
        g = _gram_into(C, rows, ws)
        W = ws.get("bulyan_W", t * rows.n)
        C.gpu_bulyan_select(g, rows.n, f, m, t, W)
        return W.view(t, rows.n)
    if rows.device.type == "cuda" and rows.n > MAX_ROWS:
        return large_select(_large_gram(rows), f, m, bulyan=True)
    D = pairwise_distances(rows.obj) if C is not None else ref.pairwise_sqdist(rows.stacked())
    if rows.n > MAX_ROWS:
        return _large_bulyan_weights(D, f, m).float().to(rows.device)
    if C is None:
        return ref.bulyan_weights(D, f, m).float().to(rows.device)
    return C.cpu_bulyan_weights(D, f, m, t)


def bulyan(gradients, f: int, m: int | None = None, **_) -> torch.Tensor:
    rows = prepare(gradients)
    m = rows.n - f - 2 if m is None else m
    t = rows.n - 2 * f - 2
    beta = t - 2 * f
    W = _bulyan_W(rows, f, m)
    if _large(rows):   # V = W·X column chunk by chunk (bounded fp32 memory), then the radix-select tail
        X, Wd = _matrix(rows), W.to(rows.device, torch.float32)
        out = torch.empty(rows.d, dtype=torch.float32, device=rows.device)
        step = max(1, (1 << 28) // (4 * max(rows.n, t)))
        Vbuf = torch.empty((t, min(step, rows.d)), dtype=torch.float32, device=rows.device)
        for c0 in range(0, rows.d, step):
            w = min(step, rows.d - c0)
            V = large_wx(Wd, X[:, c0:c0 + w], Vbuf[:, :w])
            _native.native().gpu_large_coord(V, 2, 0, beta, out[c0:c0 + w])
        return _finish(out, rows)
    if rows.n > MAX_ROWS:
        V = W.to(rows.device) @ rows.stacked().float()
        return _finish(_torch_closest_mean(V, beta), rows)
    C = _C_for(rows)
    if rows.device.type == "cuda":
        out = torch.empty(rows.d, dtype=rows.dtype, device=rows.device)
        C.gpu_coordwise(rows.obj, _MODE["bulyan-tail"], f, beta, W.reshape(-1), t, 0, 1.0, out)
        return _finish(out, rows)
    if C is None:
        return ref.bulyan(rows.stacked(), f, m).to(rows.out_dtype)
    return _finish(C.cpu_coordwise(rows.obj, _MODE["bulyan-tail"], f, beta, W.reshape(-1), t, 0, 1.0), rows)


def _coord(rows: Rows, mode: str, f: int = 0, beta: int = 0, seed: int = 0, p: float = 1.0) -> torch.Tensor:
    if _large(rows) and mode in _LARGE_MODE:
        X = _matrix(rows)
        out = torch.empty(rows.d, dtype=X.dtype, device=X.device)
        _native.native().gpu_large_coord(X, _LARGE_MODE[mode], f, beta, out)
        return _finish(out, rows)
    if rows.n > MAX_ROWS:
        return _finish(_torch_coord(rows.stacked().float(), mode, f, beta, seed, p), rows)
    C = _C_for(rows)
    code = _MODE[mode]
    if rows.device.type == "cuda":
        out = torch.empty(rows.d, dtype=rows.dtype, device=rows.device)
        C.gpu_coordwise(rows.obj, code, f, beta, None, 0, seed, p, out)
        return _finish(out, rows)
    if C is None:
        X = rows.stacked()
        r = {"median": lambda: ref.median(X), "trimmed-mean": lambda: ref.trimmed_mean(X, f),
             "averaged-median": lambda: ref.averaged_median(X, beta), "average-nan": lambda: ref.average_nan(X),
             "condense": lambda: ref.condense(X, p, seed)}[mode]()
        return r.to(rows.out_dtype)
    return _finish(C.cpu_coordwise(rows.obj, code, f, beta, None, 0, seed, p), rows)


def median(gradients, **_) -> torch.Tensor:
    return _coord(prepare(gradients), "median")


def trimmed_mean(gradients, f: int, **_) -> torch.Tensor:
    return _coord(prepare(gradients), "trimmed-mean", f=f)


def averaged_median(gradients, f: int = 0, beta: int | None = None, **_) -> torch.Tensor:
    rows = prepare(gradients)
    beta = rows.n - f if beta is None else beta
    return _coord(rows, "averaged-median", beta=beta)


def average_nan(gradients, **_) -> torch.Tensor:
    return _coord(prepare(gradients), "average-nan")


def condense(gradients, p: float = 0.9, seed: int | None = None, **_) -> torch.Tensor:
    if seed is None:
        seed = int(torch.randint(0, 2**62, (1,)).item())
    return _coord(prepare(gradients), "condense", seed=seed, p=p)


def brute_weights(gradients, f: int) -> torch.Tensor:
    rows = prepare(gradients)
    return _brute_w(rows, f)


BRUTE_MAX_SUBSETS = 2 ** 32


def _brute_w(rows: Rows, f: int) -> torch.Tensor:
    # the device search keys each subset by its 32-bit rank (gar_gram.hip k_brute_*): refuse
    # what it cannot index (C(64, 56) is 4.4e9 subsets: infeasible on any device anyway)
    subsets = math.comb(rows.n, rows.n - f) if 0 <= f <= rows.n else 0
    if subsets > BRUTE_MAX_SUBSETS:
        raise ValueError(f"brute: C({rows.n}, {rows.n - f}) = {subsets} subsets exceeds 2^32; use a smaller f "
                         "or another rule")
    C = _C_for(rows)
    if rows.device.type == "cuda" and rows.n <= 64:
        ws = workspace(rows)
        g = _gram_into(C, rows, ws)
        best = ws.get("brute_best", 1, torch.int64)
        w = ws.get("weights", rows.n)
        C.gpu_brute_select(g, rows.n, f, best, w)
        return w
    if C is None or rows.n > 64:
        return ref.brute_weights(pairwise_distances(rows.obj) if C else ref.pairwise_sqdist(rows.stacked()), f).float().to(rows.device)
    return C.cpu_brute_weights(C.cpu_pairwise(rows.obj), f)


def brute(gradients, f: int, **_) -> torch.Tensor:
    rows = prepare(gradients)
    return _combine_rows(rows, _brute_w(rows, f))


def aksel_weights(gradients, f: int, mode: str = "mid") -> torch.Tensor:
    rows = prepare(gradients)
    return _aksel_w(rows, f, mode)


def _aksel_w(rows: Rows, f: int, mode: str) -> torch.Tensor:
    c = (rows.n + 1) // 2 if mode == "mid" else rows.n - f
    C = _C_for(rows)
    if rows.device.type == "cuda" and rows.n <= MAX_ROWS:
        ws = workspace(rows)
        med = ws.get("aksel_med", rows.d)
        C.gpu_coordwise(rows.obj, _MODE["median"], 0, 0, None, 0, 0, 1.0, med)
        grid = C.sqdist_grid(rows.d)
        slabs = ws.get("aksel_slabs", grid * rows.n)
        C.gpu_sqdist(rows.obj, med, slabs)
        w = ws.get("weights", rows.n)
        dists = ws.get("aksel_dists", rows.n)
        C.gpu_aksel_select(slabs, rows.n, c, w, dists)
        return w
    if C is None or rows.n > MAX_ROWS:
        X = rows.stacked().double()
        med = _torch_coord(X, "median", 0, 0, 0, 1.0) if rows.n > MAX_ROWS else ref.median(X)
        dist = ((X - med.to(X.device)) ** 2).sum(1).cpu()
        dist = torch.where(torch.isfinite(dist), dist, torch.full_like(dist, math.inf))
        order = sorted(range(rows.n), key=lambda j: (float(dist[j]), j))
        w = torch.zeros(rows.n, dtype=torch.float32)
        w[order[:c]] = 1.0 / c
        return w.to(rows.device)
    med = C.cpu_coordwise(rows.obj, _MODE["median"], 0, 0, None, 0, 0, 1.0)
    return C.cpu_aksel_weights(C.cpu_sqdist(rows.obj, med), c)


def aksel(gradients, f: int, mode: str = "mid", **_) -> torch.Tensor:
    rows = prepare(gradients)
    return _combine_rows(rows, _aksel_w(rows, f, mode))


# --------------------------------------------------------------------------- #
# Vectorised PyTorch implementations for n > MAX_ROWS (same semantics).


def large_gram(X: torch.Tensor) -> torch.Tensor:
    """fp32 Gram matrix [n, n] of a GPU [n, d] matrix of up to LARGE_ROWS rows on the MFMA kernel of
    gar_large.hip (split-K 64 x 64 tiles, fixed-order sums; no library GEMM)."""
    C = _native.native()
    if X.stride(1) != 1 or (X.stride(0) * X.element_size()) % 16 or X.data_ptr() % 16:
        X = X.contiguous()
        if (X.shape[1] * X.element_size()) % 16:   # pad the rows to 16 bytes (zeros add nothing)
            X = torch.nn.functional.pad(X, (0, (-X.shape[1]) % (16 // X.element_size())))
    n, d = X.shape
    slabs = torch.empty(max(C.large_gram_slab_floats(n, d, X), 1), dtype=torch.float32, device=X.device)
    g = torch.empty((n, n), dtype=torch.float32, device=X.device)
    C.gpu_large_gram(X, slabs, g)
    return g


def large_wx(W: torch.Tensor, X: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """V [t, d] = W [t, n] · X [n, d] in fp32 on the MFMA kernel of gar_large.hip."""
    if X.stride(1) != 1:
        X = X.contiguous()
    V = out if out is not None else torch.empty((W.shape[0], X.shape[1]), dtype=torch.float32, device=X.device)
    _native.native().gpu_large_wx(W.contiguous(), X, V)
    return V


def _large_gram(rows: Rows) -> torch.Tensor:
    """fp32 Gram matrix of a large set: the MFMA kernel on the GPU, fp32 matmul on the CPU."""
    if rows.device.type == "cuda":
        return large_gram(_matrix(rows))
    X = rows.stacked().float()
    return X @ X.T


def _large_krum_weights(rows: Rows, f: int, m: int) -> torch.Tensor:
    g = _large_gram(rows)
    if g.is_cuda:
        return large_select(g, f, m)
    return krum_weights_from_gram(g, f, m)


def large_select(g: torch.Tensor, f: int, m: int, bulyan: bool = False) -> torch.Tensor:
    """Multi-Krum weights [n] (or Bulyan's W [t, n]) from a GPU fp32 Gram of up to LARGE_ROWS rows, on
    device (gar_large.hip: per-row neighbourhoods by an LDS bitonic sort, the selection rounds in one
    workgroup; fp64 distances): no host round trip."""
    n = g.shape[0]
    rounds = n - 2 * f - 2 if bulyan else 1
    W = torch.empty((rounds, n), dtype=torch.float32, device=g.device)
    _native.native().gpu_large_select(g.float().contiguous(), f, m, rounds, bulyan, W)
    return W if bulyan else W[0]


def distances_from_gram(g: torch.Tensor) -> torch.Tensor:
    """Squared distances [n, n] from a Gram matrix: +inf on the diagonal and where non-finite."""
    dg = torch.diagonal(g)
    D = (dg[:, None] + dg[None, :] - 2 * g)
    D = torch.where(torch.isfinite(D), D.clamp(min=0), torch.full_like(D, math.inf))
    D.fill_diagonal_(math.inf)
    return D


def krum_weights_from_gram(g: torch.Tensor, f: int, m: int) -> torch.Tensor:
    """Multi-Krum weights [n] (fp32, g's device) from a Gram matrix (vectorised, any n)."""
    n = g.shape[0]
    D = distances_from_gram(g)
    q = n - f - 2
    near = torch.sort(D, dim=1, stable=True).values[:, :q]
    scores = near.sum(1)
    scores = torch.where(torch.isnan(scores), torch.full_like(scores, math.inf), scores)
    order = torch.sort(scores, stable=True).indices
    w = torch.zeros(n, dtype=torch.float32, device=g.device)
    w[order[:m]] = 1.0 / m
    return w


def _stable_order(v: torch.Tensor) -> torch.Tensor:
    """Indices by (value, index), NaN last: reference._order."""
    return torch.sort(_nan_inf(v), stable=True).indices


def _large_bulyan_weights(D: torch.Tensor, f: int, m: int) -> torch.Tensor:
    """reference.bulyan_weights vectorised over n (fp64, CPU: t sequential tiny steps):
    each gradient's q nearest-neighbour distances P, scores = row sums, then t rounds of
    'weights over the mk best scores; remove the best; subtract its column of P'."""
    D = D.double().cpu()
    n = D.shape[0]
    t, q = n - 2 * f - 2, n - f - 2
    Dn = _nan_inf(D.clone())
    Dn.fill_diagonal_(math.inf)
    near = torch.sort(Dn, dim=1, stable=True).indices[:, :q]
    P = torch.zeros((n, n), dtype=torch.float64)
    P.scatter_(1, near, D.gather(1, near))
    scores = P.sum(1)
    W = torch.zeros((t, n), dtype=torch.float64)
    for k in range(t):
        mk = max(m - k, 1)
        order = _stable_order(scores)
        W[k, order[:mk]] = 1.0 / mk
        best = int(order[0])
        scores -= P[:, best]
        scores[best] = ref.FLT_MAX
    return W


def _nan_inf(X: torch.Tensor) -> torch.Tensor:
    return torch.where(torch.isnan(X), torch.full_like(X, math.inf), X)


def _torch_closest_mean(V: torch.Tensor, beta: int) -> torch.Tensor:
    V = torch.sort(_nan_inf(V), dim=0).values
    med = V[V.shape[0] // 2]
    key = _nan_inf((V - med).abs())
    # (key, value) order: stable sort by value first, then by key
    idx = torch.sort(key, dim=0, stable=True).indices
    return torch.gather(V, 0, idx[:beta]).sum(0) / beta


def _torch_coord(X: torch.Tensor, mode: str, f: int, beta: int, seed: int, p: float) -> torch.Tensor:
    n = X.shape[0]
    if mode == "average-nan":
        fin = torch.isfinite(X)
        cnt = fin.sum(0)
        return torch.where(cnt > 0, torch.where(fin, X, 0).sum(0) / cnt.clamp(min=1), torch.zeros_like(X[0]))
    if mode in ("median", "condense"):
        fin = torch.isfinite(X)
        cnt = fin.sum(0)
        S = torch.sort(torch.where(fin, X, torch.full_like(X, math.inf)), dim=0).values
        med = torch.gather(S, 0, (cnt // 2).clamp(max=n - 1)[None]).squeeze(0)
        med = torch.where(cnt > 0, med, torch.zeros_like(med))
        if mode == "condense":
            thr = ref.bernoulli_threshold(p)
            keep = torch.tensor([ref.mix_hash(seed, x) < thr for x in range(X.shape[1])], device=X.device)
            med = torch.where(keep, med, X[0])
        return med
    if mode == "trimmed-mean":
        S = torch.sort(_nan_inf(X), dim=0).values
        return S[f:n - f].sum(0) / (n - 2 * f)
    if mode == "averaged-median":
        return _torch_closest_mean(X, beta)
    raise ValueError(mode)


# --------------------------------------------------------------------------- #

RULES = {
    "average": average,
    "median": median,
    "krum": krum,
    "bulyan": bulyan,
    "brute": brute,
    "aksel": aksel,
    "condense": condense,
    "trimmed-mean": trimmed_mean,
    "averaged-median": averaged_median,
    "average-nan": average_nan,
}


def aggregate(rule: str, gradients, **kwargs) -> torch.Tensor:
    """Apply the named rule (see RULES) to the gradient set."""
    try:
        fn = RULES[rule]
    except KeyError:
        raise KeyError(f"unknown aggregation rule {rule!r}; available: {sorted(RULES)}") from None
    return fn(gradients, **kwargs)
