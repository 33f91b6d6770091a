"""Plain-PyTorch fp64 reference ("oracle") implementations of every GAR.

These are the specification the native CPU and HIP kernels are tested against
(SURVEY.md §4 "GAR oracle tests"), written for clarity, not speed. They follow
the native-reference semantics documented in ``docs/GAR_SEMANTICS.md``:

* distances are SQUARED L2 (``py_krum/krum.cu:92-94``), non-finite -> +inf;
* Krum score = sum of the ``n - f - 2`` nearest (``py_krum/krum.cpp:86-97``);
* every ranking is by ``(value with NaN as +inf, index)``;
* median = upper median of the finite values, 0 if none (``py_median/median.cpp:42-77``);
* Bulyan follows ``py_bulyan/bulyan.cpp:53-193`` (pruned-score selection loop,
  then averaged-median with beta = t - 2f);
* Brute enumerates (n-f)-subsets as bit masks in increasing numeric order.

All functions take ``G`` as an ``[n, d]`` tensor (any dtype / device) and return
a 1-D fp64 CPU tensor unless stated otherwise.
"""
from __future__ import annotations

import math
from itertools import combinations

import torch

FLT_MAX = 3.4028234663852886e38
_MASK64 = (1 << 64) - 1


def _g(G) -> torch.Tensor:
    if isinstance(G, (list, tuple)):
        G = torch.stack([g.reshape(-1) for g in G])
    return G.detach().to(device="cpu", dtype=torch.float64)


def _key(v: float) -> float:
    return math.inf if v != v else v


def _order(values, ids=None):
    ids = list(range(len(values))) if ids is None else list(ids)
    return sorted(ids, key=lambda i: (_key(float(values[i])), i))


def pairwise_sqdist(G) -> torch.Tensor:
    X = _g(G)
    n = X.shape[0]
    D = torch.full((n, n), math.inf, dtype=torch.float64)
    for i in range(n):
        for j in range(i + 1, n):
            v = float(((X[i] - X[j]) ** 2).sum())
            if not math.isfinite(v):
                v = math.inf
            D[i, j] = D[j, i] = v
    return D


def krum_scores(D: torch.Tensor, f: int) -> list[float]:
    n = D.shape[0]
    q = n - f - 2
    scores = []
    for i in range(n):
        near = _order(D[i].tolist(), [j for j in range(n) if j != i])[:q]
        scores.append(sum(float(D[i, j]) for j in near))
    return scores


def krum_weights(D: torch.Tensor, f: int, m: int | None = None) -> torch.Tensor:
    n = D.shape[0]
    m = n - f - 2 if m is None else m
    order = _order(krum_scores(D, f))
    w = torch.zeros(n, dtype=torch.float64)
    for i in order[:m]:
        w[i] = 1.0 / m
    return w


def combine(G, w: torch.Tensor) -> torch.Tensor:
    X = _g(G)
    out = torch.zeros(X.shape[1], dtype=torch.float64)
    for j in range(X.shape[0]):
        if float(w[j]) != 0.0:
            out += float(w[j]) * X[j]
    return out


def average(G) -> torch.Tensor:
    return _g(G).mean(dim=0)


def krum(G, f: int, m: int | None = None) -> torch.Tensor:
    return combine(G, krum_weights(pairwise_sqdist(G), f, m))


def bulyan_weights(D: torch.Tensor, f: int, m: int | None = None) -> torch.Tensor:
    n = D.shape[0]
    m = n - f - 2 if m is None else m
    t = n - 2 * f - 2
    q = n - f - 2
    scores, P = [], torch.zeros((n, n), dtype=torch.float64)
    for i in range(n):
        near = _order(D[i].tolist(), [j for j in range(n) if j != i])[:q]
        scores.append(sum(float(D[i, j]) for j in near))
        for j in near:
            P[i, j] = D[i, j]
    W = torch.zeros((t, n), dtype=torch.float64)
    for k in range(t):
        mk = max(m - k, 1)
        order = _order(scores)
        for i in order[:mk]:
            W[k, i] = 1.0 / mk
        best = order[0]
        for i in range(n):
            if i != best:
                scores[i] -= float(P[i, best])
        scores[best] = FLT_MAX
    return W


def _closest_mean(vals: list[float], beta: int) -> float:
    s = sorted(_key(v) for v in vals)
    med = s[len(s) // 2]
    kv = sorted((_key(abs(v - med)), v) for v in s)
    return sum(v for _, v in kv[:beta]) / beta


def bulyan(G, f: int, m: int | None = None) -> torch.Tensor:
    X = _g(G)
    n = X.shape[0]
    t = n - 2 * f - 2
    beta = t - 2 * f
    W = bulyan_weights(pairwise_sqdist(X), f, m)
    V = W @ X  # [t, d]
    return torch.tensor([_closest_mean(V[:, x].tolist(), beta) for x in range(X.shape[1])], dtype=torch.float64)


def median(G) -> torch.Tensor:
    X = _g(G)
    out = torch.zeros(X.shape[1], dtype=torch.float64)
    for x in range(X.shape[1]):
        v = sorted(a for a in X[:, x].tolist() if math.isfinite(a))
        out[x] = v[len(v) // 2] if v else 0.0
    return out


def trimmed_mean(G, f: int) -> torch.Tensor:
    X = _g(G)
    n = X.shape[0]
    out = torch.zeros(X.shape[1], dtype=torch.float64)
    for x in range(X.shape[1]):
        v = sorted(_key(a) for a in X[:, x].tolist())
        out[x] = sum(v[f:n - f]) / (n - 2 * f)
    return out


def averaged_median(G, beta: int) -> torch.Tensor:
    X = _g(G)
    return torch.tensor([_closest_mean(X[:, x].tolist(), beta) for x in range(X.shape[1])], dtype=torch.float64)


def average_nan(G) -> torch.Tensor:
    X = _g(G)
    fin = torch.isfinite(X)
    cnt = fin.sum(0)
    s = torch.where(fin, X, torch.zeros_like(X)).sum(0)
    return torch.where(cnt > 0, s / cnt.clamp(min=1), torch.zeros_like(s))


def mix_hash(seed: int, x: int) -> int:
    """Bit-exact Python twin of ``garfield::mix_hash`` (csrc/gar_common.hpp)."""
    z = (seed * 0x9E3779B97F4A7C15 + x + 0x632BE59BD9B4E019) & _MASK64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    z ^= z >> 31
    return z >> 32


def bernoulli_threshold(p: float) -> int:
    if p >= 1.0:
        return 1 << 32
    if p <= 0.0:
        return 0
    return int(p * 4294967296.0)


def condense(G, p: float, seed: int) -> torch.Tensor:
    X = _g(G)
    med = median(X)
    thr = bernoulli_threshold(p)
    out = med.clone()
    for x in range(X.shape[1]):
        if not mix_hash(seed, x) < thr:
            out[x] = X[0, x]
    return out


def brute_weights(D: torch.Tensor, f: int) -> torch.Tensor:
    n = D.shape[0]
    k = n - f
    Df = torch.where(torch.isfinite(D), D.clamp(min=0), torch.full_like(D, FLT_MAX)).float().double()
    best, best_mask = None, None
    # numeric order of k-bit masks == colexicographic order of the subsets
    subsets = sorted(combinations(range(n), k), key=lambda c: sum(1 << i for i in c))
    for c in subsets:
        diam = 0.0
        for a, b in combinations(c, 2):
            diam = max(diam, float(Df[a, b]))
        if best is None or diam < best:
            best, best_mask = diam, c
    w = torch.zeros(n, dtype=torch.float64)
    for i in best_mask:
        w[i] = 1.0 / k
    return w


def brute(G, f: int) -> torch.Tensor:
    return combine(G, brute_weights(pairwise_sqdist(G), f))


def aksel(G, f: int, mode: str = "mid") -> torch.Tensor:
    X = _g(G)
    n = X.shape[0]
    med = median(X)
    dist = [((X[j] - med) ** 2).sum().item() for j in range(n)]
    dist = [d if math.isfinite(d) else math.inf for d in dist]
    c = (n + 1) // 2 if mode == "mid" else n - f
    w = torch.zeros(n, dtype=torch.float64)
    for j in _order(dist)[:c]:
        w[j] = 1.0 / c
    return combine(X, w)
