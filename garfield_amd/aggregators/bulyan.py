"""Bulyan over Multi-Krum (reference: native ``py_bulyan/bulyan.cpp:53-193``; the
pure-Python ``aggregators/bulyan.py`` is broken, bug B1).

t = n - 2f - 2 Krum selection rounds with pruned-score updates build a t x n
weight matrix W; each coordinate of W·G is then reduced by the averaged median
of its b = t - 2f values closest to the median."""
import math

from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_f, check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f, m=None, **kwargs):
    """Bulyan aggregation (m defaults to n - f - 2)."""
    return gar.bulyan(gradients, f, m)


def check(gradients, f, m=None, **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    msg = check_f(f, n, lambda f: 4 * f + 3, f"1 <= f <= {(n - 3) // 4}")
    if msg:
        return msg
    if m is not None and (not isinstance(m, int) or m < 1 or m > n - f - 2):
        return f"Invalid number of selected gradients, got m = {m!r}, expected 1 <= m <= {n - f - 2}"
    return None


def upper_bound(n, f, d):
    return 1 / math.sqrt(2 * (n - f + f * (n + f * (n - f - 2) - 2) / (n - 2 * f - 2)))


def influence(honests, attacks, f, m=None, **kwargs):
    """Share of Byzantine weight in the Krum selections feeding the coordinate phase."""
    W = gar.bulyan_weights(list(honests) + list(attacks), f, m).float().cpu()
    tot = float(W.sum())
    return float(W[:, len(honests):].sum()) / tot if tot else 0.0


register("bulyan", aggregate, check, upper_bound, influence)
