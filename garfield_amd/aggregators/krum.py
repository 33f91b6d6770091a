"""Multi-Krum GAR (reference: ``aggregators/krum.py:31-166``; native ``py_krum``).

Semantics are the native / paper ones (squared L2 distances, score over the
n - f - 2 nearest neighbours; the reference's pure-Python variant used the plain
L2 norm and n - f - 1 neighbours — bug B2 in SURVEY.md §7.5)."""
import math

from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import accepted_ratio, check_f, check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f, m=None, **kwargs):
    """Average of the m lowest-scoring gradients (m defaults to n - f - 2)."""
    return gar.krum(gradients, f, m)


def check(gradients, f, m=None, **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    msg = check_f(f, n, lambda f: 2 * f + 3, f"1 <= f <= {(n - 3) // 2}")
    if msg:
        return msg
    if m is not None and (not isinstance(m, int) or m < 1 or m > n - f - 2):
        return f"Invalid number of selected gradients, got m = {m!r}, expected 1 <= m <= {n - f - 2}"
    return None


def upper_bound(n, f, d):
    return 1 / math.sqrt(2 * (n - f + f * (n + f * (n - f - 2) - 2) / (n - 2 * f - 2)))


def influence(honests, attacks, f, m=None, **kwargs):
    w = gar.krum_weights(list(honests) + list(attacks), f, m)
    return accepted_ratio(w, len(honests))


register("krum", aggregate, check, upper_bound, influence)
