"""Brute GAR: average of the (n - f)-subset with the smallest diameter
(reference: ``aggregators/brute.py:32-140``, native ``py_brute/brute.cpp:47-113``;
here the subset search itself runs on the GPU)."""
from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import accepted_ratio, check_f, check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f, **kwargs):
    """Average of the smallest-diameter subset of n - f gradients."""
    return gar.brute(gradients, f)


def check(gradients, f, **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    return check_f(f, n, lambda f: 2 * f + 1, f"1 <= f <= {(n - 1) // 2}")


def upper_bound(n, f, d):
    return (n - f) / (2 * f)


def influence(honests, attacks, f, **kwargs):
    return accepted_ratio(gar.brute_weights(list(honests) + list(attacks), f), len(honests))


register("brute", aggregate, check, upper_bound, influence)
