"""Aksel GAR (reference: ``aggregators/aksel.py:24-105``): average of the c
gradients closest (squared L2) to the coordinate-wise median, c = (n+1)//2
(``mode="mid"``) or n - f (``mode="n-f"``)."""
from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import accepted_ratio, check_f, check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f, mode="mid", **kwargs):
    """Aksel aggregation."""
    return gar.aksel(gradients, f, mode)


def check(gradients, f, mode="mid", **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    msg = check_f(f, n, lambda f: 2 * f + 1, f"1 <= f <= {(n - 1) // 2}")
    if msg:
        return msg
    if mode not in ("mid", "n-f"):
        return f"Invalid operation mode {mode!r}"
    return None


def influence(honests, attacks, f, mode="mid", **kwargs):
    return accepted_ratio(gar.aksel_weights(list(honests) + list(attacks), f, mode), len(honests))


register("aksel", aggregate, check, influence=influence)
