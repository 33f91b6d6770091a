"""Averaged-median ("MeaMed") GAR (TF reference ``rsrcs/aggregators/averaged-median.py``
-> ``deprecated_native/native.cpp:714-747``): per coordinate, mean of the beta
values closest to the median (beta = n - f by default)."""
from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f=0, beta=None, **kwargs):
    """Coordinate-wise averaged median."""
    return gar.averaged_median(gradients, f=f, beta=beta)


def check(gradients, f=0, beta=None, **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    b = n - f if beta is None else beta
    if not isinstance(b, int) or b < 1 or b > n:
        return f"Invalid number of averaged values beta = {b!r}, expected 1 <= beta <= {n}"
    return None


register("averaged-median", aggregate, check)
