"""Coordinate-wise median GAR (reference: ``aggregators/median.py:31-71``, native
``py_median``): upper median of the finite values of each coordinate, 0 if none."""
import math

from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_gradients
from garfield_amd.ops import gar


def aggregate(gradients, **kwargs):
    """NaN-resilient coordinate-wise median."""
    return gar.median(gradients)


def check(gradients, **kwargs):
    return check_gradients(gradients)


def upper_bound(n, f, d):
    return 1 / math.sqrt(n - f)


register("median", aggregate, check, upper_bound=upper_bound)
