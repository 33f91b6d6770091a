"""Coordinate-wise Trimmed-Mean GAR (NEW: absent from the reference, SURVEY.md
§2.2): per coordinate, drop the f smallest and the f largest values (NaN counts
as +inf) and average the remaining n - 2f."""
import math

from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_f, check_gradients, n_of
from garfield_amd.ops import gar


def aggregate(gradients, f, **kwargs):
    """Coordinate-wise trimmed mean."""
    return gar.trimmed_mean(gradients, f)


def check(gradients, f, **kwargs):
    msg = check_gradients(gradients)
    if msg:
        return msg
    n = n_of(gradients)
    return check_f(f, n, lambda f: 2 * f + 1, f"1 <= f <= {(n - 1) // 2}")


def upper_bound(n, f, d):
    return 1 / math.sqrt(n - 2 * f)


register("trimmed-mean", aggregate, check, upper_bound=upper_bound)
