"""Average-NaN GAR (TF reference ``rsrcs/aggregators/average-nan.py`` ->
``deprecated_native/native.cpp:756-782``): mean of the finite values of each
coordinate (0 when none is finite; the reference divides 0 by 0)."""
from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_gradients
from garfield_amd.ops import gar


def aggregate(gradients, **kwargs):
    """NaN-skipping coordinate-wise mean."""
    return gar.average_nan(gradients)


def check(gradients, **kwargs):
    return check_gradients(gradients)


register("average-nan", aggregate, check)
