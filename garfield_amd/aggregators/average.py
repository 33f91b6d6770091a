"""Average GAR (reference: ``pytorch_impl/libs/aggregators/average.py:21-49``)."""
from garfield_amd.aggregators import register
from garfield_amd.aggregators._common import check_gradients
from garfield_amd.ops import gar


def aggregate(gradients, **kwargs):
    """Arithmetic mean of the gradients."""
    return gar.average(gradients)


def check(gradients, **kwargs):
    return check_gradients(gradients)


def influence(honests, attacks, **kwargs):
    return len(attacks) / (len(honests) + len(attacks))


register("average", aggregate, check, influence=influence)
