"""TF graph-mode class registry (reference tensorflow_impl/rsrcs/aggregators/__init__.py:38-74):
every registered name instantiates and matches the functional rule it wraps."""
import pytest
import torch

from garfield_amd import aggregators
from garfield_amd.aggregators import classreg
from garfield_amd.utils.logging import UserException


def _grads(n=11, shape=(3, 5)):
    torch.manual_seed(0)
    return [torch.randn(shape) for _ in range(n)]


def test_itemize_names():
    names = set(aggregators.itemize())
    for want in ("average", "average-nan", "averaged-median", "median", "krum", "krum-py", "krum-tf",
                 "bulyan", "bulyan-py", "condense", "trimmed-mean"):
        assert want in names


@pytest.mark.parametrize("name", ["average", "average-nan", "median", "krum", "krum-tf", "krum-py",
                                  "bulyan", "bulyan-py", "trimmed-mean", "averaged-median"])
def test_matches_functional_rule(name):
    g = _grads()
    n, f = len(g), 2
    gar = aggregators.instantiate(name, n, f, None)
    out = gar.aggregate(g)
    assert out.shape == g[0].shape
    flat = torch.stack([x.reshape(-1) for x in g])
    kw = {}
    if name.startswith("krum"):
        kw["m"] = n - f - 2
    if name == "averaged-median":
        kw["beta"] = n - f
    ref = aggregators.gars[classreg._register._register[name].rule_name](gradients=flat, f=f, **kw)
    torch.testing.assert_close(out.reshape(-1), ref)
    # stacked input gives the same result
    torch.testing.assert_close(gar.aggregate(flat).reshape(-1), ref)


def test_krum_m_and_condense_args():
    g = _grads()
    out = aggregators.instantiate("krum", 11, 2, ["m:1"]).aggregate(g)
    flat = torch.stack([x.reshape(-1) for x in g])
    assert any(torch.allclose(out.reshape(-1), row) for row in flat)   # m=1 selects one gradient
    c = aggregators.instantiate("condense", 11, 2, ["ps:1.0"]).aggregate(g)
    torch.testing.assert_close(c.reshape(-1), aggregators.gars["median"](gradients=flat, f=2))
    with pytest.raises(UserException):
        aggregators.instantiate("condense", 11, 2, ["ps:0"])
    with pytest.raises(UserException):
        aggregators.instantiate("nope", 11, 2, None)
