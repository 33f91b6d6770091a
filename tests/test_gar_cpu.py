"""Native CPU (C++ thread pool) GARs vs the fp64 oracle, and the registry contract."""
import math

import pytest
import torch

from garfield_amd import aggregators
from garfield_amd.ops import gar
from garfield_amd.ops import reference as ref


def separated(n, d, seed=0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(d, generator=g)
    scales = torch.linspace(0.5, 3.0, n)[torch.randperm(n, generator=g)]
    return (base + scales[:, None] * torch.randn(n, d, generator=g)).to(dtype)


def close(a, b, tol=1e-5):
    a, b = a.double(), b.double()
    return (a - b).abs().max().item() <= tol * max(1.0, b.abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n,f", [(7, 2), (12, 3), (20, 8)])
def test_krum_cpu(native, n, f, dtype):
    X = separated(n, 500, n, dtype)
    assert close(gar.krum(X, f), ref.krum(X, f))
    w = gar.krum_weights(X, f)
    assert torch.equal(w != 0, ref.krum_weights(ref.pairwise_sqdist(X), f) != 0)


@pytest.mark.parametrize("n,f", [(7, 1), (15, 3), (19, 4)])
def test_bulyan_cpu(native, n, f):
    X = separated(n, 300, n)
    assert close(gar.bulyan(X, f), ref.bulyan(X, f))


@pytest.mark.parametrize("n,f", [(5, 1), (10, 3)])
def test_brute_cpu(native, n, f):
    X = separated(n, 200, n)
    assert close(gar.brute(X, f), ref.brute(X, f))


@pytest.mark.parametrize("n", [1, 2, 5, 8, 13])
def test_coordinatewise_cpu(native, n):
    X = torch.randn(n, 257)
    X[0, ::7] = math.nan
    if n > 2:
        X[1, ::5] = math.inf
    assert torch.equal(gar.median(X).double(), ref.median(X))
    assert close(gar.average_nan(X), ref.average_nan(X))
    if n >= 3:
        f = (n - 1) // 2
        assert close(gar.trimmed_mean(X, f), ref.trimmed_mean(X, f))
        assert close(gar.averaged_median(X, beta=n - f), ref.averaged_median(X, n - f))
    assert torch.allclose(gar.condense(X, p=0.5, seed=3).double(), ref.condense(X, 0.5, 3), rtol=0, atol=0,
                          equal_nan=True)


def test_aksel_cpu(native):
    X = separated(9, 300, 1)
    for mode in ("mid", "n-f"):
        assert close(gar.aksel(X, 2, mode), ref.aksel(X, 2, mode))


def test_list_and_tensor_inputs_agree(native):
    X = separated(9, 100)
    L = [x.clone() for x in X]
    for rule, kw in [("krum", {"f": 2}), ("median", {}), ("bulyan", {"f": 1}), ("trimmed-mean", {"f": 2})]:
        assert torch.equal(gar.aggregate(rule, X, **kw), gar.aggregate(rule, L, **kw))


def test_bf16_inputs_on_cpu_return_bf16(native):
    X = separated(8, 64).bfloat16()
    out = gar.krum(X, 2)
    assert out.dtype == torch.bfloat16


def test_large_n_cpu_path(native):
    X = separated(140, 50)
    assert torch.equal(gar.median(X).double(), ref.median(X))


# ----------------------------------------------------------------- registry


def test_registry_names():
    names = set(aggregators.gars)
    for base in ["average", "median", "krum", "bulyan", "brute", "aksel", "condense", "trimmed-mean",
                 "average-nan", "averaged-median"]:
        assert base in names and f"native-{base}" in names


def test_registry_attributes_and_checks():
    G = [torch.randn(10) for _ in range(9)]
    krum = aggregators.gars["krum"]
    for attr in ("check", "checked", "unchecked", "upper_bound", "influence"):
        assert hasattr(krum, attr)
    assert krum.check(gradients=G, f=3) is None
    assert krum.check(gradients=G, f=4) is not None
    assert krum.check(gradients=G, f=2, m=6) is not None
    assert aggregators.gars["bulyan"].check(gradients=G, f=2) is not None
    assert aggregators.gars["aksel"].check(gradients=G, f=2, mode="bad") is not None
    with pytest.raises(aggregators.UserException):
        krum(gradients=G, f=5)


def test_rules_ignore_unknown_kwargs_and_never_alias():
    G = [torch.randn(16) for _ in range(9)]
    for name in ["average", "median", "krum", "bulyan", "brute", "aksel", "condense", "trimmed-mean",
                 "average-nan", "averaged-median"]:
        out = aggregators.gars[name](gradients=G, f=1, unknown_flag=True)
        assert out.shape == (16,)
        assert all(out.data_ptr() != g.data_ptr() for g in G)


def test_influence():
    honest = [torch.randn(32) * 0.1 for _ in range(7)]
    attacks = [torch.full((32,), 50.0), torch.full((32,), -50.0)]
    assert aggregators.gars["krum"].influence(honest, attacks, f=2) == 0.0
    assert aggregators.gars["average"].influence(honest, attacks) == pytest.approx(2 / 9)
    assert aggregators.gars["brute"].influence(honest, attacks, f=2) == 0.0


def test_upper_bounds():
    assert aggregators.gars["krum"].upper_bound(9, 2, 100) == pytest.approx(
        1 / math.sqrt(2 * (9 - 2 + 2 * (9 + 2 * (9 - 2 - 2) - 2) / (9 - 4 - 2))))
    assert aggregators.gars["median"].upper_bound(9, 2, 100) == pytest.approx(1 / math.sqrt(7))
    assert aggregators.gars["brute"].upper_bound(9, 2, 100) == pytest.approx(7 / 4)


def test_brute_rejects_more_than_2_pow_32_subsets():
    """The device search ranks subsets with a 32-bit key: C(n, n - f) > 2^32 is refused
    loudly (n = 64: f = 7 is 621M subsets, f = 8 is 4.4e9)."""
    import pytest as _pytest

    from garfield_amd.ops import gar as _gar

    with _pytest.raises(ValueError, match="2\\^32"):
        _gar.brute_weights(torch.randn(64, 16), 8)
    assert _gar.BRUTE_MAX_SUBSETS == 2 ** 32


@pytest.mark.parametrize("n,f", [(20, 3), (45, 5), (140, 10)])
def test_large_bulyan_selection_equals_reference(n, f):
    """The vectorised selection of large sets (n > MAX_ROWS on the GPU path) reproduces
    reference.bulyan_weights exactly, NaN rows and ties included."""
    from garfield_amd.ops import gar as _gar
    from garfield_amd.ops import reference as _ref

    g = torch.Generator().manual_seed(n)
    X = torch.randint(-3, 4, (n, 30), generator=g).double()
    X[:f] += 5
    X[f, 0] = float("nan")
    D = _ref.pairwise_sqdist(X)
    assert torch.equal(_gar._large_bulyan_weights(D, f, n - f - 2), _ref.bulyan_weights(D, f, n - f - 2))
