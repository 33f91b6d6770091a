"""Large gradient sets (128 < n <= 1024) on the GPU kernels of gar_large.hip, against the
vectorised fp64 PyTorch semantics of ops/gar.py (ties and non-finite values included)."""
import math

import pytest
import torch

from garfield_amd.ops import gar
from garfield_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _data(n, d, dtype, seed, ties=True, nonfinite=True):
    g = torch.Generator().manual_seed(seed)
    if ties:   # few distinct values: every tie rule is exercised
        X = torch.randint(-24, 25, (n, d), generator=g).double() / 8.0
    else:
        X = torch.randn(n, d, generator=g, dtype=torch.float64)
    if nonfinite:
        X[torch.rand(n, d, generator=g) < 0.01] = math.nan
        X[torch.rand(n, d, generator=g) < 0.005] = math.inf
        X[torch.rand(n, d, generator=g) < 0.005] = -math.inf
    return X.to(dtype)


def _close(a, b, tol):
    a, b = a.double().cpu(), b.double().cpu()
    same_nonfinite = (torch.isnan(a) == torch.isnan(b)) & ((a == b) | torch.isnan(a) | torch.isfinite(a))
    fin = torch.isfinite(a) & torch.isfinite(b)
    assert bool(same_nonfinite.all()), "non-finite pattern differs"
    err = ((a - b).abs()[fin] / (1 + b.abs()[fin])).max().item() if fin.any() else 0.0
    assert err <= tol, err


@pytest.mark.parametrize("n", [129, 256, 512, 1024])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_large_coordinate_rules(cuda, n, dtype):
    d = 3000
    X = _data(n, d, dtype, n)
    Xd = X.double()
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    _close(gar.median(X.to(cuda)), gar._torch_coord(Xd, "median", 0, 0, 0, 1.0), tol)
    f = n // 5
    _close(gar.trimmed_mean(X.to(cuda), f=f), gar._torch_coord(Xd, "trimmed-mean", f, 0, 0, 1.0), tol)
    beta = n - f
    _close(gar.averaged_median(X.to(cuda), beta=beta), gar._torch_closest_mean(Xd, beta), tol)


@pytest.mark.parametrize("n", [200, 700])
def test_large_combine_and_average(cuda, n):
    X = _data(n, 5000, torch.bfloat16, 3, ties=False, nonfinite=False)
    w = torch.rand(n, dtype=torch.float64)
    w[torch.rand(n) < 0.5] = 0
    out = gar.combine(X.to(cuda), w.float())
    _close(out, w @ X.double(), 1e-2)
    _close(gar.average(X.to(cuda)), X.double().mean(0), 1e-2)


def test_large_krum_and_bulyan_selections(cuda):
    n, f, d = 160, 10, 4000
    g = torch.Generator().manual_seed(5)
    X = torch.randn(n, d, generator=g, dtype=torch.float64)
    X[:f] += 50.0                      # f far-away (Byzantine) rows
    Xg = X.float().to(cuda)
    w = gar.krum_weights(Xg, f)
    wref = ref.krum_weights(ref.pairwise_sqdist(X), f, n - f - 2)
    assert torch.equal((w.cpu() > 0), (wref > 0))
    _close(gar.krum(Xg, f), wref @ X, 1e-5)
    out = gar.bulyan(Xg, f)
    _close(out, ref.bulyan(X, f, n - f - 2), 1e-4)


@pytest.mark.parametrize("n,f", [(256, 20), (1024, 50), (129, 1)])
def test_large_select_on_device_matches_fp64_reference(cuda, n, f):
    """gar_large.hip's device selection (per-row neighbourhoods by LDS bitonic sort, the rounds in one
    workgroup) == the fp64 reference selection from the same Gram (ops/reference.py semantics),
    Multi-Krum weights and every Bulyan round's W row."""
    g = torch.Generator().manual_seed(n)
    X = torch.randn(n, 2000, generator=g, dtype=torch.float64)
    X[:f] *= 30.0
    G = (X.float().to(cuda) @ X.float().to(cuda).T).contiguous()
    D = gar.distances_from_gram(G.double()).cpu()
    m = n - f - 2
    w = gar.large_select(G, f, m)
    assert torch.equal(w.cpu(), ref.krum_weights(D, f, m).float())
    W = gar.large_select(G, f, m, bulyan=True)
    assert W.shape == (n - 2 * f - 2, n)
    assert torch.equal(W.cpu(), gar._large_bulyan_weights(D, f, m).float())


@pytest.mark.parametrize("rule", ["bulyan", "krum"])
def test_engine_n256_on_device(cuda, monkeypatch, rule):
    """n = 256 logical workers on one GPU (what 8 GPUs x 32 workers aggregate): the redundant
    (_large_update) and sharded (_gpu_large) paths select on device -- a host copy of any GPU tensor
    during the aggregation fails the test --; redundant == the fp64 reference rule on the same rows,
    sharded == redundant."""
    import torch.nn.functional as F

    from garfield_amd.models import build_model
    from garfield_amd.parallel.comm import DistContext
    from garfield_amd.parallel.engine import EngineConfig, RobustDataParallel, synthetic_batches

    n, f = 256, 20
    real_cpu = torch.Tensor.cpu

    def no_host_copy(t, *a, **k):
        if t.is_cuda:
            raise AssertionError("host copy in the n > 128 aggregation")
        return real_cpu(t, *a, **k)

    deltas = []
    for shard in (False, True):
        torch.manual_seed(0)
        eng = RobustDataParallel(build_model("mlp"), F.nll_loss, DistContext(device=cuda),
                                 EngineConfig(gar=rule, f=f, workers_per_rank=n, byzantine={5: "reverse", 77: "reverse"},
                                              lr=0.1, momentum=0.0, weight_decay=0.0, exchange_dtype=torch.float32,
                                              shard_gar=shard, cuda_graph=False))
        assert (eng._shard is not None) == shard
        eng.compute_local(synthetic_batches(n, 4, (1, 28, 28), 10, cuda))
        before = eng.flat.data[: eng.d].clone()
        G = None if shard else eng.G[:, : eng.d].double().cpu()
        monkeypatch.setattr(torch.Tensor, "cpu", no_host_copy)
        eng.aggregate_and_update()
        torch.cuda.synchronize()
        monkeypatch.setattr(torch.Tensor, "cpu", real_cpu)
        deltas.append(((before - eng.flat.data[: eng.d]) / 0.1).double().cpu())
        if G is not None:
            want = ref.bulyan(G, f, n - f - 2) if rule == "bulyan" else ref.krum(G, f, n - f - 2)
            assert ((deltas[-1] - want).norm() / want.norm()).item() < 1e-5
    assert ((deltas[1] - deltas[0]).norm() / deltas[0].norm()).item() < 1e-6


@pytest.mark.parametrize("n,d,dtype", [(129, 5000, torch.bfloat16), (256, 100000, torch.bfloat16),
                                       (1024, 20000, torch.bfloat16), (300, 7777, torch.float32),
                                       (512, 3001, torch.float16)])
def test_large_gram_mfma_matches_fp64(cuda, n, d, dtype):
    """gar_large.hip's split-K MFMA Gram (64 x 64 tiles, fixed-order slab sums; rows not a multiple of
    64, d not a multiple of the k-step) against the fp64 Gram of the same (rounded) rows."""
    g = torch.Generator().manual_seed(n + d)
    X = torch.randn(n, d, generator=g, dtype=torch.float64).to(dtype)
    G = gar.large_gram(X.to(cuda))
    ref_g = X.double() @ X.double().T
    assert G.shape == (n, n)
    err = ((G.double().cpu() - ref_g).abs() / (ref_g.abs() + d ** 0.5)).max().item()
    assert err < 1e-4, err
    assert torch.equal(G.cpu(), G.cpu().T)


@pytest.mark.parametrize("t,n,d,dtype", [(252, 256, 40000, torch.bfloat16), (70, 129, 1000, torch.float32),
                                         (1000, 1024, 3000, torch.bfloat16)])
def test_large_wx_mfma_matches_fp64(cuda, t, n, d, dtype):
    """V = W · X on fp32 MFMA (Bulyan's selection means) against fp64, W with 1/mk weights."""
    g = torch.Generator().manual_seed(t + n)
    X = torch.randn(n, d, generator=g, dtype=torch.float64).to(dtype)
    W = torch.zeros(t, n, dtype=torch.float64)
    for k in range(t):
        mk = max(n // 2 - k, 1)
        W[k, torch.randperm(n, generator=g)[:mk]] = 1.0 / mk
    V = gar.large_wx(W.float().to(cuda), X.to(cuda))
    ref_v = W.float().double() @ X.double()
    err = ((V.double().cpu() - ref_v).abs() / (ref_v.abs() + 1.0)).max().item()
    assert err < 1e-5, err
