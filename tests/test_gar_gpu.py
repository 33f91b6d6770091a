"""HIP GAR kernels vs the fp64 PyTorch oracle (garfield_amd/ops/reference.py).

Every kernel is compared against a plain fp64 reference of the same op on the
same (dtype-rounded) inputs; selection rules must pick exactly the oracle's set
on inputs with well-separated distances."""
import math

import pytest
import torch

from garfield_amd.ops import gar
from garfield_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DTYPES = [torch.float32, torch.bfloat16, torch.float16]
TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 2e-3}


def separated(n, d, dtype, dev, seed=0):
    """Rows with clearly distinct pairwise distances (distinct per-row noise scales)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(d, generator=g)
    scales = torch.linspace(0.5, 3.0, n)[torch.randperm(n, generator=g)]
    X = base + scales[:, None] * torch.randn(n, d, generator=g)
    return X.to(dtype).to(dev)


def close(a, b, dtype, scale=1.0):
    a = a.double().cpu()
    b = b.double().cpu()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    return err <= TOL[dtype] * max(scale, b.abs().max().item(), 1.0)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,d", [(1, 100), (7, 1000), (16, 4096), (17, 5003), (33, 1000), (64, 777), (100, 300)])
def test_gram(cuda, n, d, dtype):
    X = separated(n, d, dtype, cuda)
    g = gar.gram(X)
    Xd = X.double().cpu()
    assert close(g, Xd @ Xd.T, dtype, scale=float((Xd * Xd).sum(1).max()))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,f", [(7, 2), (8, 2), (15, 3), (16, 6), (33, 5), (64, 2), (128, 10)])
def test_krum_selection_and_output(cuda, n, f, dtype):
    X = separated(n, 2000, dtype, cuda, seed=n)
    w = gar.krum_weights(X, f).cpu()
    w_ref = ref.krum_weights(ref.pairwise_sqdist(X), f).float()
    assert torch.equal(w != 0, w_ref != 0)
    out = gar.krum(X, f)
    assert out.dtype == dtype
    assert close(out, ref.krum(X, f), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,f", [(7, 1), (11, 2), (15, 3), (23, 5), (26, 2), (31, 7), (33, 5), (35, 8), (40, 1),
                                 (64, 3)])
def test_bulyan(cuda, n, f, dtype):
    X = separated(n, 1500, dtype, cuda, seed=100 + n)
    W = gar.bulyan_weights(X, f).cpu()
    W_ref = ref.bulyan_weights(ref.pairwise_sqdist(X), f).float()
    assert torch.equal(W != 0, W_ref != 0)
    assert close(gar.bulyan(X, f), ref.bulyan(X, f), dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n,f", [(26, 2), (40, 1), (64, 3), (16, 3)])
def test_bulyan_tail_nonfinite_rows_take_exact_pass(cuda, n, f, dtype):
    """inf / NaN in a row that Krum never selects: the MFMA set sums of those
    64-coordinate groups turn NaN (0 * inf), so the groups go through the exact
    per-set pass (fp32: the register kernel's weighted sums likewise, per lane); the result
    must equal set means taken by indexing (fp64 oracle)."""
    d = 64 * 40 + 37
    X = separated(n, d, torch.float32, "cpu", seed=n)
    cols = torch.arange(3, d, 97)
    X[0, cols] = torch.tensor([math.inf, -math.inf, math.nan])[torch.arange(cols.numel()) % 3]
    X = X.to(dtype)
    Xc = X.to(cuda)
    W = gar.bulyan_weights(Xc, f).cpu().double()
    assert (W[:, 0] == 0).all()
    t, beta = n - 2 * f - 2, n - 4 * f - 2
    V = torch.stack([X.double()[W[k] != 0].mean(0) for k in range(t)])
    want = torch.tensor([ref._closest_mean(V[:, x].tolist(), beta) for x in range(d)])
    assert close(gar.bulyan(Xc, f), want, dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,f", [(5, 1), (9, 2), (12, 3), (20, 4)])
def test_brute(cuda, n, f, dtype):
    X = separated(n, 800, dtype, cuda, seed=7 * n)
    w = gar.brute_weights(X, f).cpu()
    w_ref = ref.brute_weights(ref.pairwise_sqdist(X), f).float()
    assert torch.equal(w != 0, w_ref != 0)
    assert close(gar.brute(X, f), ref.brute(X, f), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [1, 2, 3, 7, 8, 9, 16, 17, 32, 33, 64, 65, 128])
@pytest.mark.parametrize("d", [1, 13, 4099])
def test_median(cuda, n, d, dtype):
    X = torch.randn(n, d).to(dtype).to(cuda)
    assert torch.equal(gar.median(X).double().cpu(), ref.median(X).to(dtype).double())


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,f", [(3, 1), (8, 1), (9, 4), (16, 3), (31, 10), (64, 20), (100, 30)])
def test_trimmed_mean(cuda, n, f, dtype):
    X = torch.randn(n, 3001).to(dtype).to(cuda)
    assert close(gar.trimmed_mean(X, f), ref.trimmed_mean(X, f), dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,beta", [(5, 3), (8, 6), (16, 12), (33, 20)])
def test_averaged_median(cuda, n, beta, dtype):
    X = torch.randn(n, 2001).to(dtype).to(cuda)
    assert close(gar.averaged_median(X, beta=beta), ref.averaged_median(X, beta), dtype)


@pytest.mark.parametrize("n", [4, 9, 40])
def test_average_nan_and_nonfinite(cuda, n):
    X = torch.randn(n, 1000)
    X[0, ::3] = math.nan
    X[1, ::5] = math.inf
    X[2, :7] = -math.inf
    Xc = X.to(cuda)
    assert close(gar.average_nan(Xc), ref.average_nan(X), torch.float32)
    assert torch.equal(gar.median(Xc).cpu().double(), ref.median(X))


def test_median_all_nonfinite_is_zero(cuda):
    X = torch.full((5, 64), math.nan, device=cuda)
    assert torch.equal(gar.median(X).cpu(), torch.zeros(64))


@pytest.mark.parametrize("dtype", DTYPES)
def test_condense_mask_matches_oracle(cuda, dtype):
    X = torch.randn(9, 5000).to(dtype).to(cuda)
    out = gar.condense(X, p=0.6, seed=12345)
    assert torch.allclose(out.double().cpu(), ref.condense(X, 0.6, 12345).to(dtype).double(), rtol=0, atol=0,
                          equal_nan=True)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("mode", ["mid", "n-f"])
def test_aksel(cuda, dtype, mode):
    X = separated(11, 3000, dtype, cuda, seed=3)
    assert close(gar.aksel(X, 2, mode), ref.aksel(X, 2, mode), dtype)


def test_krum_rejects_nonfinite_and_byzantine(cuda):
    X = separated(10, 5000, torch.float32, cuda)
    X[3] = math.nan
    X[8] = -100 * X[8]
    w = gar.krum_weights(X, 2).cpu()
    assert w[3] == 0 and w[8] == 0


def test_list_input_and_unaligned_views(cuda):
    X = separated(9, 1001, torch.bfloat16, cuda)
    L = [X[i] for i in range(9)]        # row views with odd strides (misaligned)
    assert close(gar.krum(L, 2), ref.krum(X, 2), torch.bfloat16)
    assert torch.equal(gar.median(L).cpu(), gar.median(X).cpu())


@pytest.mark.parametrize("nesterov", [False, True])
def test_fused_combine_sgd_matches_torch_sgd(cuda, native, nesterov):
    n, d = 8, 10007
    X = torch.randn(n, 10016, device=cuda)[:, :d]   # padded row stride (16-byte aligned rows)
    w = torch.zeros(n, device=cuda)
    w[[1, 3, 4]] = 1 / 3
    p0 = torch.randn(d, device=cuda)
    param, mom = p0.clone(), torch.zeros(d, device=cuda)
    ref_p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.SGD([ref_p], lr=0.1, momentum=0.9, weight_decay=5e-4, nesterov=nesterov)
    for step in range(3):
        native.gpu_combine_sgd(X, w, param, mom, None, None, 0.1, 0.9, 0.0, 5e-4, nesterov, step == 0)
        ref_p.grad = (w[:, None] * X).sum(0)
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(param, ref_p.detach(), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("sdt", [torch.bfloat16, torch.float16])
def test_combine_sgd_writes_shadow(cuda, native, sdt):
    n, d = 8, 10007
    X = torch.randn(n, 10016, device=cuda, dtype=torch.bfloat16)[:, :d]   # 16-byte aligned rows
    w = torch.full((n,), 1 / n, device=cuda)
    param, mom = torch.randn(d, device=cuda), torch.zeros(d, device=cuda)
    shadow = torch.zeros(d + 9, device=cuda, dtype=sdt)
    native.gpu_combine_sgd(X, w, param, mom, None, shadow, 0.1, 0.9, 0.0, 5e-4, False, True)
    torch.cuda.synchronize()
    assert torch.equal(shadow[:d], param.to(sdt))
    assert torch.equal(shadow[d:], torch.zeros(9, device=cuda, dtype=sdt))


def test_large_n_fallback_matches_oracle(cuda):
    X = separated(130, 257, torch.float32, cuda)
    assert close(gar.median(X), ref.median(X), torch.float32)
    w = gar.krum_weights(X, 3).cpu()
    w_ref = ref.krum_weights(ref.pairwise_sqdist(X), 3).float()
    assert torch.equal(w != 0, w_ref != 0)


def test_deterministic_replicas(cuda):
    """Two runs on identical inputs give bitwise-identical results (replica consistency)."""
    X = torch.randn(16, 100003, device=cuda, dtype=torch.bfloat16)
    a = gar.krum(X, 3)
    b = gar.krum(X.clone(), 3)
    assert torch.equal(a, b)
    assert torch.equal(gar.bulyan(X, 3), gar.bulyan(X.clone(), 3))


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32, torch.float16])
def test_flatten_cast_matches_cat(cuda, native, odt):
    torch.manual_seed(0)
    shapes = [(64, 3, 7, 7), (10,), (3,), (512, 256, 3, 3), (1,), (130, 7)] * 20  # > 96 tensors: 2 launches
    ts = [torch.randn(s, device=cuda) for s in shapes]
    ts[0] = ts[0].contiguous(memory_format=torch.channels_last)
    total = sum(t.numel() for t in ts)
    dst = torch.zeros(total + 5, device=cuda, dtype=odt)
    native.gpu_flatten_cast(ts, dst)
    from garfield_amd.utils.flat import memory_order_flat
    ref_ = torch.cat([memory_order_flat(t) for t in ts]).to(odt)
    torch.cuda.synchronize()
    assert torch.equal(dst[:total], ref_)
    assert torch.equal(dst[total:], torch.zeros(5, device=cuda, dtype=odt))


@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_flatten_cast_mixed_source_dtypes(cuda, native, odt):
    torch.manual_seed(1)
    shapes = [(64, 3, 7, 7), (10,), (3,), (256, 64, 3, 3), (1,), (130, 7), (7,)]
    dts = [torch.bfloat16, torch.float32, torch.float16, torch.bfloat16, torch.float32, torch.bfloat16, torch.bfloat16]
    ts = [torch.randn(s, device=cuda).to(dt) for s, dt in zip(shapes, dts)]
    total = sum(t.numel() for t in ts)
    dst = torch.zeros(total, device=cuda, dtype=odt)
    native.gpu_flatten_cast(ts, dst)
    ref_ = torch.cat([t.reshape(-1).float() for t in ts]).to(odt)
    torch.cuda.synchronize()
    assert torch.equal(dst, ref_)


@pytest.mark.parametrize("name", ["krum-tf", "bulyan-py", "median", "averaged-median", "trimmed-mean"])
def test_class_interface_on_device(cuda, name):
    """TF graph-mode class interface (aggregators.instantiate) on bf16 device gradients:
    runs the HIP rules and matches the fp64 oracle of the same rule."""
    from garfield_amd import aggregators

    n, f, d = 15, 3, 70001
    torch.manual_seed(5)
    g = torch.randn(n, d, dtype=torch.float64)
    g[:f] *= -20.0
    dev = [row.to(cuda, torch.bfloat16) for row in g]
    out = aggregators.instantiate(name, n, f, None).aggregate(dev)
    assert out.device.type == "cuda" and out.shape == (d,)
    base = name.split("-")[0] if name in ("krum-tf", "bulyan-py") else name
    kw = {"m": n - f - 2} if base == "krum" else {"beta": n - f} if base == "averaged-median" else {}
    want = aggregators.gars[base](gradients=torch.stack([r.double().cpu() for r in dev]), f=f, **kw)
    err = (out.double().cpu() - want).norm() / want.norm()
    assert err < 1e-2, err


def _nonfinite_rows(n, d, dtype, seed):
    """Random rows with NaN / +inf / -inf sprinkled over a few coordinates (and
    whole rows of them in others), so the packed-key kernels' exact fallback runs."""
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, d, generator=g)
    cols = torch.randperm(d, generator=g)[: max(d // 50, 3)]
    for k, c in enumerate(cols.tolist()):
        r = torch.randperm(n, generator=g)[: 1 + k % max(n // 3, 1)]
        X[r, c] = (math.nan, math.inf, -math.inf)[k % 3]
    return X.to(dtype)


def _same(a, b, dtype):
    a, b = a.double().cpu(), b.double().cpu()
    fa, fb = torch.isfinite(a), torch.isfinite(b)
    assert torch.equal(fa, fb)
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    assert torch.equal(a[~fa & ~torch.isnan(a)], b[~fb & ~torch.isnan(b)])
    if fa.any():
        err = (a[fa] - b[fa]).abs().max().item()
        assert err <= TOL[dtype] * max(b[fa].abs().max().item(), 1.0), err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [5, 8, 13, 16, 32, 40, 64])
def test_packed_key_rules_with_nonfinite(cuda, n, dtype):
    """bf16/fp16 median, trimmed mean, averaged median and condense (packed 16-bit
    key networks + exact rank fallback for NaN/inf coordinates and the tail) vs
    the fp64 oracle; d is odd so the scalar tail runs too."""
    X = _nonfinite_rows(n, 2 * 1024 + 7, dtype, seed=n)
    Xc = X.to(cuda)
    assert torch.equal(gar.median(Xc).double().cpu(), ref.median(X).to(dtype).double())
    f = max((n - 1) // 4, 1)
    _same(gar.trimmed_mean(Xc, f), ref.trimmed_mean(X, f), dtype)
    beta = n - f
    _same(gar.averaged_median(Xc, beta=beta), ref.averaged_median(X, beta), dtype)
    out = gar.condense(Xc, p=0.7, seed=99)
    assert torch.allclose(out.double().cpu(), ref.condense(X, 0.7, 99).to(dtype).double(), rtol=0, atol=0,
                          equal_nan=True)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [8, 16, 32, 64])
def test_packed_key_rules_ties_and_extremes(cuda, n, dtype):
    """Heavy ties (values drawn from 5 levels), largest finite values and -0.0/+0.0:
    the order-preserving key map and the max-finite padding must not change results."""
    g = torch.Generator().manual_seed(n)
    levels = torch.tensor([-0.0, 0.0, 1.5, -2.25, torch.finfo(dtype).max])
    X = levels[torch.randint(0, 5, (n, 4096 + 3), generator=g)].to(dtype)
    Xc = X.to(cuda)
    assert torch.equal(gar.median(Xc).double().cpu(), ref.median(X).to(dtype).double())
    # sums of dtype-max values overflow fp32 accumulators (not the fp64 oracle): use 1e4 there
    X = torch.where(X.float().abs() > 1e4, torch.full_like(X, 1e4), X)
    Xc = X.to(cuda)
    f = max(n // 8, 1)
    _same(gar.trimmed_mean(Xc, f), ref.trimmed_mean(X, f), dtype)
    _same(gar.averaged_median(Xc, beta=n - f), ref.averaged_median(X, n - f), dtype)


def _near_duplicates(n, d, dtype, spread, seed):
    """n - 1 honest rows = base + s_i * noise_i (distinct small s_i: distances are a tiny
    fraction of the norms, the regime where ||a||^2 + ||b||^2 - 2ab cancels) and one
    'little is enough' row at mu + 1.035 sigma of the honest rows."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(d, generator=g)
    scales = torch.linspace(spread, 3 * spread, n - 1)[torch.randperm(n - 1, generator=g)]
    X = torch.empty(n, d)
    for i in range(n - 1):
        X[i] = base + scales[i] * torch.randn(d, generator=g)
    H = X[: n - 1].double()
    X[n - 1] = (H.mean(0) + 1.035 * H.std(0)).float()
    return X.to(dtype)


@pytest.mark.parametrize("dtype,d,spread", [(torch.bfloat16, 23_528_522, 0.02), (torch.float32, 4_000_000, 1e-3)])
@pytest.mark.parametrize("n,f", [(8, 2), (16, 3)])
def test_near_duplicate_selections_match_fp64_direct_differences(cuda, n, f, dtype, d, spread):
    """Krum and Bulyan choose exactly what fp64 direct-difference distances choose, at the
    ResNet-50 size, for near-duplicate gradients plus an ALIE row."""
    X = _near_duplicates(n, d, dtype, spread, seed=n)
    D = ref.pairwise_sqdist(X)
    Xc = X.to(cuda)
    w = gar.krum_weights(Xc, f).cpu()
    assert torch.equal(w != 0, ref.krum_weights(D, f).float() != 0)
    if n >= 4 * f + 3:
        W = gar.bulyan_weights(Xc, f).cpu()
        assert torch.equal(W != 0, ref.bulyan_weights(D, f).float() != 0)
