"""The 1x1-convolution GEMM (gemm_nt.hip) and its fused BatchNorm statistics on MI355X,
against plain fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("M,K,N", [(128000, 64, 256), (4000, 256, 64), (2000, 512, 2048), (1000, 1024, 256),
                                   (333, 128, 128), (77, 64, 64), (128000, 256, 128), (32000, 128, 512),
                                   (8000, 256, 1024), (5000, 192, 64), (8000, 1024, 256), (2000, 2048, 512)])
def test_gemm_nt_every_config_matches_fp32(cuda, native, M, K, N):
    torch.manual_seed(M + K + N)
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    add = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    mask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
    bits = ((mask.unsqueeze(1) >> torch.arange(8, device=cuda, dtype=torch.uint8)) & 1).view(M, N).bool()
    masked = torch.where(bits, add, torch.zeros((), device=cuda, dtype=torch.bfloat16))
    ran = splits = 0
    # split-K forms included (fp32 slabs + one summing pass), and the in-workgroup split-K ones (KG groups of
    # 4 waves summed through LDS)
    for cfg in range(native.gemm_nt_num_cfg()):
        if not native.gemm_nt_valid(cfg, N, K):
            continue
        c = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        native.gpu_gemm_nt(a, b, c, None, None, 0, cfg)
        assert rel(c, ref) < 5e-3, cfg
        c2 = add.clone()
        native.gpu_gemm_nt(a, b, c2, c2, None, 0, cfg)        # in place: c = a·bᵀ + c
        assert rel(c2, ref + add.float()) < 5e-3, cfg
        # add_mask: add counts only where its bit is set (the lazily applied ReLU of a residual
        # gradient): bitwise the GEMM over the materialised masked add
        c3 = torch.full((M, N), float("nan"), device=cuda, dtype=torch.bfloat16)
        native.gpu_gemm_nt(a, b, c3, add, None, 0, cfg, add_mask=mask)
        c4 = masked.clone()
        native.gpu_gemm_nt(a, b, c4, c4, None, 0, cfg)
        assert torch.equal(c3, c4), cfg
        ran += 1
        splits += native.gemm_nt_splits(cfg) > 1
    assert ran >= 2
    assert splits > 0 or K % 128 != 0
    c = torch.empty((M, N), device=cuda, dtype=torch.bfloat16)
    native.gpu_gemm_nt(a, b, c)                                 # automatic configuration
    assert rel(c, ref) < 5e-3


@pytest.mark.parametrize("G,rg,K,N,offset", [(8, 16000, 64, 256, 0.0), (8, 1000, 256, 64, 0.0),
                                              (8, 250, 512, 128, 40.0), (3, 700, 128, 128, 25.0),
                                              (2, 4000, 64, 64, 300.0), (8, 4000, 128, 512, 10.0),
                                              (5, 40, 256, 128, 0.0)])
def test_fused_bn_statistics_match_fp32(cuda, native, G, rg, K, N, offset):
    """Per-worker mean / biased variance of the STORED GEMM output, merged from tile
    statistics (tiles straddling worker boundaries included), even when |mean| >> std."""
    torch.manual_seed(rg + N)
    M = G * rg
    a = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    b = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    ran = 0
    for cfg in range(native.gemm_nt_num_cfg()):
        if not native.gemm_nt_valid(cfg, N, K) or native.gemm_nt_stats_rows(cfg) > rg:
            continue
        ran += 1
        H, E, nst = native.gemm_nt_stats_geometry(cfg, M, N, K, rg)
        assert H <= rg
        # a column of the input drives a constant offset into every output channel
        a2 = a.clone()
        a2[:, 0] = offset
        b2 = b.clone()
        b2[:, 0] = 1.0 if offset else b[:, 0]
        y = torch.empty((M, N), device=cuda, dtype=torch.bfloat16)
        st = torch.full((nst,), float("nan"), device=cuda)
        native.gpu_gemm_nt(a2, b2, y, None, st, rg, cfg)
        assert rel(y, a2.float() @ b2.float().t()) < 5e-3
        mean = torch.empty((G, N), device=cuda)
        istd, sc, sh = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
        gam = torch.rand(N, device=cuda) + 0.5
        bet = torch.randn(N, device=cuda)
        part = torch.empty(native.bn_part_floats(rg, G, N), device=cuda)
        out = torch.empty_like(y)
        native.gpu_bn_forward(y, None, G, gam, bet, 1e-5, 0.1, None, None, part, mean, istd, sc, sh, out, False,
                              tile_stats=st, tile_m=H, tile_e=E)
        yg = y.double().view(G, rg, N)
        mref, vref = yg.mean(1), yg.var(1, unbiased=False)
        assert (mean.double() - mref).abs().max().item() < 1e-4 * (1 + mref.abs().max().item()), cfg
        var = 1.0 / istd.double() ** 2 - 1e-5
        assert ((var - vref).abs() / vref.clamp_min(1e-6)).max().item() < 2e-3, cfg
        yref = ((yg - mref[:, None]) / torch.sqrt(vref[:, None] + 1e-5) * gam.double() + bet.double()).view(M, N)
        assert rel(out, yref) < 1e-2, cfg
    assert ran >= 1


@pytest.mark.parametrize("G,B,C,Co,H,pm,offset", [(8, 4, 64, 64, 32, 24, 0.0), (3, 5, 128, 128, 16, 24, 30.0),
                                                  (4, 3, 64, 128, 8, 22, 0.0), (5, 7, 128, 64, 4, 22, 10.0),
                                                  (2, 9, 64, 64, 8, 0, 0.0)])
def test_conv3x3_bn_statistics_match_fp32(cuda, native, G, B, C, Co, H, pm, offset):
    """The halo-staged 3x3 kernel's BatchNorm-statistics epilogue: per-worker mean / biased variance of
    the STORED convolution output merged from per-wave tiles (tiles straddling worker boundaries: 8x8
    and 4x4 images), |mean| >> std included, and the BatchNorm forward from them."""
    torch.manual_seed(C + H)
    x = torch.randn(G * B, C, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Co, C, 3, 3, device=cuda) / (9 * C) ** 0.5).to(torch.bfloat16)
    x[:, 0] = 1.0
    w[:, 0] = 0.0
    w[:, 0, 1, 1] = offset     # the constant channel drives an offset into every output channel
    w = w.contiguous(memory_format=torch.channels_last)
    M = G * B * H * H
    rg = M // G
    rows = native.conv3x3_stats_rows(G * B, H, H, C, Co) if pm == 0 else 16 * (pm - 20)   # forced tile size
    assert rows in (32, 64)
    st = torch.full((-(-M // rows) * 6 * Co,), float("nan"), device=cuda)
    y = torch.empty((G * B, Co, H, H), dtype=torch.bfloat16, device=cuda).contiguous(memory_format=torch.channels_last)
    native.gpu_iconv(x, w, 3, 3, 1, 1, 1, 1, 1, 1, y, None, pm, False, st, rg)
    assert rel(y.float(), F.conv2d(x.float(), w.float(), None, 1, 1)) < 1e-2
    y2 = y.permute(0, 2, 3, 1).reshape(M, Co)
    mean = torch.empty((G, Co), device=cuda)
    istd, sc, sh = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
    gam = torch.rand(Co, device=cuda) + 0.5
    bet = torch.randn(Co, device=cuda)
    part = torch.empty(native.bn_part_floats(rg, G, Co), device=cuda)
    out = torch.empty_like(y2)
    native.gpu_bn_forward(y2, None, G, gam, bet, 1e-5, 0.1, None, None, part, mean, istd, sc, sh, out, False,
                          tile_stats=st, tile_m=rows, tile_e=1)
    yg = y2.double().view(G, rg, Co)
    mref, vref = yg.mean(1), yg.var(1, unbiased=False)
    assert (mean.double() - mref).abs().max().item() < 1e-4 * (1 + mref.abs().max().item())
    var = 1.0 / istd.double() ** 2 - 1e-5
    assert ((var - vref).abs() / vref.clamp_min(1e-6)).max().item() < 2e-3
    yref = ((yg - mref[:, None]) / torch.sqrt(vref[:, None] + 1e-5) * gam.double() + bet.double()).view(M, Co)
    assert rel(out, yref) < 1e-2


@pytest.mark.parametrize("S,G,shape", [(4, 8, (64, 72)), (16, 3, (128, 9)), (2, 5, (7,))])
def test_split_reduce_into_strided_rows(cuda, native, S, G, shape):
    """Split-K slabs summed in fp32 straight into strided (exchange-row) outputs."""
    torch.manual_seed(S * G)
    part = torch.randn((S, G, *shape), device=cuda)
    n = part[0, 0].numel()
    for dt in (torch.bfloat16, torch.float32):
        flat = torch.zeros(G * (n + 40) + 8, device=cuda, dtype=dt)
        strides = [n + 40]
        acc = 1
        for d in reversed(shape):
            strides.insert(1, acc)
            acc *= d
        out = flat.as_strided((G, *shape), tuple(strides), 8)
        native.gpu_split_reduce(part, out)
        assert rel(out, part.double().sum(0)) < (1e-6 if dt == torch.float32 else 5e-3)
        # a transposed slab view ([G, S, ...] storage) works too
        p2 = part.transpose(0, 1).contiguous().transpose(0, 1)
        out.zero_()
        native.gpu_split_reduce(p2, out)
        assert rel(out, part.double().sum(0)) < (1e-6 if dt == torch.float32 else 5e-3)


def test_split_reduce_crops_padded_columns(cuda, native):
    """A padded GEMM result [S, G, Cout, Kp] cropped to K columns into exchange rows (the stem)."""
    torch.manual_seed(3)
    S, G, co, kp, k = 8, 8, 64, 152, 147
    part = torch.randn((G, S, co, kp), device=cuda).transpose(0, 1)     # the split-K bmm layout
    flat = torch.zeros(G * (co * k + 100), device=cuda, dtype=torch.bfloat16)
    out = flat.as_strided((G, co, k), (co * k + 100, k, 1), 0)
    native.gpu_split_reduce(part[..., :k], out)
    assert rel(out, part[..., :k].double().sum(0)) < 5e-3
    assert int((flat.view(G, -1)[:, co * k:] != 0).sum()) == 0          # nothing written past the rows


def test_split_reduce_multi_matches_single(cuda, native):
    """Many split-K sums in one launch (40 jobs: two launches of <= 32), mixed shapes, crops,
    strides and output dtypes, equal to the one-job kernel."""
    torch.manual_seed(7)
    parts, outs, refs = [], [], []
    for i in range(40):
        S, G = 1 + i % 5, 1 + i % 8
        co, k = 8 * (1 + i % 3), 3 + 5 * (i % 4)
        kp = k + (i % 2) * 5                    # odd jobs: padded columns cropped away
        p = torch.randn((G, S, co, kp), device=cuda).transpose(0, 1)[..., :k]
        dt = torch.bfloat16 if i % 3 else torch.float32
        flat = torch.zeros(G * (co * k + 16), device=cuda, dtype=dt)
        parts.append(p)
        outs.append(flat.as_strided((G, co, k), (co * k + 16, k, 1), 0))
        refs.append(p.double().sum(0))
    native.gpu_split_reduce_multi(parts, outs)
    for o, r in zip(outs, refs):
        assert rel(o, r) < (1e-6 if o.dtype == torch.float32 else 5e-3)


def test_transpose_multi_matches_torch(cuda, native):
    """Every 1x1 weight's Wᵀ in one launch (the data-gradient GEMMs' B operand), more jobs than one
    launch's table, ragged tile edges."""
    torch.manual_seed(11)
    shapes = [(64, 64), (256, 64), (64, 256), (2048, 512), (8, 8), (72, 136)] * 8
    srcs = [torch.randn(r, c, device=cuda).to(torch.bfloat16) for r, c in shapes]
    dsts = [torch.empty(c, r, device=cuda, dtype=torch.bfloat16) for r, c in shapes]
    native.gpu_transpose_multi(srcs, dsts)
    for a, b in zip(srcs, dsts):
        assert torch.equal(b, a.t())
