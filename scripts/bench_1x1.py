"""Micro-benchmark: the grouped ResNet-50 step's 1x1 convolution GEMMs (8 workers x 250
CIFAR images) on hipBLASLt (torch.mm) vs the implicit-GEMM MFMA kernel (gpu_iconv as a
1x1 convolution, pixel tiles PM = 1/2/4) and, when built, the dedicated 1x1 kernel
(gpu_gemm1x1).  Forward y = x·Wᵀ and data gradient dx = dy·W; prints µs and the
fraction of the 6.3 TB/s achievable HBM rate the compulsory bytes represent."""
import time

import torch

from garfield_amd import _native

N = 2000
# (name, rows M, K = Cin, Cout, count per step)
SHAPES = [
    ("l1 1x1 64->64", N * 64, 64, 64, 1), ("l1 1x1 256->64", N * 64, 256, 64, 2),
    ("l1 1x1 64->256", N * 64, 64, 256, 4),
    ("l2 1x1 256->128", N * 64, 256, 128, 1), ("l2 1x1 512->128", N * 16, 512, 128, 3),
    ("l2 1x1 128->512", N * 16, 128, 512, 4),
    ("l3 1x1 512->256", N * 16, 512, 256, 1), ("l3 1x1 1024->256", N * 4, 1024, 256, 5),
    ("l3 1x1 256->1024", N * 4, 256, 1024, 6),
    ("l4 1x1 1024->512", N * 4, 1024, 512, 1), ("l4 1x1 2048->512", N, 2048, 512, 2),
    ("l4 1x1 512->2048", N, 512, 2048, 3),
]


def bench(fn, iters=30):
    """Device time per call: ``iters`` calls captured in one HIP graph and replayed
    (host launch overhead, ~20 µs per hipBLASLt call from Python, is not counted,
    exactly as in the graphed training step)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (5 * iters) * 1e6


def main():
    dev = torch.device("cuda")
    C_ = _native.native()
    has_g = hasattr(C_, "gpu_gemm_nt")
    tot = {}
    for name, M, K, Co, cnt in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Co, K, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(M, Co, device=dev, dtype=torch.bfloat16)
        byf = 2 * (M * K + M * Co + Co * K)
        res = {}
        yref = torch.mm(x, w.t())
        dref = torch.mm(dy, w)
        res["mm fwd"] = bench(lambda: torch.mm(x, w.t()))
        res["mm dgrad"] = bench(lambda: torch.mm(dy, w))
        x4 = x.view(M, 1, 1, K).permute(0, 3, 1, 2)          # [M, K, 1, 1] channels_last
        dy4 = dy.view(M, 1, 1, Co).permute(0, 3, 1, 2)
        w4 = w.view(Co, K, 1, 1)
        y4 = torch.empty((M, Co, 1, 1), device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        dx4 = torch.empty((M, K, 1, 1), device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        for pm in (() if has_g else (11, 12, 14)):
            f = lambda: C_.gpu_iconv(x4, w4, 1, 1, 1, 1, 0, 0, 1, 1, y4, None, pm, False)
            res[f"iconv{pm - 10} fwd"] = bench(f)
            f()
            err = (y4.view(M, Co).float() - yref.float()).abs().max().item()
            assert err < 0.05 * yref.float().abs().max().item() + 1e-2, (name, pm, err)
            g = lambda: C_.gpu_iconv(dy4, w4, 1, 1, 1, 1, 0, 0, 1, 1, dx4, None, pm, True)
            res[f"iconv{pm - 10} dgrad"] = bench(g)
            g()
            err = (dx4.view(M, K).float() - dref.float()).abs().max().item()
            assert err < 0.05 * dref.float().abs().max().item() + 1e-2, (name, pm, "dgrad", err)
        G = 8
        rg = M // G
        out = torch.empty((G, Co, K), device=dev, dtype=torch.bfloat16)
        from garfield_amd.ops.grouped import _wgrad
        res["wgrad bmm"] = bench(lambda: _wgrad(dy, x, G, out))
        gi = torch.empty((G, Co, K), device=dev, dtype=torch.bfloat16)
        for S in (() if has_g else (1, 4)):
            part = torch.empty((S, G, Co, K), device=dev, dtype=torch.float32)
            if S == 1:
                f = lambda: C_.gpu_iwgrad(x4, dy4, 1, 1, 1, 1, 0, 0, 1, 1, G, gi, 1)
            else:
                f = lambda: (C_.gpu_iwgrad(x4, dy4, 1, 1, 1, 1, 0, 0, 1, 1, G, part, S), torch.sum(part, 0, out=gi))
            res[f"iwgrad S{S}"] = bench(f)
        if has_g:
            y2 = torch.empty((M, Co), device=dev, dtype=torch.bfloat16)
            dx2 = torch.empty((M, K), device=dev, dtype=torch.bfloat16)
            wt = w.t().contiguous()
            res["transpose w"] = bench(lambda: w.t().contiguous())
            for cfg in range(C_.gemm_nt_num_cfg()):
                if C_.gemm_nt_valid(cfg, Co, K):
                    f = lambda: C_.gpu_gemm_nt(x, w, y2, None, None, 0, cfg)
                    res[f"nt{cfg} fwd"] = bench(f)
                    f()
                    err = (y2.float() - yref.float()).abs().max().item()
                    assert err < 0.02 * yref.float().abs().max().item() + 1e-2, (name, cfg, err)
                if C_.gemm_nt_valid(cfg, K, Co):
                    g = lambda: C_.gpu_gemm_nt(dy, wt, dx2, None, None, 0, cfg)
                    res[f"nt{cfg} dgrad"] = bench(g)
                    g()
                    err = (dx2.float() - dref.float()).abs().max().item()
                    assert err < 0.02 * dref.float().abs().max().item() + 1e-2, (name, cfg, "dgrad", err)
            # fused BatchNorm statistics (rg rows per worker) vs torch on the stored output
            for cfg in range(C_.gemm_nt_num_cfg()):
                sr = C_.gemm_nt_stats_rows(cfg)
                if C_.gemm_nt_valid(cfg, Co, K) and sr <= rg:
                    st = torch.empty(C_.gemm_nt_stats_geometry(cfg, M, Co, K, rg)[2], device=dev, dtype=torch.float32)
                    res[f"nt{cfg}+st"] = bench(lambda: C_.gpu_gemm_nt(x, w, y2, None, st, rg, cfg))
            pf, pd, ps = C_.gemm_nt_pick(M, Co, K, 0), C_.gemm_nt_pick(M, K, Co, 0), C_.gemm_nt_pick(M, Co, K, rg)
            res[f"auto fwd(nt{pf})"] = res.get(f"nt{pf} fwd", float("nan"))
            res[f"auto dgrad(nt{pd})"] = res.get(f"nt{pd} dgrad", float("nan"))
            res[f"auto+st(nt{ps})"] = res.get(f"nt{ps}+st", float("nan"))
            cfg = C_.gemm_nt_pick(M, Co, K, rg)
            bm, be, nst = C_.gemm_nt_stats_geometry(cfg, M, Co, K, rg)
            st = torch.empty(nst, device=dev, dtype=torch.float32)
            C_.gpu_gemm_nt(x, w, y2, None, st, rg, cfg)
            mean = torch.empty((G, Co), device=dev)
            istd, sc, sh = torch.empty_like(mean), torch.empty_like(mean), torch.empty_like(mean)
            ybn = torch.empty_like(y2)
            gam = torch.rand(Co, device=dev) + 0.5
            bet = torch.randn(Co, device=dev)
            part = torch.empty(C_.bn_part_floats(rg, G, Co), device=dev)
            C_.gpu_bn_forward(y2, None, G, gam, bet, 1e-5, 0.1, None, None, part, mean, istd, sc, sh, ybn, False,
                              tile_stats=st, tile_m=bm, tile_e=be)
            yg = y2.float().view(G, rg, Co)
            mref = yg.mean(1)
            vref = yg.var(1, unbiased=False)
            em = (mean - mref).abs().max().item()
            ev = ((1.0 / istd ** 2 - 1e-5) - vref).abs().max().item() / vref.abs().max().item()
            assert em < 1e-3 * (1 + mref.abs().max().item()) and ev < 1e-3, (name, "stats", em, ev)
        floor = byf / 6.3e12 * 1e6
        print(f"{name:18s} M={M:6d} K={K:5d} N={Co:5d} x{cnt} floor {floor:5.1f}us | "
              + " ".join(f"{k} {v:6.1f}" for k, v in res.items()), flush=True)
        for k, v in res.items():
            k = k.split("(")[0]
            tot[k] = tot.get(k, 0.0) + cnt * v
    print("per-step totals (us):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
