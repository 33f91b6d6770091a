"""Times every valid gpu_gemm_nt configuration on a few latency-bound ResNet-50 CIFAR shapes
(back-to-back launches; a cold-L2 variant flushes a 512 MB buffer between calls)."""
import torch

from garfield_amd import _native

C = _native.native()
dev = torch.device("cuda", 0)
flush = torch.empty(512 * 1024 * 1024 // 4, device=dev)


def timed(fn, cold, reps=20):
    fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(reps):
        if cold:
            flush.zero_()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        fn()
        t1.record()
        t1.synchronize()
        tot += t0.elapsed_time(t1)
    return tot * 1000.0 / reps


for (M, N, K) in [(2000, 1024, 1024), (2000, 512, 2048), (2000, 2048, 512), (32000, 128, 512), (8000, 1024, 256),
                  (8000, 256, 1024)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    row = []
    for cfg in range(C.gemm_nt_num_cfg()):
        if not C.gemm_nt_valid(cfg, N, K):
            continue
        t_w = timed(lambda: C.gpu_gemm_nt(a, b, c, None, None, 0, cfg), False)
        t_c = timed(lambda: C.gpu_gemm_nt(a, b, c, None, None, 0, cfg), True)
        row.append((t_c, t_w, cfg))
    row.sort()
    print(f"M={M} N={N} K={K} pick={C.gemm_nt_pick(M, N, K, 0)}: " +
          ", ".join(f"cfg{cfg} {tc:.1f}/{tw:.1f}" for tc, tw, cfg in row[:8]), flush=True)
