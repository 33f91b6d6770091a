#!/bin/bash
# round 6: k_gemm_ws with inline-asm LDS-DMA and addend loads (now the only form): GEMM tests, per-problem timing,
# headline step x2, ImageNet step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6m; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py > $O/pytest_gemm.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_gemm_ws.py --imagenet > $O/ab_gemm_ws.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_1.json.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_2.json.log 2>&1 &&
timeout -k 10 400 python bench.py --dataset imagenet --steps 8 --warmup 3 --no-fp32 > $O/imagenet.json.log 2>&1
