#!/bin/bash
# GEMM checks on one MI355X: numerics of every gemm_nt configuration (and fused statistics),
# then the per-shape micro-bench of the step's 1x1 GEMMs against hipBLASLt.
set -o pipefail
mkdir -p gpurun_out/gemm
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/gemm
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py \
    > $O/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -40 $O/pytest_gemm.log; exit 1; }
tail -1 $O/pytest_gemm.log
timeout -k 10 400 python -u scripts/bench_1x1.py > $O/bench_1x1.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_1x1.log; exit 1; }
cat $O/bench_1x1.log | cut -c1-400
