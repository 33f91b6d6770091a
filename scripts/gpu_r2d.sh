#!/bin/bash
# 1x1 GEMM micro-benchmark + 2-rank rehearsal of the multi-rank bench path on ONE GPU
# (gloo collectives on GPU tensors; RCCL refuses two ranks on one device).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
TAG=${TAG:-r2d}
timeout -k 10 300 python scripts/bench_1x1.py > gpurun_out/bench_1x1_$TAG.log 2>&1 || { echo "bench_1x1 failed"; tail -8 gpurun_out/bench_1x1_$TAG.log; exit 1; }
cat gpurun_out/bench_1x1_$TAG.log | grep -v amdgpu.ids
[ -n "$SKIP_DIST" ] && exit 0
GARFIELD_DIST_BACKEND=gloo GARFIELD_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_gloo2_$TAG.log 2>&1 || { echo "gloo2 bench failed"; tail -30 gpurun_out/bench_gloo2_$TAG.log; exit 1; }
grep '^{' gpurun_out/bench_gloo2_$TAG.log | cut -c1-400
