#!/bin/bash
# Bulyan tail iteration: GAR GPU tests, then the Bulyan gar_bench at the ResNet-50 size.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
TAG=${TAG:-tail}
timeout -k 10 600 python -u -m pytest tests/test_gar_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 64 --d 23528522 --rules bulyan --iters 10 > gpurun_out/gar_bench_bulyan_$TAG.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/gar_bench_bulyan_$TAG.jsonl
