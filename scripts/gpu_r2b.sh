#!/bin/bash
# Round-2 second GPU session: full GPU suite, ByzPS 1-GPU bench vs plain, Bulyan gar_bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
TAG=${TAG:-r2b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_plain_$TAG.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_plain_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_plain_$TAG.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --num-ps 1 --ps-workers --mar median > gpurun_out/bench_byzps_$TAG.log 2>&1 || { echo "byzps bench failed"; tail -5 gpurun_out/bench_byzps_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_byzps_$TAG.log | cut -c1-200
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 64 --d 23528522 --rules bulyan --iters 10 > gpurun_out/gar_bench_bulyan_$TAG.jsonl 2>&1 || exit 1
grep '^{' gpurun_out/gar_bench_bulyan_$TAG.jsonl
