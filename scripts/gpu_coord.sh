#!/bin/bash
# Coordinate-wise GAR kernels: correctness tests, gar_bench sweep, rocprof kernel stats.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-coord}
if [ "${PROBE:-0}" = "1" ]; then
  timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 scripts/rccl_shared_gpu_probe.py > gpurun_out/rccl_probe.log 2>&1
  echo "probe rc=$?"; tail -4 gpurun_out/rccl_probe.log
fi
timeout -k 10 400 python -u -m pytest tests/test_gar_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "${TESTK:-median or trimmed or averaged or condense or packed or nonfinite}" > gpurun_out/pt_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
RULES=${RULES:-median trimmed-mean averaged-median}
NS=${NS:-8 16 32 64}
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n $NS --d 23528522 --rules $RULES --iters 20 \
  > gpurun_out/gar_bench_$TAG.jsonl 2>&1 || { echo "gar_bench failed"; tail -20 gpurun_out/gar_bench_$TAG.jsonl; exit 1; }
grep '^{' gpurun_out/gar_bench_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o gb -- \
  python3 -m garfield_amd.apps.gar_bench --n $NS --d 23528522 --rules $RULES --iters 5 --warmup 1 \
  > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_$TAG.csv \;
find $R/gpurun_out/prof_$TAG -name "*kernel_trace.csv" -exec rm {} \;
cut -d, -f1-8 $R/gpurun_out/kstats_$TAG.csv | head -20
