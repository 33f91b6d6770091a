#!/bin/bash
# Round-2 GPU session: GAR + engine tests, GAR kernel sweep with rocprof stats,
# headline bench, and a kernel trace of the bucketed exchange (loopback) overlap.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=${TAG:-r2}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gar_gpu.py tests/test_engine_gpu.py tests/test_grouped_gpu.py} -x -q \
  --timeout 180 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
fi
if [ "${SKIP_GARBENCH:-0}" != "1" ]; then
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n ${NS:-8 16 32 64} --d 23528522 \
  --rules ${RULES:-median trimmed-mean averaged-median bulyan krum} --iters 20 > gpurun_out/gar_bench_$TAG.jsonl 2>&1 \
  || { echo "gar_bench failed"; tail -20 gpurun_out/gar_bench_$TAG.jsonl; exit 1; }
grep '^{' gpurun_out/gar_bench_$TAG.jsonl
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 \
  || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
if [ "${TRACE:-1}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp
GARFIELD_TRACE_MARK=1 GARFIELD_LOOPBACK_EXCHANGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
  -d $R/gpurun_out/prof_ovl_$TAG -o ovl -- python3 $R/bench.py --steps 3 --warmup 3 --shard-gar \
  > $R/gpurun_out/prof_ovl_$TAG.log 2>&1 || { echo "rocprof overlap failed"; tail -20 $R/gpurun_out/prof_ovl_$TAG.log; exit 1; }
tail -1 $R/gpurun_out/prof_ovl_$TAG.log
T=$(find $R/gpurun_out/prof_ovl_$TAG -name "*kernel_trace.csv" | head -1)
python3 $R/scripts/trace_summary.py $T --steps 3 --top 30 --sequence $R/gpurun_out/ovl_sequence_$TAG.txt > $R/gpurun_out/ovl_summary_$TAG.txt
python3 $R/scripts/overlap_check.py $T > $R/gpurun_out/ovl_check_$TAG.txt 2>&1; cat $R/gpurun_out/ovl_check_$TAG.txt | tail -12
rm -f $T
fi
