#!/bin/bash
# Quick GPU iteration: grouped/engine GPU tests, one bench run, one kernel-trace profile
# of the bench step (summary + last-step dispatch sequence under gpurun_out/).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TESTS=${TESTS:-tests/test_grouped_gpu.py tests/test_engine_gpu.py}
if [ -n "$TESTS" ] && [ "$TESTS" != "none" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pt.log | head -20; tail -5 gpurun_out/pt.log; exit 1; }
  tail -1 gpurun_out/pt.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log
[ "${PROFILE:-1}" = "1" ] || exit 0
export PYTHONPATH=$R GARFIELD_TRACE_MARK=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 5 --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
python3 $R/scripts/trace_summary.py $R/gpurun_out/prof_bench/bench_kernel_trace.csv --steps 5 --top 45 --sequence $R/gpurun_out/prof_bench_sequence.txt > $R/gpurun_out/prof_bench_summary.txt
rm -f $R/gpurun_out/prof_bench/bench_kernel_trace.csv
head -3 $R/gpurun_out/prof_bench_summary.txt
