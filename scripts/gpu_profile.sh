#!/bin/bash
# Profiling session: rocprofv3 kernel stats of the bench step and of the GAR micro-bench.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTHONPATH=$R
export GARFIELD_TRACE_MARK=1
PSTEPS=${PSTEPS:-5}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps $PSTEPS --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
tail -1 $R/gpurun_out/prof_bench.log
python3 $R/scripts/trace_summary.py $R/gpurun_out/prof_bench/bench_kernel_trace.csv --steps $PSTEPS --top 40 --sequence $R/gpurun_out/prof_bench_sequence.txt > $R/gpurun_out/prof_bench_summary.txt
head -3 $R/gpurun_out/prof_bench_summary.txt
rm -f $R/gpurun_out/prof_bench/bench_kernel_trace.csv  # too large to copy back; the summary keeps the steady state
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gar -o gar -- python3 -m garfield_amd.apps.gar_bench --n 8 64 --d 23528522 --iters 3 --warmup 1 > $R/gpurun_out/prof_gar.log 2>&1 || { echo "rocprof gar failed"; tail -20 $R/gpurun_out/prof_gar.log; exit 1; }
python3 $R/scripts/trace_summary.py $R/gpurun_out/prof_gar/gar_kernel_trace.csv --marker __none__ --top 40 > $R/gpurun_out/prof_gar_summary.txt
rm -f $R/gpurun_out/prof_gar/gar_kernel_trace.csv
echo profile done
