#!/bin/bash
# Profiling session: rocprofv3 kernel stats of the bench step and of the GAR micro-bench.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > $R/gpurun_out/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
tail -1 $R/gpurun_out/prof_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gar -o gar -- python3 -m garfield_amd.apps.gar_bench --n 8 64 --d 23528522 --iters 3 --warmup 1 > $R/gpurun_out/prof_gar.log 2>&1 || { echo "rocprof gar failed"; tail -20 $R/gpurun_out/prof_gar.log; exit 1; }
echo profile done
