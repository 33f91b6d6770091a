#!/bin/bash
# Profiling session: GAR micro-bench, rocprofv3 kernel stats of bench + GAR bench, bench variants.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m garfield_amd.apps.gar_bench --n 8 16 32 64 --d 23528522 --iters 10 > gpurun_out/gar_bench.log 2>&1 || { echo "gar_bench failed"; tail -20 gpurun_out/gar_bench.log; exit 1; }
echo "gar_bench done"
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --overhead > gpurun_out/bench_overhead.log 2>&1 || { echo "bench overhead failed"; tail -20 gpurun_out/bench_overhead.log; exit 1; }
tail -1 gpurun_out/bench_overhead.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --channels-last > gpurun_out/bench_cl.log 2>&1 || { echo "bench cl failed"; tail -20 gpurun_out/bench_cl.log; }
tail -1 gpurun_out/bench_cl.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 3 --warmup 1 > $R/gpurun_out/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -20 $R/gpurun_out/prof_bench.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gar -o gar -- python3 -m garfield_amd.apps.gar_bench --n 8 64 --d 23528522 --iters 3 --warmup 1 > $R/gpurun_out/prof_gar.log 2>&1 || { echo "rocprof gar failed"; tail -20 $R/gpurun_out/prof_gar.log; exit 1; }
echo profile done
