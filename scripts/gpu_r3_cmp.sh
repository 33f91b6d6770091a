#!/bin/bash
# Kernel totals of the plain step vs the bucketed (sharded, world-1) step.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r3c
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R GARFIELD_TRACE_MARK=1
cd /tmp && export TMPDIR=/tmp
for v in plain shard; do
  args=""; [ $v == shard ] && args="--shard-gar"
  GARFIELD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3c/$v -o run -- \
      python3 $R/bench.py --steps 5 --warmup 3 $args > $R/gpurun_out/r3c/$v.log 2>&1 || { echo "rocprof $v failed"; tail -20 $R/gpurun_out/r3c/$v.log; exit 1; }
  python3 $R/scripts/trace_summary.py $R/gpurun_out/r3c/$v/run_kernel_trace.csv --steps 5 --top 80 \
      --json $R/gpurun_out/r3c/$v.json > $R/gpurun_out/r3c/${v}_summary.txt
  head -2 $R/gpurun_out/r3c/${v}_summary.txt
  rm -f $R/gpurun_out/r3c/$v/run_kernel_trace.csv
done
