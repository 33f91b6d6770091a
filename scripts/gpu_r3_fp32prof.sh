#!/bin/bash
set -o pipefail
R=$(pwd); O=$R/gpurun_out/fp32; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
GARFIELD_TRACE_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run \
    -- python3 $R/bench.py --steps 3 --warmup 2 --precision fp32 ${ARGS} > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 $R/scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps 3 --top 40 > $O/rocprof_fp32.txt
rm -rf $O/prof
head -42 $O/rocprof_fp32.txt | cut -c1-150
