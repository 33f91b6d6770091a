#!/bin/bash
# round 6: the fp32 step's dispatch sequence (its traced window is 91% busy against 97% for bf16)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6seq32; mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
GARFIELD_TRACE_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run \
    -- python3 $R/bench.py --precision fp32 --steps 3 --warmup 2 --no-fp32 > $O/bench.log 2>&1 &&
python3 $R/scripts/trace_summary.py $O/tr/run_kernel_trace.csv --steps 3 --top 10 --sequence $O/seq_f32.txt > $O/table.txt &&
rm -rf $O/tr
