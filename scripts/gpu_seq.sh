#!/bin/bash
# Kernel table + one step's dispatch sequence of a bench.py configuration:
#   bash scripts/gpu_seq.sh <name> [bench.py args...]
#   -> gpurun_out/seq/<name>.txt (table), <name>_seq.txt (last step: offset, duration, kernel), <name>.json
set -o pipefail
NAME=$1; shift
R=$(pwd); O=$R/gpurun_out/seq; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
GARFIELD_TRACE_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$NAME -o run \
    -- python3 $R/bench.py --steps 3 --warmup 2 "$@" > $O/$NAME.log 2>&1 || { tail -5 $O/$NAME.log; exit 1; }
python3 $R/scripts/trace_summary.py $O/tr_$NAME/run_kernel_trace.csv --steps 3 --top 60 --json $O/$NAME.json \
    --sequence $O/${NAME}_seq.txt > $O/$NAME.txt || exit 1
rm -rf $O/tr_$NAME
head -3 $O/$NAME.txt | cut -c1-160
