#!/bin/bash
# HIP API + kernel trace of the bucketed world-1 step with the loopback exchange and
# in-graph bucket events (when does the host enqueue the exchange, when does it run).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r3t
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R GARFIELD_TRACE_MARK=1
cd /tmp && export TMPDIR=/tmp
GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=${OV:-1} timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace \
    --output-format csv -d $R/gpurun_out/r3t/prof -o run -- python3 $R/bench.py --steps 3 --warmup 3 --shard-gar \
    > $R/gpurun_out/r3t/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/r3t/prof.log; exit 1; }
ls -la $R/gpurun_out/r3t/prof/
