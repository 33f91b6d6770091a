#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3s
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd) GARFIELD_LOOPBACK_EXCHANGE=0 GARFIELD_OVERLAP=0
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python scripts/overlap_timing.py --steps 3 $ARGS > gpurun_out/r3s/$tag.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/r3s/$tag.log; exit 1; }; echo "$tag $(grep '^{' gpurun_out/r3s/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print([(s["graph_end_ms"], s["step_end_ms"]) for s in d["steps"]])')"; }
ARGS= run both GARFIELD_XS_DEBUG=both
ARGS= run none GARFIELD_XS_DEBUG=none
ARGS= run c_waits_main GARFIELD_XS_DEBUG=c_waits_main
ARGS= run main_waits_c GARFIELD_XS_DEBUG=main_waits_c
