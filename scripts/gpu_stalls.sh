#!/bin/bash
# Stall / occupancy / LDS-conflict table of a bench.py configuration's top kernels:
#   bash scripts/gpu_stalls.sh <name> [bench.py args...]
#   -> gpurun_out/stalls/<name>/: kernel table (gpu_seq.sh), pmc_stalls_summary.txt, stalls.md
# One SQ pass of 8 counters (the SQ block's limit), --pmc only (no other trace domains).
set -o pipefail
NAME=$1; shift
R=$(pwd); O=$R/gpurun_out/stalls/$NAME; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
bash scripts/gpu_seq.sh $NAME "$@" > /dev/null || exit 1
cp gpurun_out/seq/$NAME.txt gpurun_out/seq/$NAME.json $O/ || exit 1
cd /tmp && export TMPDIR=/tmp
GARFIELD_TRACE_MARK=1 timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o p \
    -- python3 $R/bench.py --steps 2 --warmup 2 "$@" > $O/pmc.log 2>&1 || { echo "stall pass failed"; tail -5 $O/pmc.log; exit 1; }
python3 $R/scripts/pmc_summary.py $O/pmc/p_counter_collection.csv --steps 2 --json $O/pmc_stalls.json \
    > $O/pmc_stalls_summary.txt || exit 1
rm -rf $O/pmc
cd $R
python3 scripts/stall_table.py $O/$NAME.json $O/pmc_stalls.json --md $O/stalls.md --top 15 || exit 1
