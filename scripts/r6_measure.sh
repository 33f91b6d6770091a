#!/bin/bash
# round 6: GEMM census + steady-state kernel tables (plain / torch.distributed one-rank / loopback)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6m; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python scripts/gemm_census.py > $O/census_r50.txt 2>$O/census.err &&
bash scripts/gpu_prof.sh plain --no-fp32 > /dev/null &&
GARFIELD_COLL_WORLD1=1 bash scripts/gpu_prof.sh coll1 --no-fp32 --shard-gar > /dev/null &&
GARFIELD_LOOPBACK_EXCHANGE=1 bash scripts/gpu_prof.sh loopback --no-fp32 --shard-gar > /dev/null &&
cp gpurun_out/prof/*.txt $O/
