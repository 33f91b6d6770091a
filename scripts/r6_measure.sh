#!/bin/bash
# round 6: gemm_nt tests + GEMM census + steady-state kernel tables (plain / torch.distributed one-rank / loopback)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6m; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_nt_gpu.py > $O/pytest_gemm.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_census.py > $O/census_r50.txt 2>$O/census.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_plain.json.log 2>&1 &&
bash scripts/gpu_prof.sh plain --no-fp32 > /dev/null &&
GARFIELD_COLL_WORLD1=1 bash scripts/gpu_prof.sh coll1 --no-fp32 --shard-gar > /dev/null &&
GARFIELD_LOOPBACK_EXCHANGE=1 bash scripts/gpu_prof.sh loopback --no-fp32 --shard-gar > /dev/null;
cp gpurun_out/prof/*.txt $O/ 2>/dev/null; true
