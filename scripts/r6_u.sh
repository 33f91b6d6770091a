#!/bin/bash
# round 6: headline twice + CIFAR kernel table after the stem changes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6u; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/headline_1.json.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/headline_2.json.log 2>&1 &&
bash scripts/gpu_prof.sh r50 --no-fp32 > /dev/null && cp gpurun_out/prof/r50.txt $O/table_r50.txt &&
bash scripts/gpu_prof.sh r50f --precision fp32 --no-fp32 > /dev/null && cp gpurun_out/prof/r50f.txt $O/table_r50_fp32.txt
