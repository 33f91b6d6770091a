#!/bin/bash
# round 6: 1x1 weight-gradient forms (micro + whole step), fp32 overheads with the fixed baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6a; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python scripts/bench_iwgrad_wide.py > $O/iwgrad_wide_micro.txt 2>&1 &&
for v in 0 3 1 2 0 3; do
  timeout -k 10 200 python scripts/ab_variant.py iwgrad_wide $v --steps 20 --warmup 5 --no-fp32 > $O/ab_wide_v$v.$RANDOM.json.log 2>&1 || exit 1
done &&
B="timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overhead"
$B --precision fp32 > $O/krum_f2_fp32.json.log 2>&1 &&
$B --precision fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_fp32.json.log 2>&1 &&
$B --precision fp32 --gar median --f 1 > $O/median_f1_fp32.json.log 2>&1 &&
$B --precision fp32 --gar trimmed-mean --f 2 > $O/trimmed_f2_fp32.json.log 2>&1
