#!/bin/bash
# round 6: 3x3 weight-gradient wave layouts (micro + ResNet-18 step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6d; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python scripts/bench_wgrad3x3.py > $O/wgrad3x3_micro.txt 2>&1 &&
for v in 0 1 0 1; do
  timeout -k 10 200 python scripts/ab_variant.py wgrad3x3 $v --model resnet18 --steps 20 --warmup 5 --no-fp32 > $O/ab_r18_v$v.$RANDOM.json.log 2>&1 || exit 1
done &&
for v in 0 1; do
  timeout -k 10 200 python scripts/ab_variant.py wgrad3x3 $v --steps 20 --warmup 5 --no-fp32 > $O/ab_r50_v$v.$RANDOM.json.log 2>&1 || exit 1
done
