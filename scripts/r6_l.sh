#!/bin/bash
# round 6: weight-stationary GEMM with inline-asm LDS-DMA (ws_asm): bitwise A/B + timing per problem, then the
# whole steps (CIFAR headline twice per variant, ImageNet once per variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6l; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python -u scripts/ab_gemm_ws.py --imagenet > $O/ab_gemm_ws.txt 2>&1 &&
for v in 0 1 0 1; do timeout -k 10 200 python scripts/ab_variant.py ws_asm $v --steps 20 --warmup 5 --no-fp32 > $O/ab_r50_v$v.$RANDOM.json.log 2>&1 || exit 1; done &&
for v in 0 1; do timeout -k 10 400 python scripts/ab_variant.py ws_asm $v --dataset imagenet --steps 8 --warmup 3 --no-fp32 > $O/ab_in_v$v.json.log 2>&1 || exit 1; done
