#!/bin/bash
# round 6: loss curves of the headline model (ResNet-50) on the grouped bf16 path vs the per-worker fp32 engine
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6conv; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 900 python -u scripts/diag_converge.py 150 resnet50 0.001,0.002 > $O/converge_r50_lowlr.jsonl 2> $O/converge_r50.err
