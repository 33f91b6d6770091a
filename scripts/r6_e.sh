#!/bin/bash
# round 6: ImageNet-shape headline config + table, ResNet-18 config, BASELINE config 5 (loss fields fixed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6e; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 400 python bench.py --dataset imagenet --steps 10 --warmup 3 --no-fp32 > $O/imagenet_krum_f2.json.log 2>&1 &&
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/r18_krum_f2.json.log 2>&1 &&
bash scripts/gpu_prof.sh imagenet --dataset imagenet --no-fp32 > /dev/null && cp gpurun_out/prof/imagenet.txt $O/ &&
bash scripts/gpu_byzps_cfg5.sh > $O/cfg5_summary.txt 2>&1 && cp gpurun_out/byzps/*.json.log $O/
