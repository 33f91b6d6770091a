#!/bin/bash
# round 6 closing run #3 (final tree): GPU suite, smoke, headline, GAR overheads, ResNet-18, ImageNet
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6final3; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline.json.log 2>&1 &&
B="timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overhead"
$B --no-fp32 > $O/krum_f2_bf16.json.log 2>&1 &&
$B --precision fp32 > $O/krum_f2_fp32.json.log 2>&1 &&
$B --no-fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_bf16.json.log 2>&1 &&
$B --precision fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_fp32.json.log 2>&1 &&
$B --no-fp32 --gar median --f 1 > $O/median_f1_bf16.json.log 2>&1 &&
$B --no-fp32 --gar trimmed-mean --f 2 > $O/trimmed_f2_bf16.json.log 2>&1 &&
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --no-fp32 > $O/r18_krum_f2.json.log 2>&1 &&
timeout -k 10 400 python bench.py --dataset imagenet --steps 10 --warmup 3 --no-fp32 > $O/imagenet_krum_f2.json.log 2>&1 &&
bash scripts/gpu_prof.sh final3_r50 --no-fp32 > /dev/null && cp gpurun_out/prof/final3_r50.txt $O/table_r50.txt
