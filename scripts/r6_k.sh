#!/bin/bash
# round 6: the 1000-class head on gemm_nt / the 1x1 weight-gradient kernel: its GPU test, the ImageNet-shape
# config and its kernel table (no Cijk_ GEMM expected)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6k; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grouped_gpu.py -k "grouped_linear" > $O/pytest_head.log 2>&1 &&
timeout -k 10 400 python bench.py --dataset imagenet --steps 10 --warmup 3 --no-fp32 > $O/imagenet_krum_f2.json.log 2>&1 &&
bash scripts/gpu_prof.sh imagenet --dataset imagenet --no-fp32 > /dev/null && cp gpurun_out/prof/imagenet.txt $O/ &&
timeout -k 10 600 python -u scripts/gemm_census.py --dataset imagenet > $O/census_imagenet.txt 2>&1
