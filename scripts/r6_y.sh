#!/bin/bash
# round 6: stem forward's BatchNorm statistics epilogue: tests, ImageNet step + table, headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6y; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_grouped_gpu.py -k "stem or as_accurate or graph_matches_eager or headline_path or bn_kernels" > $O/pytest.log 2>&1 &&
timeout -k 10 400 python bench.py --dataset imagenet --steps 10 --warmup 3 --no-fp32 > $O/imagenet.json.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/headline.json.log 2>&1 &&
bash scripts/gpu_prof.sh imagenet --dataset imagenet --no-fp32 > /dev/null && cp gpurun_out/prof/imagenet.txt $O/imagenet_table.txt
