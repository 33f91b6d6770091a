#!/bin/bash
# round 6: mid-size (<= 4096 rows per worker) bf16 BatchNorm on the single-kernel form: BN tests, then steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6n; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grouped_gpu.py -k "bn_kernels or folded_shortcut or lazy_residual or headline_path" > $O/pytest_bn.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_1.json.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_2.json.log 2>&1 &&
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --no-fp32 > $O/r18.json.log 2>&1 &&
bash scripts/gpu_prof.sh r50 --no-fp32 > /dev/null && cp gpurun_out/prof/r50.txt $O/table_r50.txt
