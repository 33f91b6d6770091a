#!/bin/bash
# round 6: fp32 Bulyan tail kernel + short-split 1x1 wgrad ring: numerics, GAR micro-benchmark, step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6b; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gar_gpu.py \
  tests/test_grouped_gpu.py -k "bulyan or wgrad or iwgrad or shortcut" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 --d 11173962 23528522 --dtype fp32 \
  --rules bulyan > $O/gar_bench_bulyan_fp32.jsonl 2>$O/gar_bench.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overhead --precision fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_fp32.json.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default.json.log 2>&1 &&
bash scripts/gpu_prof.sh r50_fp32 --precision fp32 > /dev/null &&
bash scripts/gpu_prof.sh r18_bf16 --model resnet18 --no-fp32 > /dev/null &&
cp gpurun_out/prof/r50_fp32.txt gpurun_out/prof/r18_bf16.txt $O/
