#!/bin/bash
# round 6: measured fp32 convolution forms, more robust kernel-choice timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6h; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_fp32_gpu.py \
  tests/test_engine_gpu.py -k "fp32 or resume or wgrad" > $O/pytest.log 2>&1 &&
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_default_$i.json.log 2>&1 || exit 1
done &&
bash scripts/gpu_prof.sh r50_fp32_tuned --precision fp32 > /dev/null && cp gpurun_out/prof/r50_fp32_tuned.txt $O/
