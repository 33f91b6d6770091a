#!/bin/bash
# round 6: the headline-model convergence test (gated, ~4 min) and the ResNet-18 one
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6z; mkdir -p $O
export PYTHONPATH=$R
GARFIELD_SLOW_TESTS=1 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 700 --timeout-method thread tests/test_grouped_gpu.py -k "trains_like_fp32" > $O/pytest_converge.log 2>&1
