#!/bin/bash
# Stem kernel checks on one MI355X: numerics, the grouped/engine GPU tests, A/B of the
# step with and without stem_nhwc.hip, and a kernel-stats profile of the new step.
set -o pipefail
mkdir -p gpurun_out/stem
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/stem
timeout -k 10 180 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grouped_gpu.py -k stem \
    > $O/pytest_stem.log 2>&1 || { echo "stem tests failed"; tail -30 $O/pytest_stem.log; exit 1; }
tail -1 $O/pytest_stem.log
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
      tests/test_grouped_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
CONFIGS="GARFIELD_STEM=0;GARFIELD_STEM=1" RUNS=${RUNS:-2} TAG=stem bash scripts/gpu_ab_env.sh || exit 1
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  GARFIELD_TRACE_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 \
      > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 1; }
fi
