#!/bin/bash
# A/B bench of an environment knob: GPU tests of the grouped path, then bench.py with the
# knob at value A and B, alternating (3 runs each), one JSON line per run.
# usage: KNOB=GARFIELD_GEMM_NT_MAXN A=0 B=128 bash scripts/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > gpurun_out/pt_$TAG.log 2>&1 \
    || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
  tail -1 gpurun_out/pt_$TAG.log
fi
for i in $(seq ${RUNS:-3}); do
  for v in ${VALUES:-$A $B}; do
    env $KNOB=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_${v}_$i.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/bench_${TAG}_${v}_$i.log; exit 1; }
    echo "$KNOB=$v run $i: $(grep '^{' gpurun_out/bench_${TAG}_${v}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))')"
  done
done
