#!/bin/bash
# Round-5 quick GPU check: selected GPU tests, then the bf16 bench (20 steps) and a kernel table.
#   TESTS="tests/x.py tests/y.py" bash scripts/gpu_r5_quick.sh
set -o pipefail
R=$(pwd); O=$R/gpurun_out/quick; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error" $O/pytest.log | head -20; exit 1; }
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-fp32 ${BENCH_ARGS} > $O/bench.json.log 2>&1 || { tail -5 $O/bench.json.log; exit 1; }
  tail -1 $O/bench.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['value'])"
fi
if [ -n "$SEQ" ]; then
  bash scripts/gpu_seq.sh r50 --no-fp32 ${BENCH_ARGS} > /dev/null && head -30 gpurun_out/seq/r50.txt | cut -c1-120
fi
