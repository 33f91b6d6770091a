#!/bin/bash
# Round-6 full check: the whole GPU test suite, smoke(), the default bench (20 steps) and its kernel table.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/suite6; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error" $O/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json.log 2>&1 || { tail -5 $O/bench_default.json.log; exit 1; }
tail -1 $O/bench_default.json.log | cut -c1-300
bash scripts/gpu_prof.sh final_r50 --no-fp32 > /dev/null && cp gpurun_out/prof/final_r50.txt $O/
