#!/bin/bash
# fp32 grouped-channel path: GPU equality tests, then bench --precision fp32 vs the per-worker
# fp32 path and the reference-style implementation.
set -o pipefail
mkdir -p gpurun_out/fp32
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/fp32
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k fp32 \
    > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --steps 5 --warmup 3 --precision fp32 --ref-impl > $O/bench_fp32.json.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_fp32.json.log; exit 1; }
tail -1 $O/bench_fp32.json.log | cut -c1-300
python -c "import json; d=json.loads(open('$O/bench_fp32.json.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('ms_per_step','value','ref_impl_ms_per_step','speedup_vs_ref_impl','final_loss')})"
if [ -n "$GRAPHOFF" ]; then
  GARFIELD_NO_GRAPH=1 timeout -k 10 600 python bench.py --steps 5 --warmup 3 --precision fp32 --no-graph > $O/bench_fp32_eager.json.log 2>&1 || exit 1
  tail -1 $O/bench_fp32_eager.json.log | cut -c1-200
fi
