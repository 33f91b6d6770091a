#!/bin/bash
# Layer-wise GAR on device + col-mode GEMM changes: tests, then the flat vs layer-wise bench.
set -o pipefail
mkdir -p gpurun_out/lw
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/lw
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
    tests/test_grouped_gpu.py tests/test_gemm_nt_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_flat.json.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_flat.json.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --layerwise > $O/bench_lw.json.log 2>&1 || { echo "bench lw failed"; tail -20 $O/bench_lw.json.log; exit 1; }
for f in flat lw; do python -c "import json,sys; d=json.loads(open('$O/bench_$f.json.log').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['final_loss'])"; done
