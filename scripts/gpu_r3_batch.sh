#!/bin/bash
# Round-3 batch: layer-wise (incl. sharded) + fp32 tests, the fp32 bench and its profile.
set -o pipefail
mkdir -p gpurun_out/batch
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/batch
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
    -k "layerwise or fp32" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --steps 5 --warmup 3 --precision fp32 --ref-impl > $O/bench_fp32.json.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_fp32.json.log; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_fp32.json.log').read().strip().splitlines()[-1]); print({k: d.get(k) for k in ('ms_per_step','value','ref_impl_ms_per_step','speedup_vs_ref_impl','final_loss','first_loss')}, d['config']['hip_graphs'])"
bash scripts/gpu_r3_fp32prof.sh | head -25
