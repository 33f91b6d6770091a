#!/bin/bash
# round 6: fp32 Bulyan tail (FMA fast path), own shard kept out of the packed all-to-all
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6c; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gar_gpu.py -k "bulyan" \
  tests/test_rccl_gpu.py tests/test_gar_large_gpu.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 --d 11173962 23528522 --dtype fp32 \
  --rules bulyan > $O/gar_bench_bulyan_fp32.jsonl 2>$O/gar_bench.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overhead --precision fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_fp32.json.log 2>&1 &&
GARFIELD_COLL_WORLD1=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --shard-gar > $O/bench_coll1_shard.json.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_plain.json.log 2>&1 &&
GARFIELD_COLL_WORLD1=1 bash scripts/gpu_prof.sh coll1b --no-fp32 --shard-gar > /dev/null && cp gpurun_out/prof/coll1b.txt $O/
