#!/bin/bash
# round 6: torch.distributed sharded step staged (works waited on by the comm stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6f; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_rccl_gpu.py \
  tests/test_engine_gpu.py -k "rccl or bucketed or sharded" > $O/pytest.log 2>&1 &&
for i in 1 2; do
GARFIELD_COLL_WORLD1=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --shard-gar > $O/bench_coll1_shard_$i.json.log 2>&1 &&
GARFIELD_LOOPBACK_EXCHANGE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --shard-gar > $O/bench_loopback_$i.json.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_plain_$i.json.log 2>&1 || exit 1
done &&
GARFIELD_COLL_WORLD1=1 bash scripts/gpu_prof.sh coll1c --no-fp32 --shard-gar > /dev/null && cp gpurun_out/prof/coll1c.txt $O/
