#!/bin/bash
# round 6: one-rank RCCL rehearsal of the default multi-rank exchange + bench / trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_rccl
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rccl_gpu.py \
  "tests/test_engine_gpu.py::test_resume_in_new_process_replays_kernel_choices" \
  "tests/test_engine_gpu.py::test_capture_after_dropping_engine_in_reference_cycle" \
  tests/test_grouped_gpu.py::test_bn_folded_shortcut_matches_fp32_reference > $O/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_plain.json.log 2>&1 &&
GARFIELD_COLL_WORLD1=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --shard-gar > $O/bench_coll1_shard.json.log 2>&1 &&
GARFIELD_LOOPBACK_EXCHANGE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-fp32 --shard-gar > $O/bench_loopback_shard.json.log 2>&1 &&
GARFIELD_COLL_WORLD1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_coll1 -o run -- python3 bench.py --steps 5 --warmup 3 --no-fp32 --shard-gar > $O/prof_coll1.log 2>&1
