#!/bin/bash
# Round-3 exchange checks on one MI355X:
#  1. GPU tests of the engine / grouped path;
#  2. world-1 step: plain vs the bucketed sharded path with the loopback exchange,
#     with and without in-graph bucket events (GARFIELD_OVERLAP);
#  3. rocprof kernel trace of the overlapped loopback step;
#  4. 4-rank gloo rehearsal of the multi-GPU bench path on the one GPU.
set -o pipefail
mkdir -p gpurun_out/r3x
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
O=gpurun_out/r3x
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
      tests/test_grouped_gpu.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
run() {  # tag "bench args" env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 5 $args ${BENCH_ARGS} > $O/bench_$tag.log 2>&1 \
      || { echo "bench $tag failed"; tail -8 $O/bench_$tag.log; exit 1; }
  echo "$tag: $(grep '^{' $O/bench_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))')"
}
for i in 1 2; do
  run plain_$i "" GARFIELD_X=0
  run shard_loop_ov_$i --shard-gar GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=1
  run shard_loop_noov_$i --shard-gar GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=0
  run shard_noloop_$i --shard-gar GARFIELD_OVERLAP=0
done
for v in 1 0; do
  GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=$v timeout -k 10 300 python scripts/overlap_timing.py --steps 3 \
      > $O/overlap_$v.log 2>&1 || { echo "overlap $v failed"; tail -20 $O/overlap_$v.log; exit 1; }
  echo "overlap=$v $(grep '^{' $O/overlap_$v.log)"
done
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=1 GARFIELD_TRACE_MARK=1 timeout -k 10 300 \
      rocprofv3 --kernel-trace --stats -d $O/prof_ov -o run -- python3 bench.py --steps 5 --warmup 3 --shard-gar \
      > $O/prof_ov.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof_ov.log; exit 1; }
fi
if [ -z "$SKIP_GLOO" ]; then
  GARFIELD_DIST_BACKEND=gloo GARFIELD_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus 4 --steps 2 --warmup 2 \
      --batch 32 > $O/gloo4.log 2>&1 || { echo "gloo4 failed"; tail -20 $O/gloo4.log; exit 1; }
  grep '^{' $O/gloo4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("gloo4", d["n_gpus"], d["ms_per_step"], d.get("replicas_identical"), d.get("replica_checksums"))'
fi
