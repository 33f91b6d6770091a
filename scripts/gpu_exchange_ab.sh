#!/bin/bash
# Fixed cost of the sharded exchange at world 1: the plain step, the
# sharded step, the sharded step with the loopback exchange machinery (comm stream, bucket
# signals, per-bucket events; the own shard is read in place) after the backward and inside
# it, with the next forward staged at the bucket boundaries or as one graph, alternating
# over RUNS rounds; then overlap_timing.py's per-bucket times (steps back to back).
# usage: bash scripts/gpu_exchange_ab.sh   (results under gpurun_out/xab/)
set -o pipefail
mkdir -p gpurun_out/xab
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
names=(plain shard loop_ov0 loop_ov1 loop_ov1_onegraph)
envs=("" "" "GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=0" "GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=1"
      "GARFIELD_LOOPBACK_EXCHANGE=1 GARFIELD_OVERLAP=1 GARFIELD_STAGE_FORWARD=0")
args=("" "--shard-gar" "--shard-gar" "--shard-gar" "--shard-gar")
for i in $(seq ${RUNS:-2}); do
  for c in 0 1 2 3 4; do
    log=gpurun_out/xab/bench_${names[$c]}_$i.log
    env ${envs[$c]} timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-fp32 ${args[$c]} > $log 2>&1 \
      || { echo "bench ${names[$c]} failed"; tail -5 $log; exit 1; }
    echo "${names[$c]} run $i: $(grep '^{' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
if [ -z "$NO_TIMING" ]; then
  timeout -k 10 300 python scripts/overlap_timing.py --plain > gpurun_out/xab/timing_plain.log 2>&1 || { echo timing plain failed; tail -5 gpurun_out/xab/timing_plain.log; exit 1; }
  GARFIELD_OVERLAP=1 GARFIELD_STAGE_FORWARD=0 timeout -k 10 300 python scripts/overlap_timing.py > gpurun_out/xab/timing_ov1_onegraph.log 2>&1 || { echo timing onegraph failed; exit 1; }
  for ov in 0 1; do
    GARFIELD_OVERLAP=$ov timeout -k 10 300 python scripts/overlap_timing.py > gpurun_out/xab/timing_ov$ov.log 2>&1 || { echo timing ov$ov failed; tail -5 gpurun_out/xab/timing_ov$ov.log; exit 1; }
  done
  for f in gpurun_out/xab/timing_*.log; do echo "$f: $(grep '^{' $f)"; done
fi
