#!/bin/bash
# A/B bench over whole environment settings: CONFIGS is a ';'-separated list of
# space-separated VAR=value assignments ("" = defaults); RUNS rounds, alternating.
# usage: CONFIGS="A=0;A=1 B=4" TAG=x bash scripts/gpu_ab_env.sh
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
TAG=${TAG:-abenv}
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in $(seq ${RUNS:-3}); do
  for c in "${!CFG[@]}"; do
    env ${CFG[$c]} timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_${TAG}_${c}_$i.log 2>&1 || { echo "bench [${CFG[$c]}] failed"; tail -5 gpurun_out/bench_${TAG}_${c}_$i.log; exit 1; }
    echo "[${CFG[$c]}] run $i: $(grep '^{' gpurun_out/bench_${TAG}_${c}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("final_loss"))')"
  done
done
