#!/bin/bash
# Alternating sweep of the weight-gradient split-K targets on the bench step.
# usage: CONFIGS="WGRAD3_WG=512;WGRAD3_WG=128" RUNS=2 bash scripts/gpu_sweep_splits.sh
set -o pipefail
mkdir -p gpurun_out/splits
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
IFS=';' read -ra CFG <<< "$CONFIGS"
for i in $(seq ${RUNS:-2}); do
  for c in "${!CFG[@]}"; do
    log=gpurun_out/splits/${TAG:-s}_${c}_$i.log
    timeout -k 10 300 python scripts/sweep_splits.py ${CFG[$c]} -- --steps 30 --warmup 5 --no-fp32 ${BENCH_ARGS} > $log 2>&1 \
      || { echo "[${CFG[$c]}] failed"; tail -5 $log; exit 1; }
    echo "[${CFG[$c]}] run $i: $(grep '^{' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
