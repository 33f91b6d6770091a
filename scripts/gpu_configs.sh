#!/bin/bash
# BASELINE.md configs on one MI355X, each with the GAR overhead vs `average`.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup ${WARM:-3} --overhead "$@" > gpurun_out/cfg_$name.json.log 2>&1 \
    || { echo "$name failed"; tail -20 gpurun_out/cfg_$name.json.log; exit 1; }
  echo "$name: $(tail -1 gpurun_out/cfg_$name.json.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms; avg", d.get("avg_ms_per_step"), "ms; overhead", d.get("gar_overhead_pct_vs_average"), "%")')"
}
run r50_krum_f2 --gar krum --f 2
run r18_krum_f2 --model resnet18 --gar krum --f 2
run r50_bulyan_f3_k16 --gar bulyan --f 3 --workers-per-gpu 16
run r50_trimmed_f2 --gar trimmed-mean --f 2
run r50_median_f1 --gar median --f 1
run r50_imagenet_median_f1 --dataset imagenet --batch 32 --gar median --f 1
