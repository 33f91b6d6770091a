#!/bin/bash
# Round-5 closing numbers for the non-headline configurations (20-30 timed steps each):
# ResNet-18, Bulyan f=3 x 16 flat / layer-wise, Krum with a reverse + lie worker vs honest, ImageNet shape.
set -o pipefail
O=gpurun_out/configs; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
run() {   # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --no-fp32 "$@" > $O/$n.json.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.json.log; exit 1; }
  echo "$n: $(grep '^{' $O/$n.json.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
}
for i in 1 2; do
  run r18_$i --model resnet18 --steps 20 --warmup 5 || exit 1
  run honest_$i --steps 30 --warmup 5 || exit 1
  run attack_$i --steps 30 --warmup 5 --attack reverse,lie || exit 1
  run bulyan_$i --gar bulyan --f 3 --workers-per-gpu 16 --steps 20 --warmup 5 || exit 1
  run bulyan_lw_$i --gar bulyan --f 3 --workers-per-gpu 16 --layerwise --steps 20 --warmup 5 || exit 1
done
run imagenet_1 --dataset imagenet --steps 4 --warmup 2 || exit 1
