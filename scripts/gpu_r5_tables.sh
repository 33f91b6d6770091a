#!/bin/bash
# Round-5 kernel tables (scripts/gpu_seq.sh per configuration -> gpurun_out/seq/) and the one-rank
# real-RCCL record of the sharded step (gpurun_out/exchange/).
#   WHICH="in r18 lwb bul rccl" bash scripts/gpu_r5_tables.sh
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
WHICH=${WHICH:-"in r18 lwb bul rccl"}
for w in $WHICH; do
  case $w in
    in)  bash scripts/gpu_seq.sh r5_imagenet_krum_f2 --dataset imagenet --no-fp32 || exit 1 ;;
    r18) bash scripts/gpu_seq.sh r5_r18_krum_f2 --model resnet18 --no-fp32 || exit 1 ;;
    lwb) bash scripts/gpu_seq.sh r5_r50_bulyan_f3_w16_lw --gar bulyan --f 3 --workers-per-gpu 16 --layerwise --no-fp32 || exit 1 ;;
    bul) bash scripts/gpu_seq.sh r5_r50_bulyan_f3_w16 --gar bulyan --f 3 --workers-per-gpu 16 --no-fp32 || exit 1 ;;
    atk) bash scripts/gpu_seq.sh r5_r50_krum_f2_lie --attack reverse,lie --no-fp32 || exit 1 ;;
    rccl)
      O=gpurun_out/exchange; mkdir -p $O
      for i in 1 2; do
        timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-fp32 --shard-gar > $O/bench_shard_$i.log 2>&1 || { tail -5 $O/bench_shard_$i.log; exit 1; }
        GARFIELD_DIRECT_RCCL=1 GARFIELD_DIRECT_RCCL_WORLD1=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-fp32 --shard-gar \
          > $O/bench_rccl1_$i.log 2>&1 || { tail -5 $O/bench_rccl1_$i.log; exit 1; }
        for c in shard rccl1; do echo "$c run $i: $(grep '^{' $O/bench_${c}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
      done
      GARFIELD_DIRECT_RCCL=1 GARFIELD_DIRECT_RCCL_WORLD1=1 bash scripts/gpu_seq.sh r5_r50_shard_rccl1 --shard-gar --no-fp32 || exit 1
      ;;
  esac
done
