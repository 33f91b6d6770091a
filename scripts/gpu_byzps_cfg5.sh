#!/bin/bash
# BASELINE config 5 on one MI355X: 3 Byzantine-resilient server replicas + 5 worker ranks (8 ranks sharing
# the GPU over gloo: RCCL refuses two ranks per device), ResNet-50 CIFAR shape, 1 logical worker x 250
# per worker rank, Trimmed-Mean f_w = 1 over the 5 workers, coordinate-wise median f_ps = 1 over the
# 3 server models. Run twice: server rank 0 honest, then Byzantine (reverse: -100 x its model every
# step). Both runs print every rank's replica checksum: all equal, and equal across the two runs, means
# the Byzantine server's model was rejected. Times are gloo's on a shared GPU, not a performance figure.
set -o pipefail
O=gpurun_out/byzps; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd) OMP_NUM_THREADS=2 GARFIELD_SHARE_GPU=1 GARFIELD_DIST_BACKEND=gloo
for atk in none reverse; do
  A=""; [ "$atk" = none ] || A="--ps-attack $atk"
  timeout -k 10 600 python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 2966${#atk} \
    bench.py --gpus 8 --steps 3 --warmup 1 --no-fp32 --gar trimmed-mean --f 1 --num-ps 3 --fps 1 --mar median \
    --workers-per-gpu 1 --no-graph $A > $O/cfg5_$atk.json.log 2>&1 || { echo "cfg5 $atk failed"; tail -20 $O/cfg5_$atk.json.log; exit 1; }
  grep '^{' $O/cfg5_$atk.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$atk', d['ms_per_step'], d['config']['parallelism'], d.get('replicas_identical'), d.get('replica_checksums'))"
done
