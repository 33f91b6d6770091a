#!/bin/bash
# GPU timings of the asynchronous engines on one MI355X: the collective
# LEARN engine (decentralised, all-gathers) and the fastest-quorum Garfield_CC engine, 3 ranks
# sharing the GPU over gloo (several RCCL ranks cannot share one device). Per-step times are
# printed by --bench; results under gpurun_out/async/.
set -o pipefail
mkdir -p gpurun_out/async
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd) OMP_NUM_THREADS=4 GARFIELD_SHARE_GPU=1
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29651 \
  -m garfield_amd.apps.learn --num_nodes 3 --f 0 --gar median --collective 1 --backend gloo --device cuda \
  --model mlp --dataset mnist --num_iter 30 --acc_freq 29 --bench True > gpurun_out/async/learn_collective.log 2>&1 \
  || { echo learn failed; tail -20 gpurun_out/async/learn_collective.log; exit 1; }
grep -c "Training step" gpurun_out/async/learn_collective.log; grep "Training step" gpurun_out/async/learn_collective.log | tail -3
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29652 \
  -m garfield_amd.apps.garfield_cc --backend gloo --model resnet18 --dataset cifar10 --aggregator median --fw 1 \
  --workers_per_rank 2 --batch 32 --num_iter 30 --quorum 2 --bench True > gpurun_out/async/cc_quorum.log 2>&1 \
  || { echo quorum failed; tail -20 gpurun_out/async/cc_quorum.log; exit 1; }
tail -5 gpurun_out/async/cc_quorum.log
