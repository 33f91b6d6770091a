#!/bin/bash
# Launch an RPC application (aggregathor | byzsgd | learn | centralized) on the hosts
# listed in the "servers" and "workers" files (one host per line), one process per
# host over ssh. Reference: pytorch_impl/applications/Aggregathor/run_exp.sh (same
# files, same flags). Every remote PID is recorded in run_exp.pids for kill.sh.
#
# Single-node MI355X jobs do not need this script: use torchrun, e.g.
#   torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m garfield_amd.apps.garfield_cc --aggregator krum --fw 2
set -euo pipefail

APP=${APP:-aggregathor}
PS_FILE=${PS_FILE:-servers}
WORKER_FILE=${WORKER_FILE:-workers}
NUM_WRK=${NUM_WRK:-1000}          # upper bound on the number of workers used
FW=${FW:-0}
FPS=${FPS:-0}
ITER=${ITER:-100000}
DATASET=${DATASET:-cifar10}
MODEL=${MODEL:-resnet50}
OPTIMIZER=${OPTIMIZER:-sgd}
BATCH=${BATCH:-25}
LOSS=${LOSS:-cross-entropy}
LR=${LR:-0.2}
GAR=${GAR:-average}
PORT=${PORT:-29500}
SSH=${SSH:-ssh}
REMOTE_DIR=${REMOTE_DIR:-Garfield-MI355X}
PYTHON=${PYTHON:-python3}

mapfile -t PS < <(grep -v '^\s*$' "$PS_FILE")
mapfile -t WK < <(grep -v '^\s*$' "$WORKER_FILE" | head -n "$NUM_WRK")
MASTER=${PS[0]%:*}
COMMON="cd $REMOTE_DIR && $PYTHON -m garfield_amd.apps.$APP --master $MASTER --port $PORT --num_iter $ITER"
COMMON="$COMMON --dataset $DATASET --model $MODEL --batch $BATCH --loss $LOSS --optimizer $OPTIMIZER"
COMMON="$COMMON --opt_args '{\"lr\":\"$LR\",\"momentum\":\"0.9\",\"weight_decay\":\"0.0005\"}'"
COMMON="$COMMON --num_ps ${#PS[@]} --num_workers ${#WK[@]} --fw $FW --fps $FPS --gar $GAR"

: > run_exp.pids
rank=0
for host in "${PS[@]}" "${WK[@]}"; do
  cmd="$COMMON --rank $rank"
  echo "running on ${host%:*}: $cmd"
  # nohup + echo $!: the remote shell prints the PID of the trainer it started
  pid=$($SSH "${host%:*}" "nohup bash -c \"$cmd\" > garfield_rank$rank.log 2>&1 & echo \$!")
  echo "${host%:*} $pid" >> run_exp.pids
  rank=$((rank + 1))
done
echo "started $rank processes; PIDs in run_exp.pids (stop them with deploy/kill.sh)"
