#!/bin/bash
# round 6: multi-rank rehearsal of the default sharded GPU step on ONE MI355X: 2 and 4 ranks sharing the
# device over gloo (RCCL refuses two ranks per device). Exercises the comm stream, the device-side
# hand-offs, the staged three-graph forward, the packed all-to-all with the own shard kept in place, the
# kernel-choice agreement and the replica checksums -- everything of the 8-GPU run except RCCL itself.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6mr; mkdir -p $O
export PYTHONPATH=$R OMP_NUM_THREADS=2 GARFIELD_SHARE_GPU=1 GARFIELD_DIST_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2977$n \
    bench.py --gpus $n --steps 4 --warmup 3 --no-fp32 --batch 64 > $O/sharded_gloo_$n.json.log 2>&1 || { tail -30 $O/sharded_gloo_$n.json.log; exit 1; }
  grep '^{' $O/sharded_gloo_$n.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['ms_per_step'], d['config']['hip_graphs'], d.get('replicas_identical'), d.get('replica_checksums'), d['final_loss'])"
done
