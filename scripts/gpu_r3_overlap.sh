#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r3o
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$(pwd)
GARFIELD_LOOPBACK_EXCHANGE=0 timeout -k 10 300 python scripts/overlap_timing.py --steps 3 --plain > gpurun_out/r3o/plain.log 2>&1 \
    || { echo "plain failed"; tail -20 gpurun_out/r3o/plain.log; exit 1; }
grep '^{' gpurun_out/r3o/plain.log
GARFIELD_LOOPBACK_EXCHANGE=0 GARFIELD_OVERLAP=0 timeout -k 10 300 python scripts/overlap_timing.py --steps 3 > gpurun_out/r3o/noloop.log 2>&1 \
    || { echo "noloop failed"; tail -20 gpurun_out/r3o/noloop.log; exit 1; }
grep '^{' gpurun_out/r3o/noloop.log
for v in 1 0; do
  GARFIELD_OVERLAP=$v timeout -k 10 300 python scripts/overlap_timing.py --steps 3 > gpurun_out/r3o/ov$v.log 2>&1 \
      || { echo "overlap $v failed"; tail -20 gpurun_out/r3o/ov$v.log; exit 1; }
  grep '^{' gpurun_out/r3o/ov$v.log
done
