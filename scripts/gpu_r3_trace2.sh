#!/bin/bash
# hipGraphLaunch host time: plain step vs bucketed step without / with in-graph event nodes.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r3t2
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R GARFIELD_TRACE_MARK=1
cd /tmp && export TMPDIR=/tmp
for v in plain noov ov; do
  args=""; envs="GARFIELD_OVERLAP=0"
  [ $v != plain ] && args="--shard-gar"
  [ $v == ov ] && envs="GARFIELD_OVERLAP=1 GARFIELD_LOOPBACK_EXCHANGE=1"
  env $envs timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d $R/gpurun_out/r3t2/$v -o run -- \
      python3 $R/bench.py --steps 3 --warmup 3 $args > $R/gpurun_out/r3t2/$v.log 2>&1 || { echo "rocprof $v failed"; tail -20 $R/gpurun_out/r3t2/$v.log; exit 1; }
  python3 - $R/gpurun_out/r3t2/$v/run_hip_api_trace.csv $v <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Function"] == "hipGraphLaunch"]
print(sys.argv[2], "hipGraphLaunch us:", [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, 1) for r in rows][-6:])
PY
  rm -f $R/gpurun_out/r3t2/$v/run_hip_api_trace.csv
done
