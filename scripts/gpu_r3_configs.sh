#!/bin/bash
# Every BASELINE config on one MI355X: bench (with the GAR overhead vs average) and a rocprofv3
# kernel table of the steady-state step. CONFIGS selects a subset (space-separated names).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/cfg
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
run() {  # name, args...
  local name=$1; shift
  if [ -n "$CONFIGS" ] && [[ " $CONFIGS " != *" $name "* ]]; then return 0; fi
  timeout -k 10 500 python bench.py --steps ${STEPS:-10} --warmup ${WARM:-3} --overhead "$@" > $O/$name.json.log 2>&1 \
    || { echo "$name failed"; tail -20 $O/$name.json.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.json.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms; avg", d.get("avg_ms_per_step"), "ms; overhead", d.get("gar_overhead_pct_vs_average"), "%")')"
  if [ -z "$NOPROF" ]; then
    (cd /tmp && TMPDIR=/tmp GARFIELD_TRACE_MARK=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$name -o run \
        -- python3 $R/bench.py --steps 3 --warmup 2 "$@" > $O/prof_$name.log 2>&1) \
        || { echo "rocprof $name failed"; tail -5 $O/prof_$name.log; exit 1; }
    python3 $R/scripts/trace_summary.py $O/prof_$name/run_kernel_trace.csv --steps 3 --top 40 > $O/rocprof_$name.txt
    head -1 $O/rocprof_$name.txt
    rm -rf $O/prof_$name
  fi
}
run r50_krum_f2 --gar krum --f 2
run r18_krum_f2 --model resnet18 --gar krum --f 2
run r50_bulyan_f3_k16 --gar bulyan --f 3 --workers-per-gpu 16
run r50_trimmed_f2 --gar trimmed-mean --f 2
run r50_median_f1 --gar median --f 1
run r50_imagenet_median_f1 --dataset imagenet --batch ${IMNET_BATCH:-250} --gar median --f 1
run r50_byzps_trimmed --gar trimmed-mean --f 1 --num-ps 1 --ps-workers --mar median
echo done
