#!/bin/bash
# round 6: the second half of the BASELINE metric on the final kernels -- GAR overhead vs average
# (bf16 and fp32), the GAR micro-benchmark with rocprof bandwidth, the reference-algorithms baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6o; mkdir -p $O
export PYTHONPATH=$R
B="timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overhead"
$B --no-fp32 > $O/krum_f2_bf16.json.log 2>&1 &&
$B --precision fp32 > $O/krum_f2_fp32.json.log 2>&1 &&
$B --no-fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_bf16.json.log 2>&1 &&
$B --precision fp32 --gar bulyan --f 3 --workers-per-gpu 16 > $O/bulyan_f3_w16_fp32.json.log 2>&1 &&
$B --no-fp32 --gar median --f 1 > $O/median_f1_bf16.json.log 2>&1 &&
$B --precision fp32 --gar median --f 1 > $O/median_f1_fp32.json.log 2>&1 &&
$B --no-fp32 --gar trimmed-mean --f 2 > $O/trimmed_f2_bf16.json.log 2>&1 &&
$B --precision fp32 --gar trimmed-mean --f 2 > $O/trimmed_f2_fp32.json.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-fp32 --ref-impl > $O/refimpl_bf16.json.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --precision fp32 --ref-impl > $O/refimpl_fp32.json.log 2>&1 &&
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 --d 11173962 23528522 --dtype bf16 \
  --rules average krum bulyan median trimmed-mean > $O/gar_bench_bf16.jsonl 2>$O/gar_bench.err &&
timeout -k 10 300 python -m garfield_amd.apps.gar_bench --n 8 16 32 --d 11173962 23528522 --dtype fp32 \
  --rules average krum bulyan median trimmed-mean > $O/gar_bench_fp32.jsonl 2>>$O/gar_bench.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gb_prof -o run -- \
  python3 -m garfield_amd.apps.gar_bench --n 8 16 32 --d 23528522 --dtype bf16 --iters 5 \
  --rules average krum bulyan median trimmed-mean > $O/gar_bench_prof.log 2>&1
cd $R; find $O/gb_prof -name "*kernel_stats.csv" -exec cp {} $O/gar_kernel_stats.csv \; ; rm -rf $O/gb_prof; true
