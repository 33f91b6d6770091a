#!/bin/bash
# Round-2 (third session) GPU call: GPU suite + smoke + bench on the restored tree, the
# step's kernel-time profile, and per-kernel HBM bytes / MFMA ops (rocprofv3 --pmc, one
# counter group per run) for the roofline table (scripts/roofline.py).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
TAG=${TAG:-r2c}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" gpurun_out/pt_$TAG.log | head -20; tail -5 gpurun_out/pt_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-220
[ -n "$SKIP_PROF" ] && exit 0
export GARFIELD_TRACE_MARK=1
PSTEPS=5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o bench -- python3 $R/bench.py --steps $PSTEPS --warmup 3 ${BENCH_ARGS} > $R/gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof bench failed"; tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
python3 $R/scripts/trace_summary.py $R/gpurun_out/prof_$TAG/bench_kernel_trace.csv --steps $PSTEPS --top 60 \
  --sequence $R/gpurun_out/prof_${TAG}_sequence.txt --json $R/gpurun_out/prof_${TAG}_times.json > $R/gpurun_out/prof_${TAG}_summary.txt
head -2 $R/gpurun_out/prof_${TAG}_summary.txt
rm -f $R/gpurun_out/prof_$TAG/bench_kernel_trace.csv
[ -n "$SKIP_PMC" ] && exit 0
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
MSTEPS=2
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o p -- python3 $R/bench.py --steps $MSTEPS --warmup 2 ${BENCH_ARGS} > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$i/p_counter_collection.csv --steps $MSTEPS --json $R/gpurun_out/pmc_${TAG}_$i.json > $R/gpurun_out/pmc_${TAG}_${i}_summary.txt || { echo "pmc summary $i failed"; ls -R $R/gpurun_out/pmc_${TAG}_$i | head; exit 1; }
  head -1 $R/gpurun_out/pmc_${TAG}_${i}_summary.txt
  rm -f $R/gpurun_out/pmc_${TAG}_$i/p_counter_collection.csv
done
echo done
