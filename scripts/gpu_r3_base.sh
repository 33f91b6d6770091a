#!/bin/bash
# Round-3 checkpoint on one MI355X: GPU test suite, smoke, bench (20 steps), and a
# rocprofv3 kernel-stats profile of the bench step. Every GPU step has its own limit.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${TAG:-base}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 10 --timeout 200 --timeout-method thread \
      > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
      || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > $O/bench.json.log 2>&1 \
    || { echo "bench failed"; tail -30 $O/bench.json.log; exit 1; }
tail -1 $O/bench.json.log
if [ -z "$SKIP_PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  GARFIELD_TRACE_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
      -- python3 $R/bench.py --steps 5 --warmup 3 ${BENCH_ARGS} > $O/prof.log 2>&1 \
      || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
  python3 $R/scripts/trace_summary.py $O/prof/run_kernel_trace.csv --steps 5 --top 60 \
      --sequence $O/prof_sequence.txt > $O/prof_summary.txt
  head -3 $O/prof_summary.txt
  rm -f $O/prof/run_kernel_trace.csv
fi
echo done
