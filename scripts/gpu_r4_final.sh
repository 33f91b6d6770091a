#!/bin/bash
# Closing GPU session of round 4: the GPU suite, smoke, the driver's bench, every BASELINE
# configuration (+ the round-4 configurations), steady-state kernel tables and the roofline PMC
# passes of the bf16 headline step. Everything lands in gpurun_out/final/ (copied to profiles/r4/).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p $O/configs
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
STAGE=${STAGE:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = suite ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
timeout -k 10 400 python -u bench.py > $O/bench_default.json.log 2>&1 || { tail -5 $O/bench_default.json.log; exit 1; }
tail -1 $O/bench_default.json.log | cut -c1-160
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-fp32 > $O/bench_bf16_20.json.log 2>&1 || exit 1
tail -1 $O/bench_bf16_20.json.log | cut -c1-160
run_cfg() {   # name, bench args
  timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-fp32 --overhead "${@:2}" > $O/configs/$1.json.log 2>&1 \
    || { tail -5 $O/configs/$1.json.log; return 1; }
  tail -1 $O/configs/$1.json.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['ms_per_step'], d['value'], d.get('gar_overhead_pct_vs_average'))"
}
run_cfg r50_krum_f2 --gar krum --f 2 || exit 1
run_cfg r18_krum_f2 --model resnet18 --gar krum --f 2 || exit 1
run_cfg r50_bulyan_f3_w16 --gar bulyan --f 3 --workers-per-gpu 16 || exit 1
run_cfg r50_bulyan_f3_w16_layerwise --gar bulyan --f 3 --workers-per-gpu 16 --layerwise || exit 1
run_cfg r50_krum_f2_layerwise --gar krum --f 2 --layerwise || exit 1
run_cfg r50_trimmed_f2 --gar trimmed-mean --f 2 || exit 1
run_cfg r50_median_f1 --gar median --f 1 || exit 1
run_cfg r50_byzps_trimmed --gar trimmed-mean --f 1 --num-ps 1 --ps-workers --mar median || exit 1
run_cfg r50_krum_f2_reverse_lie --gar krum --f 2 --attack reverse,lie || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --no-fp32 --dataset imagenet --gar krum --f 2 > $O/configs/r50_imagenet_krum_f2.json.log 2>&1 || exit 1
tail -1 $O/configs/r50_imagenet_krum_f2.json.log | cut -c1-160
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --precision fp32 --ref-impl > $O/configs/r50_fp32_refimpl.json.log 2>&1 || exit 1
tail -1 $O/configs/r50_fp32_refimpl.json.log | cut -c1-160
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
bash scripts/gpu_prof.sh bf16_r50 --no-fp32 > /dev/null && cp gpurun_out/prof/bf16_r50.txt $O/rocprof_bf16_r50_krum_f2.txt || exit 1
bash scripts/gpu_prof.sh fp32_r50 --precision fp32 > /dev/null && cp gpurun_out/prof/fp32_r50.txt $O/rocprof_fp32_r50_krum_f2.txt || exit 1
bash scripts/gpu_prof.sh imagenet --dataset imagenet --gar krum --f 2 --no-fp32 > /dev/null && cp gpurun_out/prof/imagenet.txt $O/rocprof_imagenet_r50_krum_f2.txt || exit 1
cp gpurun_out/prof/bf16_r50.json $O/times_bf16_r50.json
head -3 $O/rocprof_bf16_r50_krum_f2.txt; head -3 $O/rocprof_fp32_r50_krum_f2.txt; head -3 $O/rocprof_imagenet_r50_krum_f2.txt
fi
if [ "$STAGE" = all ] || [ "$STAGE" = pmc ]; then
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES"; do
  i=$((i+1))
  GARFIELD_TRACE_MARK=1 timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o p -- python3 $R/bench.py --steps 2 --warmup 2 --no-fp32 > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $O/pmc_$i/p_counter_collection.csv --steps 2 --json $O/pmc_$i.json > $O/pmc_${i}_summary.txt || exit 1
  rm -rf $O/pmc_$i
done
cd $R
python3 scripts/roofline.py $O/times_bf16_r50.json $O/pmc_1.json $O/pmc_2.json $O/pmc_3.json --md $O/roofline_bf16_r50.md > $O/roofline_bf16_r50.txt || exit 1
head -30 $O/roofline_bf16_r50.txt
fi
echo done
