#!/bin/bash
# Iteration session: GPU tests, then bench variants given as ';'-separated arg lists in $VARIANTS.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail 10 --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py $v > gpurun_out/variant_$i.log 2>&1 || { echo "variant $i failed: $v"; tail -20 gpurun_out/variant_$i.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/variant_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms", "loss", d["final_loss"], d.get("gar_overhead_pct_vs_average",""))')"
done
