#!/bin/bash
# PMC counters of the Bulyan tail kernels (n = 32 and 64), one counter pass per run.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-t}
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${TAG}_$i -o p -- \
    python3 -m garfield_amd.apps.gar_bench --n ${NS:-32 64} --d 23528522 --rules bulyan --iters 2 --warmup 1 \
    > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $R/gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
python3 - $R/gpurun_out/pmc_${TAG} <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(sys.argv[1] + '_*/**/*counter_collection.csv', recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0][-60:]
        if 'tail' not in k and 'gram' not in k and 'select' not in k:
            continue
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
