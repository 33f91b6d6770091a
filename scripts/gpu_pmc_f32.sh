#!/bin/bash
# PMC passes (one counter group per run) over scripts/prof_conv_f32_one.py: where the fp32
# (split-bf16) convolution kernels spend their cycles.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/pmcf32
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/scripts/prof_conv_f32_one.py \
      > $O/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, sys
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "garfield" not in r["Kernel_Name"]:
            continue
        rows[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in rows.items():
    print(k)
    print("   " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(d.items())))
PY
