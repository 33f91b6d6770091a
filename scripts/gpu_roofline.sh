#!/bin/bash
# Kernel table + PMC roofline of one bench.py configuration:
#   bash scripts/gpu_roofline.sh <name> [bench.py args...]
#   -> gpurun_out/roof/<name>/: rocprof table + sequence (gpu_seq.sh), pmc_{1,2,3}_summary.txt, roofline.md
# Passes: FETCH_SIZE | WRITE_SIZE | MFMA ops + busy cycles, each its own run (counter limits per pass).
set -o pipefail
NAME=$1; shift
R=$(pwd); O=$R/gpurun_out/roof/$NAME; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
bash scripts/gpu_seq.sh $NAME "$@" > /dev/null || exit 1
cp gpurun_out/seq/$NAME.txt gpurun_out/seq/${NAME}_seq.txt gpurun_out/seq/$NAME.json $O/ || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES"; do
  i=$((i+1))
  GARFIELD_TRACE_MARK=1 timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o p -- python3 $R/bench.py --steps 2 --warmup 2 "$@" > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
  python3 $R/scripts/pmc_summary.py $O/pmc_$i/p_counter_collection.csv --steps 2 --json $O/pmc_$i.json > $O/pmc_${i}_summary.txt || exit 1
  rm -rf $O/pmc_$i
done
cd $R
python3 scripts/roofline.py $O/$NAME.json $O/pmc_1.json $O/pmc_2.json $O/pmc_3.json --md $O/roofline.md > $O/roofline.txt || exit 1
head -12 $O/roofline.txt
