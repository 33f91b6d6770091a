#!/bin/bash
# round 6: PMC counters of the ImageNet-size stem kernels (one counter pass per run)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r6r; mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $O/p1 -o run -- python3 $R/scripts/stem_probe.py > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d $O/p2 -o run -- python3 $R/scripts/stem_probe.py > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/scripts/stem_probe.py > $O/t.log 2>&1
cd $R; for d in p1 p2 t; do find $O/$d -name "*.csv" -exec cp {} $O/ \; ; done; true
