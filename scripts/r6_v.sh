#!/bin/bash
# round 6: stem forward on the channel-padded staging: stem tests, ImageNet step + table, headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6v; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grouped_gpu.py tests/test_fp32_gpu.py -k "stem" > $O/pytest_stem.log 2>&1 &&
timeout -k 10 400 python bench.py --dataset imagenet --steps 10 --warmup 3 --no-fp32 > $O/imagenet.json.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/headline.json.log 2>&1 &&
bash scripts/gpu_prof.sh imagenet --dataset imagenet --no-fp32 > /dev/null && cp gpurun_out/prof/imagenet.txt $O/imagenet_table.txt
cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python3 $R/scripts/stem_probe.py > $O/p1.log 2>&1
