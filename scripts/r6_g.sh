#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd); O=$R/gpurun_out/r6g; mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 300 python scripts/diag_host.py > $O/host_plain.txt 2>&1 &&
GARFIELD_COLL_WORLD1=1 timeout -k 10 300 python scripts/diag_host.py --shard-gar > $O/host_coll1.txt 2>&1 &&
GARFIELD_LOOPBACK_EXCHANGE=1 timeout -k 10 300 python scripts/diag_host.py --shard-gar > $O/host_loopback.txt 2>&1
