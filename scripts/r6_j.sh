#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j; mkdir -p $O
export PYTHONPATH=$(pwd)
timeout -k 10 300 python scripts/probe_concurrency.py > $O/concurrency.txt 2>&1
