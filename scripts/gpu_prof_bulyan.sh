#!/bin/bash
# Per-kernel times of the Bulyan GAR at the ResNet-50 size (n = 8 .. 64).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-b}
for N in ${NS:-8 16 32 64}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bul_${TAG}_$N -o p -- \
    python3 -m garfield_amd.apps.gar_bench --n $N --d 23528522 --rules bulyan --iters 5 --warmup 2 \
    > $R/gpurun_out/prof_bul_${TAG}_$N.log 2>&1 || { echo "prof $N failed"; tail -5 $R/gpurun_out/prof_bul_${TAG}_$N.log; exit 1; }
  echo "== n=$N"; python3 - $R/gpurun_out/prof_bul_${TAG}_$N <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:8]:
    print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:110]}")
PY
done
