#!/bin/bash
# Round-3 closing run on one MI355X: GPU suite, the opt-in stride-2 halo test, smoke, the headline
# bench, profiled ResNet-50 / ResNet-18 configs, the remaining configs, and two knob A/Bs.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/final
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1 \
  || { echo "suite failed"; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GARFIELD_CONV3X3_S2=1 timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_grouped_gpu.py -k stride2 > $O/pytest_s2.log 2>&1 || { echo "s2 failed"; tail -5 $O/pytest_s2.log; exit 1; }
tail -1 $O/pytest_s2.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 200 python -u bench.py > $O/bench.json.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 $O/bench.json.log | cut -c1-160
CONFIGS="r50_krum_f2 r18_krum_f2" bash scripts/gpu_r3_configs.sh > $O/cfg.log 2>&1 || { echo "cfg failed"; exit 1; }
cat $O/cfg.log
[ -n "$LEAN" ] && { cp gpurun_out/cfg/rocprof_r50_krum_f2.txt gpurun_out/cfg/rocprof_r18_krum_f2.txt gpurun_out/cfg/*.json.log $O/; echo done; exit 0; }
NOPROF=1 CONFIGS="r50_bulyan_f3_k16 r50_trimmed_f2 r50_median_f1 r50_byzps_trimmed" bash scripts/gpu_r3_configs.sh > $O/cfg2.log 2>&1 \
  || { echo "cfg2 failed"; exit 1; }
cat $O/cfg2.log
for f in r50_krum_f2 r18_krum_f2 r50_bulyan_f3_k16 r50_trimmed_f2 r50_median_f1 r50_byzps_trimmed; do
  cp gpurun_out/cfg/$f.json.log $O/ 2>/dev/null
done
cp gpurun_out/cfg/rocprof_r50_krum_f2.txt gpurun_out/cfg/rocprof_r18_krum_f2.txt gpurun_out/cfg/*.json.log $O/
[ -n "$LEAN" ] && { echo done; exit 0; }
GARFIELD_WGRAD3X3_MINTILES=4 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/ab_r50_mintiles4.json.log 2>&1 && \
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/ab_r50_mintiles1.json.log 2>&1 && \
  GARFIELD_CONV3X3_RES=0 timeout -k 10 300 python -u bench.py --model resnet18 --steps 10 --warmup 3 > $O/ab_r18_res0.json.log 2>&1 && \
  timeout -k 10 300 python -u bench.py --model resnet18 --steps 10 --warmup 3 > $O/ab_r18_res1.json.log 2>&1
for f in $O/ab_*.json.log; do echo "$(basename $f): $(tail -1 $f | cut -c1-120)"; done
echo done
