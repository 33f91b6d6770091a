set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_fp32.log 2>&1
rc1=$?
tail -2 gpurun_out/r4/pytest_fp32.log
[ $rc1 -eq 0 ] || exit $rc1
bash scripts/gpu_prof.sh fp32_r50 --precision fp32 | head -30
