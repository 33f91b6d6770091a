set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_fp32.log 2>&1
rc1=$?
tail -2 gpurun_out/r4/pytest_fp32.log
[ $rc1 -eq 0 ] || exit $rc1
timeout -k 10 300 python -u scripts/bench_conv_f32.py > gpurun_out/r4/bench_conv_f32.log 2>&1 || exit 1
cut -c1-300 gpurun_out/r4/bench_conv_f32.log
bash scripts/gpu_prof.sh fp32_r50 --precision fp32 | head -14
