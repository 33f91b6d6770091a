set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py tests/test_engine_gpu.py -v -s --timeout 300 --timeout-method thread -k "fp32_grouped_rows or layerwise_bulyan" > gpurun_out/r4/pytest_fp32_rows.log 2>&1
rc1=$?
grep -E "PASS|FAIL|Error|assert|^resnet|fraction" gpurun_out/r4/pytest_fp32_rows.log | tail -30
[ $rc1 -le 1 ] || exit $rc1
bash scripts/gpu_prof.sh fp32_r50 --precision fp32
rc2=$?
exit $((rc1 + rc2))
