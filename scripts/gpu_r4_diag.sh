set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -v -s --timeout 300 --timeout-method thread -k "reference_precision or stem_f32" > gpurun_out/r4/pytest_fp32_rows.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|assert|^resnet" gpurun_out/r4/pytest_fp32_rows.log | tail -30
exit $rc
