set -o pipefail
mkdir -p gpurun_out/r4
PYTHONPATH=. timeout -k 10 300 python -u scripts/diag_fp32_rows.py resnet18 2>&1 | tee gpurun_out/r4/diag_fp32_r18.log
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_fp32.log 2>&1
grep -E "PASS|FAIL|Error|assert" gpurun_out/r4/pytest_fp32.log | tail -40
