# round 4: the fp32 kernels' GPU tests, then the fp32 and bf16 benches (short)
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_fp32_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/pytest_fp32.log 2>&1
rc=$?
tail -15 gpurun_out/r4/pytest_fp32.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --precision fp32 --steps 10 --warmup 3 > gpurun_out/r4/bench_fp32.json.log 2>&1 || { tail -30 gpurun_out/r4/bench_fp32.json.log; exit 1; }
tail -2 gpurun_out/r4/bench_fp32.json.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_bf16.json.log 2>&1 || { tail -30 gpurun_out/r4/bench_bf16.json.log; exit 1; }
tail -2 gpurun_out/r4/bench_bf16.json.log
