set -o pipefail
mkdir -p gpurun_out/r4
export PYTHONPATH=.
bash scripts/gpu_prof.sh imagenet --dataset imagenet --gar krum --f 2 --no-fp32 | head -3
grep -E "iwgrad|split_reduce" gpurun_out/prof/imagenet.txt
