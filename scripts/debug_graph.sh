#!/bin/bash
set -o pipefail
run() { echo "== $1 | $2" >> gpurun_out/debug_graph4.log; env $1 timeout -k 10 300 python scripts/debug_graph.py $2 2>&1 | grep "graph=True" | cut -c1-40,150-300 >> gpurun_out/debug_graph4.log || exit 1; }
run "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0" "vgg11_cifar 64 bf16"
run "MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0" "vgg11_cifar 64 bf16"
run "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0" "vgg11_cifar 64 bf16"
run "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0" "resnet50 250 bf16"
