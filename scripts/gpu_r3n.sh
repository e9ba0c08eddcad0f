#!/bin/bash
# K12 split cap 256 + per-shape timed 3x3 wgrad: per-shape candidates, GEMM/conv tests, ResNet-50 A/B of the 3x3 routing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/resnet_wgrad_shapes.py --batch 2048 --json gpurun_out/wgrad_shapes_b2048_n.json \
    > gpurun_out/wgrad_shapes_n.log 2>&1 || { tail -n 30 gpurun_out/wgrad_shapes_n.log; exit 3; }
grep -v Warn gpurun_out/wgrad_shapes_n.log | cut -c1-260
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_n.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_n.log; exit 4; }
tail -n 1 gpurun_out/gpu_tests_n.log
timeout -k 10 600 python bench/resnet_flag_ab.py --flag madnn.ops:_K13_WGRAD --on auto --off wide --batch 2048 --windows 6 --steps 4 \
   --json-out gpurun_out/ab_k13_wgrad_auto.json > gpurun_out/ab_k13_wgrad_auto.log 2>&1 || { tail -n 30 gpurun_out/ab_k13_wgrad_auto.log; exit 5; }
tail -n 1 gpurun_out/ab_k13_wgrad_auto.log | cut -c1-300
