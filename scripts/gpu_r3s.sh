#!/bin/bash
# downsample gradient added in conv1's K9 data-grad epilogue: conv tests, ResNet-50 A/B at 2048.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_s.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_s.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_s.log
timeout -k 10 400 python -u bench/resnet_flag_ab.py --flag madnn.ops:SUB_IN_DGRAD --batch 2048 --windows 5 --steps 5 \
    > gpurun_out/ab_sub_in_dgrad.log 2>&1 || { tail -n 30 gpurun_out/ab_sub_in_dgrad.log; exit 4; }
tail -n 1 gpurun_out/ab_sub_in_dgrad.log | cut -c1-400
