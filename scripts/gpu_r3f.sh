#!/bin/bash
# ResNet-50: 1x1-conv weight gradients per shape (MIOpen / K12 split-K) vs MIOpen only, at 2048 and 512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_f.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_f.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_f.log
for b in 2048 512; do
  timeout -k 10 500 python -u bench/resnet_flag_ab.py --flag madnn.ops:WGRAD --on auto --off lt --batch $b \
      --windows 6 --steps 4 --json-out gpurun_out/ab_resnet_wgrad_b$b.json > gpurun_out/ab_resnet_wgrad_b$b.log 2>&1 \
      || { tail -n 30 gpurun_out/ab_resnet_wgrad_b$b.log; exit 4; }
  tail -n 1 gpurun_out/ab_resnet_wgrad_b$b.log | cut -c1-400
done
