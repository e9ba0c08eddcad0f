#!/bin/bash
# Norm-backward column sums as Linear bias grads + compact downsample: kernel tests, GPT-2 A/B, ResNet A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_q.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_q.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_q.log
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch colsum --windows 6 --steps 6 \
    > gpurun_out/ab_colsum.log 2>&1 || { tail -n 30 gpurun_out/ab_colsum.log; exit 4; }
tail -n 1 gpurun_out/ab_colsum.log | cut -c1-300
for b in 2048 512; do
  timeout -k 10 600 python bench/resnet_flag_ab.py --flag madnn.models.resnet:_DS_SUB --on true --off false --batch $b \
     --windows 6 --steps 4 --json-out gpurun_out/ab_ds_sub_b$b.json > gpurun_out/ab_ds_sub_b$b.log 2>&1 \
     || { tail -n 30 gpurun_out/ab_ds_sub_b$b.log; exit 5; }
  tail -n 1 gpurun_out/ab_ds_sub_b$b.log | cut -c1-260
done
