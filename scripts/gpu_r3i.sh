#!/bin/bash
# K12 fused GELU forward: kernel tests + GPT-2 A/B (K12 GELU epilogue vs hipBLASLt + K11 GELU); planner accuracy case.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_i.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_i.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_i.log
timeout -k 10 300 python -u bench/plan_accuracy.py --cases gpt2-medium:16,resnet50:512,gpt2-medium:16 > gpurun_out/plan_acc_i.log 2>&1 \
    || { tail -n 30 gpurun_out/plan_acc_i.log; exit 4; }
grep '"model"' gpurun_out/plan_acc_i.log | cut -c1-400
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch gelu_fwd --windows 6 --steps 6 \
    > gpurun_out/ab_gelu_fwd.log 2>&1 || { tail -n 30 gpurun_out/ab_gelu_fwd.log; exit 5; }
tail -n 1 gpurun_out/ab_gelu_fwd.log | cut -c1-400
