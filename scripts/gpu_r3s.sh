#!/bin/bash
# dQKV column sums in the K8 backward as the qkv bias grad: attention + kernel tests, GPT-2 A/B, GPT-2 bench half.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_s.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_s.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_s.log
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch attn_colsum --windows 6 --steps 6 \
    > gpurun_out/ab_attn_colsum.log 2>&1 || { tail -n 30 gpurun_out/ab_attn_colsum.log; exit 4; }
tail -n 1 gpurun_out/ab_attn_colsum.log | cut -c1-300
