#!/bin/bash
# Norm-backward early loads: kernel tests + GPT-2 A/B; then K12 PMC passes (fwd / dgrad / wgrad).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_g2.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_g2.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_g2.log
timeout -k 10 400 python -u bench/gpt2_ab.py --switch native --native madnn_norm_tune:2:1:0 --windows 6 --steps 8 \
    > gpurun_out/ab_norm_early.log 2>&1 || { tail -n 30 gpurun_out/ab_norm_early.log; exit 4; }
tail -n 1 gpurun_out/ab_norm_early.log | cut -c1-300
bash scripts/gpu_k12_pmc.sh
