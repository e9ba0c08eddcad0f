#!/bin/bash
# K12 on the 16x16x32 MFMA shape: correctness (both shapes), GEMM and wgrad A/Bs, then the ResNet 1x1 wgrad A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_g.log 2>&1 || { tail -n 60 gpurun_out/gpu_tests_g.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_g.log
timeout -k 10 300 python -u bench/gemm_ab.py --rounds 5 --json gpurun_out/gemm_ab_m16.json > gpurun_out/gemm_ab_m16.log 2>&1 \
    || { tail -n 30 gpurun_out/gemm_ab_m16.log; exit 4; }
cat gpurun_out/gemm_ab_m16.log | grep '^{'
timeout -k 10 300 python -u bench/wgrad_ab.py --json gpurun_out/wgrad_ab_m16.json > gpurun_out/wgrad_ab_m16.log 2>&1 \
    || { tail -n 30 gpurun_out/wgrad_ab_m16.log; exit 5; }
grep '^{' gpurun_out/wgrad_ab_m16.log | cut -c1-330
