#!/bin/bash
# K12 split-K weight gradient: correctness tests, then the A/B against hipBLASLt on GPT-2 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_d.log 2>&1 || { tail -n 60 gpurun_out/gpu_tests_d.log; exit 3; }
tail -n 3 gpurun_out/gpu_tests_d.log
timeout -k 10 300 python -u bench/wgrad_ab.py --json gpurun_out/wgrad_ab.json > gpurun_out/wgrad_ab.log 2>&1 \
    || { tail -n 40 gpurun_out/wgrad_ab.log; exit 4; }
cat gpurun_out/wgrad_ab.log
