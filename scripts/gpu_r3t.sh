#!/bin/bash
# Full GPU test suite + qkv-bias colsum A/B on GPT-2 medium.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_t.log 2>&1; rc=$?
tail -n 3 gpurun_out/gpu_tests_t.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch attn_colsum --windows 6 --steps 6 \
    > gpurun_out/ab_attn_colsum.log 2>&1 || { tail -n 30 gpurun_out/ab_attn_colsum.log; exit 4; }
tail -n 1 gpurun_out/ab_attn_colsum.log | cut -c1-300
