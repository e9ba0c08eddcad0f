#!/bin/bash
# K8 occupancy-held register budgets (fwd 3 waves/SIMD, dK/dV 2): attention tests, per-kernel A/B, GPT-2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_k.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_k.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_k.log
timeout -k 10 300 python -u bench/attention.py --native madnn_attn_tune:1:1:0 --json gpurun_out/attn_ab_occ.json \
    > gpurun_out/attn_ab_occ.log 2>&1 || { tail -n 30 gpurun_out/attn_ab_occ.log; exit 4; }
grep shape gpurun_out/attn_ab_occ.log | cut -c1-400
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch native --native madnn_attn_tune:1:1:0 --windows 6 --steps 6 \
    > gpurun_out/ab_attn_occ.log 2>&1 || { tail -n 30 gpurun_out/ab_attn_occ.log; exit 5; }
tail -n 1 gpurun_out/ab_attn_occ.log | cut -c1-400
