#!/bin/bash
# GPT-2 medium DP1 at 64 sequences: weight gradients per-shape (hipBLASLt / K12 split-K) vs hipBLASLt only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench/gpt2_ab.py --batch 64 --windows 6 --steps 4 --switch wgrad \
    > gpurun_out/ab_wgrad.log 2>&1 || { tail -n 40 gpurun_out/ab_wgrad.log; exit 4; }
tail -n 1 gpurun_out/ab_wgrad.log
