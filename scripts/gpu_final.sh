#!/bin/bash
# K13 epilogue check + its kernel A/B, then the full round-end rehearsal (tests, smoke, bench, profile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_conv3x3_gpu.py \
   > "$OUT/conv_tests.log" 2>&1 || { tail -30 "$OUT/conv_tests.log"; exit 3; }
tail -n 1 "$OUT/conv_tests.log"
PROF_ENV=MADNN_BN_DGRAD_EPI bash scripts/gpu_prof_ab.sh > /dev/null || exit 6
bash scripts/gpu_check.sh
