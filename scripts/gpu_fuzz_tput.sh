#!/bin/bash
# Hypothesis shape fuzzing of the kernels, then the transformer-config throughput refresh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/fuzz_gpu.log 2>&1; rc=$?; tail -n 30 gpurun_out/fuzz_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_tput_r2.sh
