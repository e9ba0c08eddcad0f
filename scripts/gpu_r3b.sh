#!/bin/bash
# Round 3: changed GPU tests (TP bf16 path, K5 absent peer, engine/planner), then planner accuracy.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_oneshot_gpu.py tests/test_engine_gpu.py -x -v \
    --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_b.log 2>&1 || { tail -n 60 gpurun_out/gpu_tests_b.log; exit 3; }
tail -n 3 gpurun_out/gpu_tests_b.log
timeout -k 10 600 python -u bench/plan_accuracy.py --json-out gpurun_out/plan_acc.json > gpurun_out/plan_acc.log 2>&1 \
    || { tail -n 40 gpurun_out/plan_acc.log; exit 4; }
grep '^{' gpurun_out/plan_acc.log
